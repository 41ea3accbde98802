#!/usr/bin/env python3
"""Timed-region anatomy of a traced 20-step headline run (tools/gpurun/r6_s20trace.sh): span, busy time and
mean kernel durations of the timed runs against the steady runs, then each timed run's prep / bucket / tail
intervals."""
import csv, collections
rows=list(csv.DictReader(open('gpurun_out/r6s20trace/prof/run_kernel_trace.csv')))
iv=sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows if r["Kernel_Name"].startswith("k_msm"))
# assign kernels to runs: by order per kernel name
byname=collections.defaultdict(list)
for s,e,n in iv: byname[n].append((s,e))
K=['k_msm_prep','k_msm_hist','k_msm_wscan','k_msm_scatter','k_msm_bucket','k_msm_tail']
for n in K: byname[n].sort()
def run(i): return {n: byname[n][i] for n in K}
def window(a,b):
    runs=[run(i) for i in range(a,b)]
    t0=min(r['k_msm_prep'][0] for r in runs); t1=max(r['k_msm_tail'][1] for r in runs)
    sel=[(s,e) for s,e,n in iv if s<t1 and e>t0]
    ev=sorted([(max(s,t0),1) for s,e in sel]+[(min(e,t1),-1) for s,e in sel])
    busy=0;d=0;last=None
    for t,x in ev:
        if last is not None and d>0: busy+=t-last
        d+=x; last=t
    mean={n: sum(r[n][1]-r[n][0] for r in runs)/len(runs)/1e3 for n in K}
    lat=[(r['k_msm_tail'][1]-r['k_msm_prep'][0])/1e3 for r in runs]
    return (t1-t0)/1e3, busy/1e3, mean, lat
for nm,(a,b) in (('timed',(17,37)),('steady',(53,101))):
    span,busy,mean,lat=window(a,b)
    print(nm, 'span_us %.0f busy_us %.0f per_step_us %.1f'%(span,busy,span/(b-a)), {k:round(v,1) for k,v in mean.items()}, 'lat first/last', [round(x) for x in lat[:3]], [round(x) for x in lat[-3:]])
# timed region detail: prep starts and tail ends relative to t0
runs=[run(i) for i in range(17,37)]
t0=runs[0]['k_msm_prep'][0]
for i,r in enumerate(runs):
    print(i, 'prep %.0f-%.0f'%((r['k_msm_prep'][0]-t0)/1e3,(r['k_msm_prep'][1]-t0)/1e3), 'bucket %.0f-%.0f'%((r['k_msm_bucket'][0]-t0)/1e3,(r['k_msm_bucket'][1]-t0)/1e3), 'tail %.0f-%.0f'%((r['k_msm_tail'][0]-t0)/1e3,(r['k_msm_tail'][1]-t0)/1e3))
# previous run end (warmup) relative
w=run(16); print('warmup last tail end', (w['k_msm_tail'][1]-t0)/1e3)
