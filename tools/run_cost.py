import os, sys, time, json
os.environ["GPU_MAX_HW_QUEUES"] = "16"
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np
import narwhal_amd
import bench
eng = narwhal_amd.Engine(device=0)
pk, sg, msgs, offs, lens = bench.synth(eng, 65536, 512, 1)
stages = [eng.stage(pk, sg, msgs, offs, lens) for _ in range(12)]
for s in stages: s.run(mode=1)
for s in stages: s.sync()
out = {}
for label, seed in (("null", None), ("bytes", b"\x07" * 32)):
    for K in (20, 200):
        for s in stages: s.sync()
        t0 = time.perf_counter(); calls = []
        for k in range(K):
            c = time.perf_counter()
            stages[k % 12].run(mode=1, seed=seed)
            calls.append(time.perf_counter() - c)
        t1 = time.perf_counter()
        for s in stages: s.sync()
        t2 = time.perf_counter()
        out[f"{label}_{K}"] = {"enqueue_ms": (t1 - t0) * 1e3, "total_ms": (t2 - t0) * 1e3,
                               "call_us_p50": float(np.median(calls)) * 1e6, "call_us_max": max(calls) * 1e6,
                               "ms_per_step": (t2 - t0) * 1e3 / K}
print(json.dumps(out))
