#!/bin/bash
# in-flight batches re-sweep at HEAD (headline only, same box): 10 / 12 / 14 / 16, then 12 again
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
for k in 10 12 14 16 12; do
  timeout -k 10 200 python3 -u bench.py --no-configs --no-cpu-baseline --latency-reps 20 --h2h-seconds 0 --steps 384 --inflight $k > $O/if2_$k.json 2> $O/if2_$k.err || exit $?
  python3 -c "import json;b=json.loads(open('$O/if2_$k.json').read().strip().splitlines()[-1]);print('inflight $k', round(b['value']/1e6,1))"
done
echo ALLDONE
