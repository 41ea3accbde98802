"""the BLS12-381 leg alone (tools/config_legs.leg_bls) -> one JSON line"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
import config_legs as CL  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import usable_cpus  # noqa: E402
e = narwhal_amd.Engine(device=0)
from bench import valu_peak  # noqa: E402
pk = valu_peak()
print(json.dumps(CL.leg_bls(e, threads=usable_cpus(), throughput_n=n, peak=pk)), flush=True)
