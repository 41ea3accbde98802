"""configs[4] (C5) leg alone (tools/config_legs.leg_c5) -> one JSON line"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import narwhal_amd  # noqa: E402
import config_legs as CL  # noqa: E402

e = narwhal_amd.Engine(device=0)
out, _ = CL.leg_c5(e, rounds=int(sys.argv[1]) if len(sys.argv) > 1 else 20)
print(json.dumps(out), flush=True)
