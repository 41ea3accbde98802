"""Host-side control flow of the mixed-batch types path (nwv_types.cpp) on the CPU: the engine calls
are stubbed (tools/hostbench/types_hostbench.cpp), so this checks that a whole 100-node round
(headers, votes, certificates) goes through nwv_verify_mixed_many with every item Ok and reports the
host cost.  No GPU."""
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mixed_round_host_path(tmp_path):
    exe = tmp_path / "types_hostbench"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-o", str(exe),
                    os.path.join(ROOT, "tools/hostbench/types_hostbench.cpp"),
                    os.path.join(ROOT, "narwhal_amd/csrc/nwv_types.cpp")], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    assert r["host_us_per_round_min"] > 0
