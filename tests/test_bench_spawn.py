"""bench.py --gpus N without torch.distributed.run: the script spawns one rank process per GPU
itself (before anything touches the GPU), the ranks rendezvous over gloo on 127.0.0.1, shard the
configs[1] timed region on every rank (value = all ranks' signatures / max-over-ranks time), then
shard the configs[2] index range and merge their verdict bitmaps; rank 0 prints one JSON line
with n_gpus = N.  NWV_BENCH_DRYRUN=1 replaces the engine by a shard verifier that rejects exactly the
injected indices, so this runs on the CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_spawns_ranks_and_merges(gpus):
    env = dict(os.environ, NWV_BENCH_DRYRUN="1", NWV_BENCH_DRYRUN_N="200000")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "4",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == gpus and d["dry_run"]
    # the headline is the configs[1] workload on every rank, value over all ranks (weak scaling)
    assert "configs[1]" in d["config"]["workload"] and d["scaling"] == "weak"
    assert d["value"] == pytest.approx(gpus * d["config"]["sigs_per_batch"] / (d["ms_per_step"] * 1e-3), rel=1e-9)
    assert d["firehose"]["exact_bad_set"]["exact"]
    assert d["firehose"]["sigs_total"] == 200000


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
