"""The committed measurement evidence (SURVEY §8 d) is self-consistent: the newest kernel trace of
the headline alone with ONE batch in flight (profiles/*_headline_inflight1_rocprof_kernel_stats.csv,
rocprofv3 --kernel-trace --stats of `bench.py --headline-only --inflight 1`) reproduces the
single-stream kernel times of the bench line printed by that same run
(*_headline_inflight1_bench_line.json) within 10 %, for the three kernels the roofline is read
from.  The trace with 12 batches in flight is kept under its own name (*_inflight12_*): its
averages are stretched by the overlap and are not kernel costs.  bench.py cites the inflight-1
trace in roofline.rocprof_source only while the pair carries HEAD's kernel_source_hash; the second
test reports (skips) when the newest pair predates today's device sources."""
import csv
import glob
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_msm_prep", "k_msm_bucket", "k_msm_tail")


def _pairs():
    out = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_headline_inflight1_rocprof_kernel_stats.csv"))):
        line = f.replace("_rocprof_kernel_stats.csv", "_bench_line.json")
        if os.path.exists(line):
            out.append((f, line))
    return out


def _load(pair):
    f, line = pair
    with open(f) as fh:
        avg = {r["Name"]: float(r["AverageNs"]) * 1e-6 for r in csv.DictReader(fh)}
    with open(line) as fh:
        bl = json.load(fh)
    return avg, bl


def test_newest_inflight1_trace_reproduces_its_bench_line():
    pairs = _pairs()
    assert pairs, "no committed *_headline_inflight1_rocprof_kernel_stats.csv with its bench line"
    avg, bl = _load(pairs[-1])
    assert bl["config"]["inflight_batches"] == 1
    for k in KERNELS:
        got, want = avg[k], bl["kernel_ms"][k]
        assert abs(got - want) <= 0.10 * want, (k, got, want)


def test_inflight12_trace_is_stored_apart():
    """the 12-in-flight trace never overwrites the one-in-flight one"""
    for f, _ in _pairs():
        twelve = f.replace("_inflight1_", "_inflight12_")
        assert twelve != f
        if os.path.exists(twelve):
            with open(twelve) as a, open(f) as b:
                assert a.read() != b.read()


def test_newest_pair_matches_head_sources():
    import sys
    sys.path.insert(0, ROOT)
    from narwhal_amd._lib import kernel_source_hash
    avg, bl = _load(_pairs()[-1])
    if bl.get("kernel_source_hash") != kernel_source_hash():
        pytest.skip("the newest headline trace predates today's Ed25519 device sources "
                    f"({bl.get('kernel_source_hash')} vs {kernel_source_hash()}): re-run "
                    "tools/gpurun/r5_evidence.sh")
