"""The split of an Ed25519 call over a multi-device context (narwhal_amd/csrc/shard.h, used by
nwv_host.hip for_shards -- the path a one-context-for-all-GPUs caller such as the Rust crate's
nwv_init(ctx, 0, 0) takes): contiguous 64-aligned ranges, at most one per device, at least
NWV_SHARD_MIN signatures each so that a certificate or a 1K batch stays on one device, and
verdict words written by several host threads at once merging into exactly the per-index
verdicts (the semantics of primary/src/block_synchronizer/responses.rs:115-138 survive the split).
tests/test_gpu_shard.py runs the real split over a 3-replica context on the GPU."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "_build", "libblsshard.so")


@pytest.fixture(scope="module")
def lib():
    subprocess.run(["make", "-s", "-C", ROOT, "tests/_build/libblsshard.so"], check=True)
    L = ctypes.CDLL(SO)
    vp = ctypes.c_void_p
    u64 = ctypes.c_uint64
    L.bst_ed_ranges.argtypes = [u64, u64, u64, vp, ctypes.c_int]
    L.bst_ed_merge.argtypes = [u64, u64, u64, vp, vp, ctypes.c_int]
    return L


def _ranges(lib, n, ndev, mn):
    out = np.zeros(2 * 64, dtype=np.uint64)
    k = lib.bst_ed_ranges(n, ndev, mn, out.ctypes.data, 64)
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(k)]


CASES = [(1, 8, 16384), (4, 8, 16384), (1024, 8, 16384), (32767, 8, 16384), (32768, 8, 16384),
         (65536 + 37, 3, 16384), (65536 + 37, 8, 16384), (16 << 20, 8, 16384), (6999, 8, 1024),
         (65, 2, 1), (64, 8, 1), (1000, 3, 1), (300, 1, 16384), (2 << 20, 8, 16384)]


@pytest.mark.parametrize("n,ndev,mn", CASES)
def test_ranges(lib, n, ndev, mn):
    r = _ranges(lib, n, ndev, mn)
    assert r[0][0] == 0 and r[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))  # contiguous, in order
    assert all(hi > lo for lo, hi in r)  # no empty range (no idle host thread)
    assert all(lo % 64 == 0 for lo, _ in r)  # every range owns whole verdict words
    assert len(r) <= ndev
    if n < 2 * mn:
        assert len(r) == 1  # a certificate, a 1K batch, a DAG round: one device
    else:
        assert len(r) == min(ndev, n // mn, -(-n // 64))
        assert all(hi - lo >= mn - 64 for lo, hi in r)
        sizes = [hi - lo for lo, hi in r]
        assert max(sizes) - min(sizes) <= 128  # near-equal, counted in whole words


def test_min_shard_keeps_small_calls_on_device0(lib):
    # the default NWV_SHARD_MIN: a 4-node certificate and the 1K batch are one range on 8 devices
    for n in (3, 4, 68, 1024, 6999, 16384):
        assert _ranges(lib, n, 8, 16384) == [(0, n)]
    # the headline batch splits over 4 devices (16,384 each), the firehose over all 8
    assert len(_ranges(lib, 65536, 8, 16384)) == 4
    assert len(_ranges(lib, 2 << 20, 8, 16384)) == 8


@pytest.mark.parametrize("n,ndev,mn", [(65536 + 37, 3, 16384), (6999, 8, 64), (1000, 7, 1), (200, 4, 1)])
def test_verdict_words_merge_exactly(lib, n, ndev, mn):
    rnd = np.random.default_rng(n)
    valid = (rnd.random(n) > 0.01).astype(np.uint8)
    r = _ranges(lib, n, ndev, mn)
    # invalid signatures on both sides of every range boundary
    for lo, _ in r[1:]:
        valid[lo - 1] = 0
        valid[lo] = 0
    words = (n + 63) // 64
    bits = np.full(words, 0xFFFFFFFFFFFFFFFF, dtype=np.uint64)  # stale words from an earlier call
    k = lib.bst_ed_merge(n, ndev, mn, valid.ctypes.data, bits.ctypes.data, 20)
    assert k == len(r)
    got = np.unpackbits(bits.view(np.uint8), bitorder="little")[:n]
    assert (got == valid).all()
    assert sorted(np.flatnonzero(got == 0).tolist()) == sorted(np.flatnonzero(valid == 0).tolist())
