"""The split of nwv_bls_verify_many over a multi-device context (narwhal_amd/csrc/bls_shard.h,
SURVEY §8 e for the reference's default scheme): contiguous index ranges, one per device and host
thread, small calls on one device, statuses merged in item order, key registration on every
device, the failing range's code returned.  A stub stands in for the per-device verifier (CPU);
tests/test_gpu_bls.py runs the real split on the GPU against the oracle."""
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
    L.bst_ranges.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, vp, ctypes.c_int]
    L.bst_run.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_int]
    return L


def _ranges(lib, n, ndev, mn):
    out = np.zeros(2 * 64, dtype=np.uint64)
    k = lib.bst_ranges(n, ndev, mn, out.ctypes.data, 64)
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(k)]


@pytest.mark.parametrize("n,ndev,mn", [(1, 8, 256), (100, 8, 256), (511, 2, 256), (512, 2, 256),
                                       (16384, 8, 256), (16385, 8, 256), (1000, 3, 1), (7, 8, 1),
                                       (300, 1, 256), (5000, 8, 1000)])
def test_ranges_cover_items_in_order(lib, n, ndev, mn):
    r = _ranges(lib, n, ndev, mn)
    assert r[0][0] == 0 and r[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(r, r[1:]))  # contiguous, in order
    assert len(r) <= ndev
    assert all(hi > lo for lo, hi in r)
    if n < 2 * mn:
        assert len(r) == 1  # a small call stays on device 0
    else:
        assert all(hi - lo >= mn for lo, hi in r[:-1])
        sizes = [hi - lo for lo, hi in r]
        assert max(sizes) - min(sizes) <= max(mn, -(-n // ndev))


@pytest.mark.parametrize("n,ndev", [(16384, 8), (1000, 3), (300, 1), (100, 8)])
def test_statuses_land_in_item_order(lib, n, ndev):
    items = np.arange(n, dtype=np.int32) * 5 + 2
    status = np.zeros(n, dtype=np.int32)
    dev = np.full(n, -1, dtype=np.int32)
    reg = np.zeros(ndev, dtype=np.int32)
    threads = lib.bst_run(n, ndev, 256, items.ctypes.data, status.ctypes.data, dev.ctypes.data,
                          reg.ctypes.data, -1)
    r = _ranges(lib, n, ndev, 256)
    assert threads == len(r)  # one host thread per range
    assert (status == items * 3 + 1).all()
    for k, (lo, hi) in enumerate(r):
        assert (dev[lo:hi] == k).all()
    assert (reg == 1).all()  # every device got the committee's keys


def test_failing_range_code_returned(lib):
    n, ndev = 4096, 4
    items = np.arange(n, dtype=np.int32)
    status = np.zeros(n, dtype=np.int32)
    dev = np.zeros(n, dtype=np.int32)
    reg = np.zeros(ndev, dtype=np.int32)
    assert lib.bst_run(n, ndev, 256, items.ctypes.data, status.ctypes.data, dev.ctypes.data, reg.ctypes.data, 2) >= 1
