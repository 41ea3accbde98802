#!/usr/bin/env python3
"""Device time of BLAKE2b-256 over worker batches (configs[4]: 100 x 500,224 B) and over many
small digests, against hashlib on the host cores (same run)."""
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import narwhal_amd  # noqa: E402
from narwhal_amd import _lib  # noqa: E402


def timed(fn, reps):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


def main():
    eng = narwhal_amd.Engine(device=0)
    rng = np.random.default_rng(1)
    out = {}
    for nb, size in [(100, 500224), (1, 500224), (8192, 80), (100000, 80)]:
        msgs = [rng.bytes(size) for _ in range(nb)]
        # the arena is packed once, as a caller holding its messages in one buffer passes it; the
        # timed region is the C call (host buffers in, digests back on the host)
        lens = np.full(nb, size, dtype=np.uint64)
        offs = np.arange(nb, dtype=np.uint64) * np.uint64(size)
        arena = np.frombuffer(b"".join(msgs) + bytes(16), dtype=np.uint8)
        dig = np.zeros(32 * nb, dtype=np.uint8)

        def gpu():
            _lib._check(eng.lib.nwv_blake2b256_many(eng._h, nb, _lib._ptr(arena), _lib._ptr(offs), _lib._ptr(lens),
                                                    _lib._ptr(dig)))
        gpu()
        assert dig[:32].tobytes() == hashlib.blake2b(msgs[0], digest_size=32).digest()
        t = timed(gpu, 5 if size > 1000 else 3)
        threads = min(16, os.cpu_count() or 1)
        with ThreadPoolExecutor(threads) as ex:
            tc = timed(lambda: list(ex.map(lambda m: hashlib.blake2b(m, digest_size=32).digest(), msgs)), 3)
        t1 = timed(lambda: [hashlib.blake2b(m, digest_size=32).digest() for m in msgs[:max(1, nb // 10)]], 3) * (nb / max(1, nb // 10))
        out[f"{nb}x{size}"] = {"gpu_ms_host_to_host": t * 1e3, "cpu_threads_ms": tc * 1e3, "threads": threads,
                               "cpu_1thread_ms": t1 * 1e3, "gpu_GBps": nb * size / t / 1e9}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
