"""Multi-GPU plumbing of the firehose (configs[2]) on the CPU: 64-aligned index
shards, and the host-side verdict merge over gloo with world_size 2 and 3.  The per-rank shard
verifier here is the oracle (the checker) -- on the GPU box each rank runs
narwhal_amd.firehose.gpu_shard_verifier on its own device."""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from narwhal_amd import firehose as fh


def test_shards_cover_and_align():
    for n in [0, 1, 63, 64, 65, 1000, 4096, 16777216]:
        for world in [1, 2, 3, 4, 8]:
            rs = [fh.shard_range(n, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c
            assert all(lo % 64 == 0 for lo, hi in rs if hi > lo)


def _items(n, seed):
    import oracle_ffi as of
    rnd = random.Random(seed)
    items = []
    for i in range(n):
        s = bytes([i % 256, i // 256]) + bytes(30)
        m = rnd.randbytes(32)
        sig = bytearray(of.sign(s, m))
        if rnd.random() < 0.05:
            sig[rnd.randrange(64)] ^= 1
        items.append((of.pubkey(s), bytes(sig), m))
    return items


def _oracle_shard(items):
    import oracle_ffi as of

    def run(lo, hi):
        v = np.array([of.verify(*items[i]) for i in range(lo, hi)], dtype=bool)
        w = np.zeros(((hi - lo + 63) // 64) * 8, dtype=np.uint8)
        b = np.packbits(v, bitorder="little")
        w[:b.size] = b
        return bool(v.all()), w.view(np.uint64)

    return run


def _worker(rank, world, port, n, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    items = _items(n, 3)
    ok, words = fh.firehose(_oracle_shard(items), n, dist)
    dist.destroy_process_group()
    q.put((rank, ok, words.tobytes()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,n", [(2, 300), (3, 200)])
def test_gloo_verdict_merge(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle_ffi as of
    items = _items(n, 3)
    want = np.array([of.verify(*it) for it in items], dtype=bool)
    for rank, ok, raw in res:
        got = np.unpackbits(np.frombuffer(raw, dtype=np.uint8), bitorder="little")[:n].astype(bool)
        assert (got == want).all()
        assert ok == bool(want.all())
