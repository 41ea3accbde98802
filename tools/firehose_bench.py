#!/usr/bin/env python3
"""configs[2]: a firehose of N signatures (default 16,777,216, 32 B messages) sharded by index
over the ranks of one node (python -m torch.distributed.run --nproc-per-node G ...; one GPU per
rank), verified as one batch MSM per shard, per-rank verdict bitmaps merged on the host over
gloo.  Each rank signs only its own shard (seeds derived from the global index), so no
signature data crosses ranks.  Prints one JSON line on rank 0."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16777216)
    ap.add_argument("--msg-len", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--bad", type=int, default=0, help="corrupt this many seeded indices")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    import narwhal_amd
    from narwhal_amd import firehose as fh

    eng = narwhal_amd.Engine(device=local)
    lo, hi = fh.shard_range(args.n, world, rank)
    m = hi - lo
    idx = np.arange(lo, hi, dtype=np.uint64)
    seeds = np.zeros((m, 32), dtype=np.uint8)
    seeds[:, :8] = idx.view(np.uint8).reshape(m, 8)
    seeds[:, 8] = 0xA5
    msgs = np.zeros((m, args.msg_len), dtype=np.uint8)
    msgs[:, :8] = (idx * np.uint64(0x9E3779B97F4A7C15)).view(np.uint8).reshape(m, 8)
    msgs = np.concatenate([msgs.reshape(-1), np.zeros(64, np.uint8)])
    offs = np.arange(m, dtype=np.uint64) * np.uint64(args.msg_len)
    lens = np.full(m, args.msg_len, dtype=np.uint32)
    t0 = time.perf_counter()
    pk, sg = eng.sign_many_arrays(seeds.reshape(-1), msgs, offs, lens)
    t_sign = time.perf_counter() - t0
    bad = set()
    if args.bad:
        rng = np.random.default_rng(4)
        bad = set(int(x) for x in rng.choice(args.n, size=args.bad, replace=False))
        for g in bad:
            if lo <= g < hi:
                sg[64 * (g - lo) + 40] ^= 1
    verify = fh.gpu_shard_verifier(eng, pk, sg, msgs, offs, lens)
    # stage once and time repeated batch verdicts of the resident shard
    st = eng.stage(pk, sg, msgs, offs, lens)
    st.run(mode=1, seed=b"\x01" * 32)
    st.sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for r in range(args.reps):
        st.run(mode=1, seed=bytes([r + 2]) * 32)
    st.sync()
    dt = time.perf_counter() - t0
    st.kernel_times(1, reset=True)
    st.run(mode=1, seed=b"\x09" * 32, timed=True)  # one kernel-by-kernel pass for the breakdown
    st.sync()
    kt = st.kernel_times(1)
    st.free()
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # merged verdicts (host bitmap merge over gloo) once, with the exact bad set
    t1 = time.perf_counter()
    ok, words = fh.firehose(lambda a, b: verify(a - lo, b - lo), args.n, dist)
    t_merge = time.perf_counter() - t1
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:args.n]
    got_bad = set(np.flatnonzero(bits == 0).tolist())
    assert got_bad == bad, (len(got_bad), len(bad))
    assert ok == (not bad)
    if rank == 0:
        print(json.dumps({"config": "firehose (BASELINE.json configs[2])", "n_total": args.n, "n_gpus": world,
                          "sigs_per_s": args.n * args.reps / dt, "ms_per_pass": dt / args.reps * 1e3,
                          "kernel_ms": kt, "verify_and_merge_s": t_merge, "sign_s": t_sign,
                          "bad": len(bad), "bad_found_exact": True}), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
