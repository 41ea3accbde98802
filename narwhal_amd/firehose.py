"""Firehose verification across the GPUs of one node (BASELINE.json configs[2]).

One process per GPU (torch.distributed.run).  The global signature index range [0, N) is split
into contiguous shards, 64-aligned so every shard's verdict words are whole; rank r verifies its
shard on its own GPU (batch MSM, per-signature fallback only for a rejected shard) and the host
merges the per-rank verdict bitmaps with one all_gather over gloo (N/8 bytes in total) and ANDs the
batch bits.  There is no data-path collective: signatures never leave their GPU, and the merged
result equals single-batch verification because each shard's batch check and the AND of
per-signature verdicts agree (up to the reference's own ~2^-128 bound).
"""
import numpy as np


def shard_range(n, world, rank):
    """contiguous 64-aligned [lo, hi) of rank `rank` among `world` for n signatures"""
    words = (n + 63) // 64
    per = (words + world - 1) // world
    lo = min(n, rank * per * 64)
    hi = min(n, (rank + 1) * per * 64)
    return lo, hi


def merge_verdicts(parts, n):
    """[(lo, hi, all_valid, words)] from every rank -> (all_valid, merged verdict words)"""
    out = np.zeros((n + 63) // 64, dtype=np.uint64)
    ok = True
    for lo, hi, allv, words in parts:
        if hi <= lo:
            continue
        assert lo % 64 == 0
        w = (hi - lo + 63) // 64
        out[lo // 64:lo // 64 + w] = words[:w]
        ok &= bool(allv)
    return ok, out


def firehose(verify_shard, n, dist=None):
    """Run verify_shard(lo, hi) -> (all_valid, verdict words of [lo, hi)) on this rank's shard and
    merge over `dist` (torch.distributed, gloo) when given.  Returns (all_valid, words) on every
    rank."""
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    lo, hi = shard_range(n, world, rank)
    allv, words = verify_shard(lo, hi) if hi > lo else (True, np.zeros(0, dtype=np.uint64))
    mine = (lo, hi, bool(allv), np.asarray(words, dtype=np.uint64))
    if dist is None:
        return merge_verdicts([mine], n)
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    return merge_verdicts(parts, n)


def gpu_shard_verifier(engine, pk, sig, arena, offs, lens, seed=None):
    """verify_shard for firehose(): stages [lo, hi) of the global SoA arrays on this rank's GPU
    and runs the batch MSM (fallback for exact verdicts only when the shard rejects)."""
    import os

    def run(lo, hi):
        st = engine.stage(pk[32 * lo:32 * hi], sig[64 * lo:64 * hi], arena, offs[lo:hi], lens[lo:hi])
        try:
            st.run(mode=1, seed=seed if seed is not None else os.urandom(32))
            allv, bits = st.fetch()
        finally:
            st.free()
        words = np.packbits(bits, bitorder="little").view(np.uint8)
        padded = np.zeros(((hi - lo + 63) // 64) * 8, dtype=np.uint8)
        padded[:words.size] = words
        return allv, padded.view(np.uint64)

    return run
