#!/usr/bin/env python3
"""bench.py -- Ed25519 signatures verified per second on MI355X (BASELINE.json metric).

N = 1 (default): BASELINE.json configs[1].  A step is one batch verdict over one resident batch of
65,536 valid signatures with 512-byte messages and distinct keys (synthetic: seeded keys and
messages, RFC 8032 signatures made on the GPU), through the batch MSM (K5, ed25519_consensus
batch::Verifier semantics).  --inflight K keeps K resident batches on K streams and issues the
steps round-robin; the single-stream step time is reported beside it.

N > 1 (--gpus N): the same configs[1] workload on every rank, one process per GPU, no collective
in the data path; value = all ranks' signatures / the max-over-ranks time (weak scaling, so the
1/2/4/8 values form a same-workload series).  Without WORLD_SIZE in the environment, --gpus N
spawns the N rank processes itself (before anything touches the GPU); torch.distributed.run
launches them the same way.  The configs[2] firehose then runs as the `firehose` field: 16,777,216
signatures (32-byte messages) sharded by contiguous 64-aligned index ranges over the ranks (strong
scaling), verified as resident sub-shards, the verdict bitmaps merged once over gloo for the
exact-bad-set check.

Extra fields: roofline (dominant kernel) and roofline_per_kernel, cpu_baseline (the oracle's
batch verifier on the host's usable cores, rank 0, N = 1), host_to_host (pipelined verification of
host-resident batches, PCIe included), latency of a 1,024-signature batch host -> host, the C3
firehose on one GPU, the C1 / C4 / C5 legs with their CPU counterparts, and configs.BLS: the
reference's default scheme (BLS12-381) -- a 100-certificate round, single Verifier::verify latency,
concurrent callers, 16,384 single-key items, the C5 DAG round through the BLS types layer -- with
its oracle checks and CPU baseline.  With N > 1 the firehose also appears at top level
(firehose_sigs_per_s, firehose_scaling "strong").
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

import numpy as np

# Hardware queues per process (HIP's default is 4).  Each resident batch runs on its own stream;
# with 4 queues the streams share queues and a batch's latency-bound MSM tail serialises the work
# queued behind it (profiles/round1_hwq_sweep.jsonl).  Must be set before the HIP runtime
# initialises (NWV_BENCH_HW_QUEUES picks another count).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("NWV_BENCH_HW_QUEUES", "16")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FIREHOSE_N = 16777216
SUBSHARD = 2097152

# Algorithmic field multiplications (one 255-bit product: a 10 x 10 limb schoolbook = 100
# v_mad_u64_u32; a squaring 55), counted on the host-emulation build
# (tests/test_hostemu.py::test_phase_op_counts, tests/test_msm_hostemu.py)
MADS_PER_MUL, MADS_PER_SQ = 100, 55
OPS_POINTS = (174, 514)      # k_ed_points, per signature: decompress R and A + the 0..8 A and R tables
OPS_MSM_POINTS = (48, 514)   # MSM decompression, per signature: R_i and A_i
MADS_DECOMPRESS = (OPS_MSM_POINTS[0] * MADS_PER_MUL + OPS_MSM_POINTS[1] * MADS_PER_SQ) // 2  # per point
MADS_MIXED_ADD = 7 * MADS_PER_MUL                          # per bucket entry (affine Niels)
MADS_ADD = 9 * MADS_PER_MUL                                # extended + extended
MADS_DBL = 4 * MADS_PER_MUL + 4 * MADS_PER_SQ              # projective doubling
# SHA-512 (sha512.h), 32-bit VALU instructions per 128-byte block: a round is 34 (two 64-bit
# rotations x3 as v_alignbit pairs, two v_xor3 pairs, two v_bitop3 pairs, six 64-bit adds), a
# message-schedule step 22 (four rotations, a shift, two v_xor3 pairs, three 64-bit adds); 80
# rounds + 64 steps + the state update.  Counted against the v_mad_u64_u32 roofline at the
# guide's 2:1 issue ratio (a 32-bit form issues in half the time of a 64-bit-result form)
SHA512_VALU_PER_BLOCK = 80 * 34 + 64 * 22 + 16


def sha512_blocks(nbytes):
    return (nbytes + 17 + 127) // 128


OPS_STRAUS = (1155, 524)     # k_ed_straus: half-size scalars, 132 doublings (ed25519_lane.h)
# guide-derived VALU peaks (MI355X_MICROARCH.md: 256 CUs x 4 SIMD-32 x 2.4 GHz, a wave64 VALU
# instruction issues over 2 cycles): 78.6 T lane-ops/s for full-rate 32-bit forms; the 64-bit
# result VOP3 forms (v_mad_u64_u32) issue at half that
GUIDE_VALU32 = 256 * 4 * 32 * 2.4e9
GUIDE_MAD64 = GUIDE_VALU32 / 2
HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def usable_cpus():
    """CPUs this process may use: its affinity set, capped by the cgroup CPU quota and by the
    job's thread budget (OMP_NUM_THREADS; the GPU box exposes the whole machine to nproc but
    grants each job a share of 16).  NWV_CPU_THREADS overrides."""
    if os.environ.get("NWV_CPU_THREADS"):
        return max(1, int(os.environ["NWV_CPU_THREADS"]))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        n = min(n, max(1, int(os.environ["OMP_NUM_THREADS"])))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def valu_peak():
    exe = os.path.join(ROOT, "tools", "ubench_valu")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # measurement helper only
        log("ubench failed:", e)
        return None


def synth(eng, n, mlen, seed, keys=0):
    """n signatures over seeded random messages; keys > 0: signed by `keys` seeded keys in turn
    (signature i by key i % keys), else every signature by its own key"""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
    if keys:
        seeds = np.tile(seeds[:32 * keys], (n + keys - 1) // keys)[:32 * n].copy()
    msgs = rng.integers(0, 256, size=n * mlen + 64, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(mlen)
    lens = np.full(n, mlen, dtype=np.uint32)
    pk, sg = eng.sign_many_arrays(seeds, msgs, offs, lens)
    return pk, sg, msgs, offs, lens


def firehose_shard_data(eng, lo, hi, mlen=32):
    """signatures [lo, hi) of the configs[2] firehose: key seed and message derived from the global
    index, so every rank signs only its own shard and no signature data crosses ranks"""
    m = hi - lo
    idx = np.arange(lo, hi, dtype=np.uint64)
    seeds = np.zeros((m, 32), dtype=np.uint8)
    seeds[:, :8] = idx.view(np.uint8).reshape(m, 8)
    seeds[:, 8] = 0xA5
    msgs = np.zeros((m, mlen), dtype=np.uint8)
    msgs[:, :8] = (idx * np.uint64(0x9E3779B97F4A7C15)).view(np.uint8).reshape(m, 8)
    msgs = np.concatenate([msgs.reshape(-1), np.zeros(64, np.uint8)])
    offs = np.arange(m, dtype=np.uint64) * np.uint64(mlen)
    lens = np.full(m, mlen, dtype=np.uint32)
    pk, sg = eng.sign_many_arrays(seeds.reshape(-1), msgs, offs, lens)
    return pk, sg, msgs, offs, lens


# ------------------------------------------------------------------------------- CPU legs --
def cpu_baseline(pk, sg, msgs, offs, lens, seconds, threads):
    """the oracle's batch verifier (dalek's algorithms in C: radix-2^51, Pippenger) over the SAME
    65,536 x 512 B batch, split by index over `threads` host threads"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as of  # the checker; timed here as the CPU baseline only
    n = len(offs)
    P, S, M = pk[:32 * n].tobytes(), sg[:64 * n].tobytes(), msgs.tobytes()
    done, reps, t0 = 0, 0, time.perf_counter()
    while True:
        ok = of.verify_batch_mt(P, S, M, offs.copy(), lens.copy(), threads, seed=os.urandom(32))
        assert ok, "CPU baseline rejected a valid batch"
        done += n
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "sigs/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x the same {n}-signature batch of 512 B messages (configs[1]), "
                      f"split by index over {threads} threads (all CPUs granted to this job), "
                      "oracle/nwv_oracle.c batch verifier: radix-2^51 field and Pippenger as "
                      "curve25519-dalek-ng u64_backend / ed25519-consensus",
            "ms_per_batch": dt / reps * 1e3}


def cpu_baseline_configs(legs, data, threads):
    """CPU legs of C1 / C4 / C5 (the oracle: dalek's algorithms in C, the reference's control flow
    in Python).  C1 and C5's signature checks run on ONE core: the reference verifies inside its
    single Core task (primary/src/core.rs:614-714); C4 and the C5 digests use `threads` threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import hashlib
    from concurrent.futures import ThreadPoolExecutor
    import oracle_ffi as of  # checker / CPU baseline only
    import narwhal_types as nt

    def ocom(c):
        return nt.Committee(list(c.keys), list(c.stakes), c.epoch, [list(w) for w in c.workers])

    def hdict(h):
        return {"author": h.author, "round": h.round, "epoch": h.epoch, "payload": list(h.payload),
                "parents": list(h.parents), "id": h.id, "signature": h.signature}

    def cert_verify(c, cert):
        """Certificate::verify as the reference runs it: header check, quorum, then the
        aggregate signature as ONE batch verification (ed25519-consensus batch::Verifier)"""
        h = hdict(cert.header)
        r = nt.header_verify(c, h, of.verify)
        if r:
            return r
        pks = [c.keys[a] for a in cert.signed_authorities]
        if sum(c.stakes[a] for a in cert.signed_authorities) < c.quorum_threshold():
            return nt.REQUIRES_QUORUM
        d = nt.certificate_digest(h["id"], h["round"], h["epoch"], h["author"])
        return 0 if of.verify_batch([(pk, s, d) for pk, s in zip(pks, cert.aggregated_signature)]) else 1

    def timed(fn, reps):
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t)
        return float(np.median(ts)) * 1e3

    out = {}
    c1 = data["C1"]
    com1 = ocom(c1["committee"])
    assert cert_verify(com1, c1["cert"]) == 0
    out["C1"] = {"certificate_verify_n4_ms": timed(lambda: cert_verify(com1, c1["cert"]), 200),
                 "verify_batch_1024_m32_ms": timed(lambda: of.verify_batch(c1["items"]), 20), "cores": 1,
                 "note": "one core, as the reference's single Core task verifies"}
    c4 = data["C4"]
    pk, sig, msg, offs, lens = of.pack(c4["items"])
    t = time.perf_counter()
    ok = of.verify_batch_mt(pk, sig, msg, offs, lens, threads)
    bits = of.verify_each_mt(pk, sig, msg, offs, lens, threads)
    dt = time.perf_counter() - t
    ref = np.unpackbits(bits.view(np.uint8), bitorder="little")[:len(offs)].astype(bool)
    out["C4"] = {"ms_per_batch": dt * 1e3, "sigs_per_s": len(offs) / dt, "cores": threads,
                 "batch_verdict": ok, "gpu_bits_equal_oracle": bool((ref == np.asarray(c4["bits"])).all())}
    c5 = data["C5"]
    com5 = ocom(c5["committee"])

    def round_cpu():
        assert all(cert_verify(com5, c) == 0 for c in c5["certs"])
        assert all(nt.header_verify(com5, hdict(h), of.verify) == 0 for h in c5["headers"])
        assert all(nt.vote_verify(com5, {"id": v.id, "round": v.round, "epoch": v.epoch, "origin": v.origin,
                                         "author": v.author, "signature": v.signature}, of.verify) == 0
                   for v in c5["votes"])
    ms5 = timed(round_cpu, 3)
    with ThreadPoolExecutor(threads) as ex:
        msd = timed(lambda: list(ex.map(lambda b: hashlib.blake2b(b, digest_size=32).digest(), c5["batches"])), 3)
    one = c5["batches"][0]
    ms1 = timed(lambda: hashlib.blake2b(one, digest_size=32).digest(), 20)
    out["C5"] = {"verify_ms_per_round": ms5, "verify_cores": 1,
                 "verify_sigs_per_s": legs["C5"]["signatures_per_round"] / (ms5 * 1e-3),
                 "worker_batch_digests_ms_per_round": msd, "digest_threads": threads,
                 "one_worker_batch_digest_ms_1core": ms1}
    return out


# ------------------------------------------------------------------------------ roofline --
MSM_KERNELS = ("k_msm_prep", "k_msm_hash", "k_msm_decomp", "k_msm_hist", "k_msm_wscan", "k_msm_scatter",
               "k_msm_lsort", "k_msm_sort1", "k_msm_bucket", "k_msm_bucket_q", "k_msm_tail", "k_msm_keysum",
               "k_msm_fixup", "k_msm_bscalar")


def pmc_file(n, launch):
    """(summary, path) of the newest committed rocprofv3 --pmc summary (tools/pmc_summary.py) that
    describes TODAY's pipeline at batch size n: its kernel_source_hash equals the hash of the
    device sources at HEAD, and its MSM kernels are exactly `launch` (the kernels this run
    launched); else (None, None), and the counter-derived fields are reported as null"""
    import glob
    from narwhal_amd._lib import kernel_source_hash
    want = kernel_source_hash()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("n") != n or d.get("kernel_source_hash") != want:
            continue
        have = {k for k in d.get("kernels", {}) if k in MSM_KERNELS}
        if have != set(k for k in launch if k in MSM_KERNELS):
            continue
        return d, os.path.relpath(f, ROOT)
    return None, None


def rocprof_headline(kernels=("k_msm_prep", "k_msm_bucket", "k_msm_tail")):
    """the newest committed rocprofv3 --kernel-trace --stats summary of the headline alone with ONE
    batch in flight (profiles/*_headline_inflight1_rocprof_kernel_stats.csv) whose stored bench line
    (*_headline_inflight1_bench_line.json, the same run) carries today's kernel_source_hash: its
    per-kernel averages are single-stream kernel times, comparable with the line's kernel_ms
    (tests/test_profiles_evidence.py); else None"""
    import csv
    import glob
    from narwhal_amd._lib import kernel_source_hash
    want = kernel_source_hash()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_headline_inflight1_rocprof_kernel_stats.csv")),
                    reverse=True):
        line = f.replace("_rocprof_kernel_stats.csv", "_bench_line.json")
        try:
            with open(line) as fh:
                bl = json.load(fh)
            with open(f) as fh:
                rows = {r["Name"]: r for r in csv.DictReader(fh)}
        except (OSError, ValueError, KeyError):
            continue
        if bl.get("kernel_source_hash") != want:
            continue
        return {"source": os.path.relpath(f, ROOT), "bench_line": os.path.relpath(line, ROOT),
                "avg_ms": {k: float(rows[k]["AverageNs"]) * 1e-6 for k in kernels if k in rows},
                "line_kernel_ms": {k: bl.get("kernel_ms", {}).get(k) for k in kernels}}
    return None


def pmc_kernel(kernel, n, launch):
    """(counters, source) of `kernel` from pmc_file(n, launch), or (None, None)"""
    d, src = pmc_file(n, launch)
    k = (d or {}).get("kernels", {}).get(kernel)
    return (k, src) if k else (None, None)


def pmc_traffic(kernels, n, launch):
    """HBM bytes per launch from the committed rocprofv3 --pmc passes (FETCH_SIZE doubled for
    gfx950's half-counted wide reads + WRITE_SIZE, MI355X_MICROARCH.md HBM section)"""
    total, srcs = 0.0, set()
    for k in kernels:
        c, src = pmc_kernel(k, n, launch)
        if not c or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            return None
        total += 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
        srcs.add(src)
    return {"bytes": total, "source": sorted(srcs)}


def issue_floor(kernels, n, kms, peak, launch):
    """mix-weighted VALU issue floor: the committed PMC pass's wave-level VALU instructions of the
    kernel, the 64-bit integer forms (SQ_INSTS_VALU_INT64) priced at the measured v_mad_u64_u32
    rate and the rest at the measured v_add_u32 rate, against the live kernel time"""
    if not peak or kms <= 0:
        return None
    v = i64 = 0.0
    srcs = set()
    for k in kernels:
        c, src = pmc_kernel(k, n, launch)
        if not c or "SQ_INSTS_VALU" not in c or "SQ_INSTS_VALU_INT64" not in c:
            return None
        v += c["SQ_INSTS_VALU"]
        i64 += c["SQ_INSTS_VALU_INT64"]
        srcs.add(src)
    floor_s = i64 * 64 / peak["v_mad_u64_u32_per_s"] + (v - i64) * 64 / peak["v_add_u32_per_s"]
    return {"valu_insts_per_launch": v, "int64_insts": i64, "floor_ms": floor_s * 1e3,
            "frac": floor_s / (kms * 1e-3), "source": sorted(srcs)}


def kernel_rooflines(kt, stats, n, na, peak, mlen):
    """roofline of every kernel of the batch MSM from its single-stream, event-timed duration"""
    mad_peak = peak["v_mad_u64_u32_per_s"] / 1e12 if peak else None
    nw, nwz, buckets, E = stats["windows"], stats["windows_z"], stats["buckets"], stats["entries"]
    digit_slots = (na + 1) * nw + n * nwz
    cnt_len = buckets * stats["chunks"]
    launch = list(kt)
    out = {}

    def valu(name, pmc, mads, what):
        kms = kt.get(name, 0.0)
        a = mads / (kms * 1e-3) / 1e12 if kms > 0 else None
        out[name] = {"bound": "valu", "achieved": a, "unit": "T v_mad_u64_u32/s", "peak": mad_peak,
                     "frac": (a / mad_peak) if (a and mad_peak) else None,
                     "peak_guide": GUIDE_MAD64 / 1e12, "frac_guide": (a / (GUIDE_MAD64 / 1e12)) if a else None,
                     "algorithmic": what, "mads_per_launch": mads, "kernel_ms": kms,
                     "traffic": (pmc_traffic(pmc, n, launch) or {}).get("bytes"),
                     "issue_floor": issue_floor(pmc, n, kms, peak, launch)}

    def mem(name, pmc, nbytes, what):
        kms = kt.get(name, 0.0)
        a = nbytes / (kms * 1e-3) / 1e9 if kms > 0 else None
        tr = pmc_traffic(pmc, n, launch)
        out[name] = {"bound": "hbm", "achieved": a, "unit": "GB/s", "peak": HBM_PEAK_GBS,
                     "frac": (a / HBM_PEAK_GBS) if a else None, "algorithmic": what,
                     "bytes_per_launch": nbytes, "kernel_ms": kms,
                     "traffic": tr["bytes"] if tr else None,
                     "traffic_over_algorithmic": (tr["bytes"] / nbytes) if tr and nbytes else None}

    sha_blocks = sha512_blocks(64 + mlen)
    sha_eq = SHA512_VALU_PER_BLOCK * sha_blocks // 2
    valu("k_msm_prep", ["k_msm_prep"], MADS_DECOMPRESS * (na + n) + sha_eq * n,
         f"{MADS_DECOMPRESS} multiply-adds per decompressed point (24 mul + 257 sq) x {na + n} points "
         f"(R_i and the A points), plus SHA-512(R || A || M) per signature: {sha_blocks} blocks x "
         f"{SHA512_VALU_PER_BLOCK} 32-bit VALU instructions = {sha_eq} multiply-add equivalents "
         f"(2 : 1 issue) x {n} signatures")
    # the SHA-512 share is a count of compiled 32-bit instructions, not multiply-adds: the
    # decompression-only figure (round 3's numerator, a lower bound) stays beside it
    pr = out["k_msm_prep"]
    pr["mads_sha512_equiv_per_launch"] = sha_eq * n
    pr["mads_decompression_per_launch"] = MADS_DECOMPRESS * (na + n)
    kms = pr["kernel_ms"]
    a_dec = MADS_DECOMPRESS * (na + n) / (kms * 1e-3) / 1e12 if kms > 0 else None
    pr["achieved_decompression_only"] = a_dec
    pr["frac_decompression_only"] = (a_dec / mad_peak) if (a_dec and mad_peak) else None
    mem("k_msm_hist", ["k_msm_hist"], 2 * digit_slots + 4 * cnt_len,
        f"read the i16 digit rows ({digit_slots} slots), write {cnt_len} u32 counts")
    mem("k_msm_wscan", ["k_msm_wscan"], 8 * cnt_len,
        f"read the {cnt_len} counts and write them back as offsets (unique bytes: the workgroup's "
        "second pass re-reads its window's counts from L2, and k_msm_hist has just written them, so "
        "part of the first read can come from the MALL too)")
    mem("k_msm_scatter", ["k_msm_scatter"], 2 * digit_slots + 4 * cnt_len + 4 * E,
        f"read the digit rows and the {cnt_len} bucket offsets, write {E} u32 entries")
    valu("k_msm_bucket", ["k_msm_bucket"], MADS_MIXED_ADD * E,
         f"{MADS_MIXED_ADD} multiply-adds per bucket entry (one mixed addition, 7 mul) x {E} entries")
    valu("k_msm_tail", ["k_msm_tail"], 2 * MADS_ADD * buckets + 256 * MADS_DBL * nw,
         f"window sums: two extended additions ({MADS_ADD} multiply-adds each) per bucket x {buckets} "
         f"buckets (running sums), then each of the {nw} windows scaled by up to ~256 doublings "
         f"({MADS_DBL} multiply-adds each; the top window's chain is latency-bound by construction); "
         "the joins of buckets spanning bucket lanes (about one extended addition per bucket) are not counted")
    return out


# ------------------------------------------------------------------------------- N = 1 ----
def timed_region(stages, args, dist, run):
    """The bench contract's timed region: W untimed warmup steps, then (every stage synchronised,
    barrier) exactly K steps, step s on stage s % len(stages), then every stage synchronised and a
    barrier.  Returns (this rank's seconds, the max over ranks)."""
    for w in range(args.warmup):
        run(stages[w % len(stages)])
    for s_ in stages:
        s_.sync()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(args.steps):
        run(stages[s % len(stages)])
    for s_ in stages:
        s_.sync()
    dt = time.perf_counter() - t0
    dt_max = dt
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_max = float(t.item())
        dist.barrier()
    return dt, dt_max


def steady_state(stages, args, run):
    """After the contract's timed region (never part of `value`): `args.steady_steps` more steps
    through the same stages, a HIP event recorded on each step's stream when it completes, and
    the interval between completions from the quarter mark on -- the pipeline's steady-state rate,
    which a short timed region (the driver's --steps 20) cannot show because it starts from an
    idle GPU (every stage synchronised) and ends with a drain.  `ramp_and_drain_cost` = how much
    longer the contract's K steps took than K steady steps."""
    K = args.steady_steps
    if K < 16 or K >= 65535 or not hasattr(stages[0], "mark"):
        return None
    for s_ in stages:
        s_.sync()
    stages[0].mark(0)
    for s in range(K):
        run(stages[s % len(stages)])
        stages[s % len(stages)].mark(s + 1)
    for s_ in stages:
        s_.sync()
    c = sorted(stages[0].mark_elapsed(0, stages[s % len(stages)], s + 1) for s in range(K))
    q = K // 4
    slope = (c[-1] - c[q]) / (K - 1 - q)
    return {"ms_per_step": slope, "sigs_per_s": args.n / (slope * 1e-3), "steps": K,
            "first_completion_ms": c[0], "last_completion_ms": c[-1],
            "note": f"{K} extra steps after the timed region, HIP events on step completion: interval "
                    f"between completions from the {q}-th on (not `value`, which is the contract's host-timed "
                    "K steps from an idle GPU, ramp and drain included)"}


class DryStage:
    """NWV_BENCH_DRYRUN stand-in for a resident batch (CPU tests of the multi-rank timing path):
    a step is a fixed amount of host work, every verdict valid"""

    def __init__(self, n):
        self.n = n
        self.runs = 0

    def run(self, mode=1, timed=False):
        self.runs += 1
        np.sort(np.random.default_rng(self.runs).integers(0, 1 << 30, 20000))

    def sync(self):
        pass


def run_headline_dry(args, rank, world, dist):
    stages = [DryStage(args.n) for _ in range(max(1, args.inflight))]
    dt, dt_max = timed_region(stages, args, dist, lambda st: st.run())
    return {"dt": dt, "dt_max": dt_max}


def run_headline(args, eng, rank, world, dist):
    from narwhal_amd import _lib
    pk, sg, msgs, offs, lens = synth(eng, args.n, args.msg_len, seed=1000 + rank, keys=args.keys)
    if args.keys:
        kidx = np.arange(args.n, dtype=np.uint32) % np.uint32(args.keys)
        stages = [eng.stage_keyed(pk[:32 * args.keys].copy(), kidx, sg, msgs, offs, lens)
                  for _ in range(max(1, args.inflight))]
    else:
        stages = [eng.stage(pk, sg, msgs, offs, lens) for _ in range(max(1, args.inflight))]

    def check_all(what):
        for s_ in stages:
            allv, bits = s_.fetch()
            if not (allv and bits.all()):
                raise SystemExit(f"verification of a valid synthetic batch failed ({what})")

    # setup (untimed, not counted as warmup): every stage's first run allocates its MSM scratch
    # and captures its HIP graph; every verdict is checked
    for s_ in stages:
        s_.run(mode=args.mode)
    check_all("setup")
    dt, dt_max = timed_region(stages, args, dist, lambda st: st.run(mode=args.mode))  # seed None: OS entropy
    check_all("timed region: last run of every stage")
    steady = steady_state(stages, args, lambda st: st.run(mode=args.mode))
    if steady is not None:
        steady["ramp_and_drain_cost"] = dt_max / (args.steps * steady["ms_per_step"] * 1e-3) - 1.0
        check_all("steady-state steps")
    if args.mode == 1:
        # every run's batch verdict, graph replays included, as tallied on the device by the runs
        runs = len(stages) + args.warmup + args.steps + (steady["steps"] if steady else 0)
        acc = rej = 0
        for s_ in stages:
            a_, r_ = s_.run_tally()
            acc, rej = acc + a_, rej + r_
        if rej or acc != runs:
            raise SystemExit(f"batch verdicts over the bench: {acc} accepted, {rej} rejected of {runs} runs")
    # single-stream pass: step latency and per-kernel device times without overlap
    st = stages[0]
    st.kernel_times(args.mode, reset=True)
    single = []
    for s in range(args.single_steps):
        ts = time.perf_counter()
        st.run(mode=args.mode, timed=True)
        st.sync()
        single.append((time.perf_counter() - ts) * 1e3)
    kt = st.kernel_times(args.mode, reset=True)
    stats = st.msm_stats() if args.mode == 1 else None
    assert st.fetch()[0]
    for s_ in stages:
        s_.free()
    return {"dt": dt, "dt_max": dt_max, "single": single, "kt": kt, "stats": stats,
            "data": (pk, sg, msgs, offs, lens), "steady": steady}


def kernels_1k(eng, data, reps=20):
    """per-kernel device times of a resident 1,024-signature batch (single stream, HIP events)"""
    pk, sg, msgs, offs, lens = data
    n1 = 1024
    st = eng.stage(pk[:32 * n1], sg[:64 * n1], msgs, offs[:n1], lens[:n1])
    try:
        st.run(mode=1, timed=True)
        st.kernel_times(1, reset=True)
        for _ in range(reps):
            st.run(mode=1, timed=True)
        kt = st.kernel_times(1, reset=True)
        assert st.fetch()[0]
        return {"kernel_ms": kt, "sum_ms": sum(kt.values()), "msm_shape": st.msm_stats()}
    finally:
        st.free()


def latency_1k(eng, data, reps):
    """1,024-signature batch, host buffers in -> verdict out (H2D + D2H included)"""
    from narwhal_amd import _lib
    pk, sg, msgs, offs, lens = data
    n1 = 1024
    lat = []
    bitsbuf = np.zeros(n1 // 64 + 1, dtype=np.uint64)
    allv = _lib._i32(0)
    for r in range(reps + 5):
        t = time.perf_counter()
        rc = eng.lib.nwv_ed25519_verify_batch(eng._h, n1, pk.ctypes.data, sg.ctypes.data, msgs.ctypes.data,
                                              offs.ctypes.data, lens.ctypes.data, None, _lib.ctypes.byref(allv),
                                              bitsbuf.ctypes.data)
        if r >= 5:
            lat.append((time.perf_counter() - t) * 1e3)
        assert rc == 0 and allv.value == 1
    lat = np.array(lat)
    mlen = int(lens[:n1].max()) if n1 <= len(lens) else None
    return {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)), "reps": len(lat),
            "msg_len": mlen,
            "note": "the first 1,024 signatures of the headline batch (its message length); configs.C1."
                    "verify_batch_1024_m32 is the same call on configs[0]'s 32 B messages"}


def host_to_host(eng, data, threads, seconds):
    """host-resident batches verified end to end (pack + H2D + MSM + verdict D2H per call) by
    `threads` host threads on one context: the library's lanes overlap one call's copy with
    another's kernels.  This is the rate a verify_batch caller holding host buffers sees."""
    from narwhal_amd import _lib
    pk, sg, msgs, offs, lens = data
    n = len(offs)
    counts = [0] * threads
    stop = time.perf_counter() + seconds
    err = []

    def worker(k):
        allv = _lib._i32(0)
        while time.perf_counter() < stop:
            rc = eng.lib.nwv_ed25519_verify_batch(eng._h, n, pk.ctypes.data, sg.ctypes.data, msgs.ctypes.data,
                                                  offs.ctypes.data, lens.ctypes.data, None,
                                                  _lib.ctypes.byref(allv), None)
            if rc != 0 or allv.value != 1:
                err.append(rc)
                return
            counts[k] += 1

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    if err:
        raise SystemExit(f"host-to-host verification failed: {err}")
    calls = sum(counts)
    return {"sigs_per_s": calls * n / dt, "calls": calls, "threads": threads, "seconds": dt,
            "bytes_per_call_h2d": int(96 * n + int(lens.sum()) + 12 * n),
            "note": "nwv_ed25519_verify_batch on host buffers (65,536 x 512 B): pinned packing, H2D, "
                    "batch MSM, verdict D2H; PCIe Gen5 x16 (63 GB/s spec) bounds it"}


def firehose_subshard(m):
    """sub-shard size for a rank's m signatures: at most SUBSHARD (2M: the MSM's per-point cost
    flattens out there), and at least 4 sub-shards per rank, so that consecutive passes overlap
    one sub-shard's latency-bound tail with another's bulk kernels also at 8 GPUs (2M per rank).
    Env NWV_FIREHOSE_SUBSHARD overrides."""
    env = os.environ.get("NWV_FIREHOSE_SUBSHARD")
    if env:
        return max(64, int(env))
    return max(64, min(SUBSHARD, -(-m // 4) + 63 & ~63))


def firehose_pass(eng, lo, hi, reps, warm=1, dist=None):
    """verify [lo, hi) of the firehose as resident sub-shards (firehose_subshard) on their own
    streams: returns (seconds for `reps` passes, data, stages' kernel times)"""
    pk, sg, msgs, offs, lens = firehose_shard_data(eng, lo, hi)
    m = hi - lo
    subs = []
    sub = firehose_subshard(m)
    for a in range(0, m, sub):
        b = min(m, a + sub)
        subs.append(eng.stage(pk[32 * a:32 * b], sg[64 * a:64 * b], msgs, offs[a:b], lens[a:b]))
    for st in subs:
        for _ in range(warm):
            st.run(mode=1)
        allv, bits = st.fetch()
        if not (allv and bits.all()):
            raise SystemExit("firehose sub-shard of valid signatures rejected")
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        for st in subs:
            st.run(mode=1)
    for st in subs:
        st.sync()
    dt = time.perf_counter() - t0
    ok = True
    for st in subs:
        allv, bits = st.fetch()
        ok &= bool(allv and bits.all())
    if not ok:
        raise SystemExit("firehose pass of valid signatures rejected")
    subs[0].kernel_times(1, reset=True)
    subs[0].run(mode=1, timed=True)
    kt = subs[0].kernel_times(1, reset=True)
    firehose_pass.last_stats = subs[0].msm_stats()  # MSM shape of one sub-shard (roofline)
    firehose_pass.last_sub = subs[0].n
    for st in subs:
        st.free()
    return dt, (pk, sg, msgs, offs, lens), kt, len(subs)


def firehose_bad_set(eng, data, lo, hi, n_total, dist):
    """the exact-bad-set path of the firehose: seeded global indices corrupted, each rank verifies
    its shard as one batch (fallback only because it rejects), verdict bitmaps merged on the host
    (one all_gather over gloo); the merged bad set must equal the injected one"""
    from narwhal_amd import firehose as fh
    pk, sg, msgs, offs, lens = data
    rng = np.random.default_rng(4)
    bad = sorted(int(x) for x in rng.choice(n_total, size=64, replace=False))
    sg2 = sg.copy()
    for g in bad:
        if lo <= g < hi:
            sg2[64 * (g - lo) + 40] ^= 1
    verify = fh.gpu_shard_verifier(eng, pk, sg2, msgs, offs, lens)
    t0 = time.perf_counter()
    ok, words = fh.firehose(lambda a, b: verify(a - lo, b - lo), n_total, dist)
    dt = time.perf_counter() - t0
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n_total]
    got = np.flatnonzero(bits == 0).tolist()
    return {"injected": len(bad), "found": len(got), "exact": got == bad and not ok, "seconds": dt}


def run_firehose(args, eng, rank, world, dist):
    """configs[2]: 16,777,216 signatures over `world` ranks, one pass per step"""
    from narwhal_amd import firehose as fh
    import torch
    lo, hi = fh.shard_range(FIREHOSE_N, world, rank)
    dt, data, kt, nsub = firehose_pass(eng, lo, hi, args.steps, warm=1 + args.warmup, dist=dist)
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    badset = firehose_bad_set(eng, data, lo, hi, FIREHOSE_N, dist)
    o = torch.tensor([int(badset["exact"])], dtype=torch.int32)
    dist.all_reduce(o, op=dist.ReduceOp.MIN)
    if not o.item():
        raise SystemExit("firehose exact-bad-set check failed")
    if rank != 0:
        return None
    # rank 0's sub-shard MSM against the integer roofline (event-timed kernels of one sub-shard)
    sub_n = firehose_pass.last_sub
    per = kernel_rooflines(kt, firehose_pass.last_stats, sub_n, sub_n, valu_peak(), 32)
    roof = dict(per["k_msm_prep"], kernel="k_msm_prep", selected_by="largest VALU kernel of the bulk phase",
                kernel_share=per["k_msm_prep"]["kernel_ms"] / sum(kt.values()), subshard_sigs=sub_n)
    return {
        "workload": "configs[2]: firehose of 16,777,216 sigs (32 B messages) sharded by index over the "
                    "GPUs, host verdict-bitmap merge; strong scaling (the total is fixed)",
        "sigs_per_s": FIREHOSE_N * args.steps / dt, "passes": args.steps, "ms_per_pass": dt / args.steps * 1e3,
        "sigs_total": FIREHOSE_N, "sigs_per_gpu": hi - lo, "subshards_per_gpu": nsub,
        "parallelism": f"signature-index shards x{world}, no collective",
        "kernel_ms_rank0_subshard": kt,
        "roofline": roof,
        "roofline_per_kernel": per,
        "exact_bad_set": badset,
    }


def run_firehose_dry(args, rank, world, dist):
    """NWV_BENCH_DRYRUN=1 (CPU tests of the rank spawn and the verdict merge, no GPU): the same
    sharding, timing and gloo bitmap merge as run_firehose, with a shard verifier that rejects
    exactly the injected indices instead of the engine"""
    from narwhal_amd import firehose as fh
    import torch
    n_total = int(os.environ.get("NWV_BENCH_DRYRUN_N", "1048576"))
    lo, hi = fh.shard_range(n_total, world, rank)
    rng = np.random.default_rng(4)
    bad = sorted(int(x) for x in rng.choice(n_total, size=64, replace=False))

    def verify(a, b):
        v = np.ones(b - a, dtype=bool)
        for g in bad:
            if a <= g < b:
                v[g - a] = False
        w = np.zeros(((b - a + 63) // 64) * 8, dtype=np.uint8)
        pb = np.packbits(v, bitorder="little")
        w[:pb.size] = pb
        return bool(v.all()), w.view(np.uint64)

    dist.barrier()
    t0 = time.perf_counter()
    ok, words = fh.firehose(verify, n_total, dist)
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n_total]
    exact = np.flatnonzero(bits == 0).tolist() == bad and not ok
    if rank == 0:
        return {"workload": "firehose plumbing dry run (no GPU)", "sigs_per_s": n_total / float(t.item()),
                "sigs_total": n_total, "sigs_per_rank": hi - lo, "dry_run": True,
                "exact_bad_set": {"injected": len(bad), "exact": exact}}
    return None


def base_line(args, world, dt):
    """the contract's fields of the headline line: configs[1] on every rank, dt = max over ranks"""
    return {
        "metric": "Ed25519 sigs verified/sec",
        "value": world * args.n * args.steps / dt,
        "unit": "sigs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded keys/messages, RFC 8032 signatures made on the GPU)",
        "config": {"workload": "verify_batch of 65,536 valid sigs, 512 B messages, distinct keys "
                               "(BASELINE.json configs[1]) on every GPU",
                   "sigs_per_batch": args.n, "msg_len": args.msg_len,
                   "path": "batch MSM (K5)" if args.mode == 1 else "per-signature (K1-K4)",
                   "distinct_keys": args.keys or args.n,
                   "parallelism": "one GPU" if world == 1 else f"x{world} GPUs, one resident batch "
                                  "stream per rank, no collective",
                   "inflight_batches": args.inflight},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=192)
    ap.add_argument("--warmup", type=int, default=48)
    ap.add_argument("--n", type=int, default=65536, help="signatures per batch (N = 1 headline)")
    ap.add_argument("--msg-len", type=int, default=512)
    ap.add_argument("--mode", type=int, default=1, help="1 batch MSM (K5), 0 per-signature pipeline")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-reps", type=int, default=1000)
    ap.add_argument("--inflight", type=int, default=12,
                    help="resident batches in flight on separate streams (step s runs batch s %% K)")
    ap.add_argument("--keys", type=int, default=0,
                    help="distinct verifying keys (0: one per signature, the configs[1] worst case; "
                         "100: its committee variant, keyed batch MSM)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C1 / C3 / C4 / C5 legs (other BASELINE.json configs, GPU and CPU)")
    ap.add_argument("--steady-steps", type=int, default=96,
                    help="extra steps after the timed region that measure the steady-state rate (not `value`)")
    ap.add_argument("--single-steps", type=int, default=8,
                    help="single-stream steps timed after the run (step latency, per-kernel times)")
    ap.add_argument("--h2h-seconds", type=float, default=2.0)
    ap.add_argument("--headline-only", action="store_true",
                    help="only the timed headline steps (no 1K latency, host-to-host, configs or CPU baseline): "
                         "a rocprofv3 trace of this run is the headline alone")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, started before anything touches the GPU (never an exec)
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        procs = []
        for r in range(args.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                       LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                          stdout=None if r == 0 else sys.stderr))
        rcs = [p.wait() for p in procs]
        sys.exit(next((rc if rc > 0 else 1 for rc in rcs if rc != 0), 0))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    if os.environ.get("NWV_BENCH_ONE_DEVICE") == "1":
        local = 0  # rehearsal of the multi-rank path on a one-GPU box (ranks share device 0)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # host-side barrier / max / bitmap merge only: no data-path collective.  Gloo prints its
        # connection messages on fd 1; they go to stderr so stdout carries only the result line.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    if os.environ.get("NWV_BENCH_DRYRUN") == "1":
        if dist is None:
            raise SystemExit("NWV_BENCH_DRYRUN needs --gpus N > 1")
        h = run_headline_dry(args, rank, world, dist)
        fire = run_firehose_dry(args, rank, world, dist)
        if rank == 0:
            line = base_line(args, world, h["dt_max"])
            line.update(dry_run=True, firehose=fire)
            line["config"]["workload"] += " -- DRY RUN: host stand-in steps, no GPU"
            print(json.dumps(line), flush=True)
        dist.destroy_process_group()
        return

    import narwhal_amd

    eng = narwhal_amd.Engine(device=local)
    if world > 1:
        # the same configs[1] workload as N = 1 on every rank (weak scaling: value = all ranks'
        # signatures / the max-over-ranks time), then the configs[2] firehose as an extra field
        h = run_headline(args, eng, rank, world, dist)
        fire = run_firehose(args, eng, rank, world, dist)
        if rank == 0:
            line = base_line(args, world, h["dt_max"])
            line.update(rank0_ms_per_step=h["dt"] / args.steps * 1e3, kernel_ms_rank0=h["kt"],
                        single_stream_rank0={"ms_per_step": float(np.median(h["single"]))},
                        steady_state_rank0=h["steady"], firehose=fire,
                        # configs[2] at top level, labelled: the fixed 16M-signature total sharded by
                        # index over the ranks (strong scaling), beside the weak-scaling `value`
                        firehose_metric="configs[2] firehose: 16,777,216 sigs sharded by index, sigs/s",
                        firehose_sigs_per_s=fire["sigs_per_s"], firehose_scaling="strong",
                        firehose_exact_bad_set=fire["exact_bad_set"]["exact"])
            print(json.dumps(line), flush=True)
        eng.close()
        dist.destroy_process_group()
        return

    h = run_headline(args, eng, rank, world, dist)
    dt, kt, stats = h["dt"], h["kt"], h["stats"]
    value = args.n * args.steps / dt
    threads = usable_cpus()
    if args.headline_only:
        args.no_configs = args.no_cpu_baseline = True
        lat, h2h = None, None
    else:
        lat = latency_1k(eng, h["data"], args.latency_reps)
        lat["device_breakdown"] = kernels_1k(eng, h["data"]) if args.mode == 1 else None
        h2h = host_to_host(eng, h["data"], 4, args.h2h_seconds) if args.h2h_seconds > 0 else None
    peak = valu_peak()
    if args.mode == 1:
        na = args.keys or args.n
        per = kernel_rooflines(kt, stats, args.n, na, peak, args.msg_len)
        # the dominant kernel of the THROUGHPUT regime: the most VALU work (issue floor) -- with
        # batches in flight the latency-bound tail overlaps other batches' work; by single-stream
        # time when no PMC pass of today's kernels is committed for this size
        floors = {k: (v.get("issue_floor") or {}).get("floor_ms") for k, v in per.items() if v["bound"] == "valu"}
        if all(f is not None for f in floors.values()):
            dom, how = max(floors, key=floors.get), "largest VALU issue floor (committed PMC pass of HEAD's kernels)"
        else:
            dom, how = "k_msm_prep", "the bulk VALU kernel (no PMC pass of HEAD's kernels is committed)"
        roof = dict(per[dom], kernel=dom, selected_by=how,
                    kernel_share=per[dom]["kernel_ms"] / sum(kt.values()))
        # the kernel that takes the most single-stream device time (the MSM tail: one dependent
        # doubling chain per window, latency-bound) -- reported beside the throughput kernel
        tdom = max(per, key=lambda k: per[k]["kernel_ms"])
        roof["dominant_by_time"] = dict(per[tdom], kernel=tdom, kernel_share=per[tdom]["kernel_ms"] / sum(kt.values()))
        # the whole step against the chip's VALU issue rate: every kernel of the launch list, its
        # committed PMC instruction counts (64-bit forms at the v_mad_u64_u32 rate, the rest at
        # v_add_u32's) over the measured time per batch with batches in flight
        launch = list(kt)
        fl = issue_floor(launch, args.n, dt / args.steps * 1e3, peak, launch)
        if fl:
            fl["kernels"] = launch
            fl["note"] = ("VALU issue floor of one whole batch (every kernel of the launch list) against the "
                          "step time with batches in flight")
        roof["batch_issue_floor"] = fl
        # the kernel trace this line's kernel times can be checked against (committed, same sources)
        rp = rocprof_headline()
        roof["rocprof_source"] = rp["source"] if rp else None
        roof["rocprof_headline_inflight1"] = rp
        pmc_src = (roof.get("issue_floor") or {}).get("source")
        roof["pmc_source"] = pmc_src
    else:
        kms = kt.get("k_ed_straus", 0.0)
        m = (OPS_STRAUS[0] * MADS_PER_MUL + OPS_STRAUS[1] * MADS_PER_SQ) * args.n
        a = m / (kms * 1e-3) / 1e12 if kms else None
        pk_ = peak["v_mad_u64_u32_per_s"] / 1e12 if peak else None
        per = None
        roof = {"bound": "valu", "kernel": "k_ed_straus", "achieved": a, "peak": pk_, "unit": "T v_mad_u64_u32/s",
                "frac": a / pk_ if (a and pk_) else None, "traffic": None}
    cpu = None
    if not args.no_cpu_baseline:
        pk, sg, msgs, offs, lens = h["data"]
        cpu = cpu_baseline(pk, sg, msgs, offs, lens, args.cpu_seconds, threads)
    configs = None
    if not args.no_configs:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import config_legs as CL
        configs, cdata = {}, {}
        configs["C1"], cdata["C1"] = CL.leg_c1(eng)
        fdt, _, fkt, nsub = firehose_pass(eng, 0, FIREHOSE_N, 3)
        configs["C3"] = {"sigs": FIREHOSE_N, "gpus": 1, "subshards": nsub, "sigs_per_s": FIREHOSE_N * 3 / fdt,
                         "ms_per_pass": fdt / 3 * 1e3, "kernel_ms_subshard": fkt,
                         "note": "all of configs[2] on ONE GPU as 8 resident 2,097,152-signature sub-shards "
                                 "(the per-GPU share at 8 GPUs), 32 B messages; --gpus N shards it over N GPUs"}
        configs["C4"], cdata["C4"] = CL.leg_c4(eng)
        configs["C5"], cdata["C5"] = CL.leg_c5(eng)
        # the reference's default scheme, BLS12-381 (GPU legs, oracle checks, CPU baseline)
        configs["BLS"] = CL.leg_bls(eng, threads, cpu=not args.no_cpu_baseline, peak=peak)
        if not args.no_cpu_baseline:
            for k, v in cpu_baseline_configs(configs, cdata, threads).items():
                configs[k]["cpu_baseline"] = v
            c5 = configs["C5"]
            # a time ratio (> 1: the GPU is slower), named as one; every throughput ratio in the line
            # is a `*_speedup` (> 1: the GPU is faster)
            c5["worker_batch_digests_gpu_time_over_cpu_time"] = (
                c5["worker_batch_digests_ms_per_round"] / c5["cpu_baseline"]["worker_batch_digests_ms_per_round"])
        del cdata
    result = base_line(args, 1, dt)
    from narwhal_amd._lib import kernel_source_hash
    result.update({
        "kernel_source_hash": kernel_source_hash(),
        "steady_state": h["steady"],
        "single_stream": {"ms_per_step": float(np.median(h["single"])),
                          "sigs_per_s": args.n / (float(np.median(h["single"])) * 1e-3)},
        "latency_1k_batch_ms": lat,
        "host_to_host": h2h,
        "roofline": roof,
        "roofline_per_kernel": per,
        "kernel_ms": kt,
        "msm_shape": stats,
        "cpu_baseline": cpu,
        "configs": configs,
        "valu_ubench": peak,
    })
    print(json.dumps(result), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
