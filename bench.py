#!/usr/bin/env python3
"""bench.py -- Ed25519 signatures verified per second on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): verify_batch of 65,536 valid signatures over 512-byte
messages, distinct keys, synthetic (seeded keys and messages, signed on the GPU).  A "step" is
one batch verdict over one whole resident batch (inputs already in HBM): by default the batch
MSM (K5: k_msm_scalars -> k_msm_points -> counting sort -> buckets -> window sums -> Horner,
ed25519_consensus batch::Verifier semantics); --mode 0 runs the per-signature pipeline instead
(K1-K4, per-signature verdict bits whose AND is the batch verdict).  --inflight K keeps K
resident batches on K streams and issues the steps round-robin (a verification firehose: each
step still verifies one full 65,536-signature batch); the single-stream step time is reported
beside it.  With --gpus N the driver launches one rank per GPU (torch.distributed.run); each rank
verifies its own batches (weak scaling, signature-index sharding, no data-path collective: the
only exchange is the host-side max of the step times and the AND of verdicts over gloo).

Extra fields: roofline (VALU: 32x32->64 multiply-adds of the dominant bulk kernel vs the measured
v_mad_u64_u32 peak), cpu_baseline (the oracle's multi-threaded batch verifier on the host
cores, rank 0 only), p50/p99 latency of a 1,024-signature batch host->host, per-kernel times.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

# Hardware queues per process (HIP's default is 4).  Each resident batch runs on its own stream;
# with 4 queues the streams share queues and a batch's latency-bound MSM tail (window sums,
# Horner: a few workgroups for ~0.5 ms) serialises the work queued behind it.  16 queues let
# the tails of up to 16 batches run beside other batches' bulk kernels
# (profiles/round1_hwq_sweep.jsonl).  Must be set before the HIP runtime initialises; the GPU
# boxes export 4, so it is overridden here (NWV_BENCH_HW_QUEUES picks another count).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("NWV_BENCH_HW_QUEUES", "16")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic field operations per signature, counted on the host-emulation build
# (tests/test_hostemu.py::test_phase_op_counts and tests/test_msm_hostemu.py pin these
# numbers): (mul, sq) per phase.
OPS_POINTS = (111, 514)
OPS_STRAUS = (1505, 1020)
OPS_MSM_POINTS = (48, 514)  # k_msm_points: decompress R and A + affine Niels entries
MADS_PER_MUL, MADS_PER_SQ = 100, 55  # 10x10 and 55-term schoolbook, one v_mad_u64_u32 each


def mads(ops):
    return ops[0] * MADS_PER_MUL + ops[1] * MADS_PER_SQ


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    msgs = rng.integers(0, 256, size=n * mlen + 16, dtype=np.uint8)
    offs = np.arange(n, dtype=np.uint64) * mlen
    lens = np.full(n, mlen, dtype=np.uint32)
    pk, sg = eng.sign_many_arrays(seeds, msgs, offs, lens)
    return pk, sg, msgs, offs, lens


def cpu_baseline(pk, sg, msgs, offs, lens, seconds):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as of  # the checker; timed here as the CPU baseline only
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
    n = min(len(offs), 8192)
    done, t0 = 0, time.perf_counter()
    while True:
        ok = of.verify_batch_mt(pk[:32 * n].tobytes(), sg[:64 * n].tobytes(), msgs.tobytes(),
                                offs[:n].copy(), lens[:n].copy(), threads)
        assert ok, "CPU baseline rejected a valid batch"
        done += n
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "sigs/s", "cores": threads, "kind": "port",
            "sample": f"{done} sigs ({n}-sig batches of 512 B messages, {threads} threads, "
                      f"oracle/nwv_oracle.c batch verifier: Pippenger/Straus as dalek)"}


def cpu_baseline_configs(legs, data, threads):
    """CPU legs of C1 / C4 / C5 on the host cores (the oracle: dalek's algorithms in C, the
    reference's control flow in Python), and the check that the GPU's C4 verdict bits equal the
    oracle's per-signature verdicts"""
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
                 "verify_batch_1024_m32_ms": timed(lambda: of.verify_batch(c1["items"]), 20), "cores": 1}
    c4 = data["C4"]
    pk, sig, msg, offs, lens = of.pack(c4["items"])
    t = time.perf_counter()
    ok = of.verify_batch_mt(pk, sig, msg, offs, lens, threads)
    bits = of.verify_each_mt(pk, sig, msg, offs, lens, threads)
    dt = time.perf_counter() - t
    ref = [bool((int(bits[i >> 6]) >> (i & 63)) & 1) for i in range(len(offs))]
    out["C4"] = {"ms_per_batch": dt * 1e3, "sigs_per_s": len(offs) / dt, "cores": threads,
                 "batch_verdict": ok, "gpu_bits_equal_oracle": ref == list(c4["bits"])}
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
    out["C5"] = {"verify_ms_per_round": ms5, "verify_cores": 1,
                 "verify_sigs_per_s": legs["C5"]["signatures_per_round"] / (ms5 * 1e-3),
                 "worker_batch_digests_ms_per_round": msd, "digest_threads": threads}
    return out


def roofline_entry(kname, kt, mads_launch, peak_t, algorithmic, n):
    kms = float(kt.get(kname, 0.0))
    achieved = mads_launch / (kms * 1e-3) / 1e12 if kms > 0 else None
    traffic = pmc_traffic(kname, n)
    return {
        "bound": "valu",
        "kernel": kname,
        "achieved": achieved,
        "peak": peak_t,
        "unit": "T v_mad_u64_u32/s",
        "frac": (achieved / peak_t) if (peak_t and achieved) else None,
        "traffic": traffic["bytes"] if traffic else None,
        "traffic_source": traffic,
        "algorithmic": algorithmic,
    }


def split_prep_times(args, pk, sg, msgs, offs, lens, reps=5):
    """per-kernel times of the same batch with hashing and decompression as separate kernels"""
    import narwhal_amd
    from narwhal_amd import _lib
    e = narwhal_amd.Engine(device=0, flags=_lib.NWV_FLAG_MSM_SPLIT_PREP)
    try:
        if args.keys:
            kidx = (np.arange(args.n) % args.keys).astype(np.uint32)
            st = e.stage_keyed(pk[:32 * args.keys].copy(), kidx, sg, msgs, offs, lens)
        else:
            st = e.stage(pk, sg, msgs, offs, lens)
        st.run(mode=1, seed=b"\x11" * 32, timed=True)
        st.sync()
        st.kernel_times(1, reset=True)
        for r in range(reps):
            st.run(mode=1, seed=bytes([r + 1]) * 32, timed=True)
        kt = st.kernel_times(1, reset=True)
        assert st.fetch()[0]
        st.free()
        return kt
    finally:
        e.close()


def pmc_kernel(kernel, n):
    """(counters, source) of `kernel` in the newest committed rocprofv3 --pmc summary at batch
    size n, or (None, None)"""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(kernel)
        if d.get("n") == n and k:
            return k, os.path.relpath(f, ROOT)
    return None, None


def valu_issue_entry(kname, kt, n, peak):
    """VALU instruction throughput of `kernel`: SQ_INSTS_VALU per launch (wave-level
    instructions, committed PMC pass) over the live event-timed duration, against the
    full-rate 32-bit VALU issue peak measured on the box (v_add_u32 lane-ops/s / 64 lanes)."""
    insts, src = 0.0, None
    for part in kname.split("+"):  # "k_msm_bucket+fixup" is timed as one span
        k, src = pmc_kernel(part if part.startswith("k_") else "k_msm_" + part, n)
        if not k or "SQ_INSTS_VALU" not in k:
            return None
        insts += k["SQ_INSTS_VALU"]
    kms = float(kt.get(kname, 0.0))
    if not peak or kms <= 0:
        return None
    rate = insts / (kms * 1e-3) / 1e9
    pk = peak["v_add_u32_per_s"] / 64 / 1e9
    out = {"kernel": kname, "insts_per_launch": insts, "achieved": rate, "peak": pk,
           "unit": "G wave-VALU-instr/s", "frac": rate / pk, "source": src,
           "note": "frac prices every VALU instruction at the VOP2 rate (v_add_u32, a lower bound on "
                   "the busy fraction); frac_vop3 at the measured rate of 64-bit-encoded VOP3 forms "
                   "(v_mad_u64_u32 is one; so are v_alignbit_b32, v_lshl_add_u64, v_lshrrev_b64, "
                   "which issue at about half the VOP2 rate): an upper bound"}
    vop3 = [peak.get(k) for k in ("v_lshl_add_u64_per_s", "v_lshrrev_b64_per_s", "v_alignbit_b32_per_s")]
    if all(vop3):
        pk3 = sum(vop3) / len(vop3) / 64 / 1e9
        out["peak_vop3"] = pk3
        out["frac_vop3"] = rate / pk3
    return out


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc pass (FETCH_SIZE
    doubled for gfx950's half-counted wide reads + WRITE_SIZE, MI355X_MICROARCH.md HBM section),
    or None when no profile for it is committed."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
            k = d.get("kernels", {}).get(kernel)
            if d.get("n") != n:
                continue
            if k and "FETCH_SIZE" in k and "WRITE_SIZE" in k:
                return {"bytes": 2 * k["FETCH_SIZE"] * 1024 + k["WRITE_SIZE"] * 1024,
                        "source": os.path.relpath(f, ROOT), "n": d.get("n")}
        except (OSError, ValueError):
            continue
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=192)
    ap.add_argument("--warmup", type=int, default=48)
    ap.add_argument("--n", type=int, default=65536, help="signatures per batch (per GPU)")
    ap.add_argument("--msg-len", type=int, default=512)
    ap.add_argument("--mode", type=int, default=1, help="1 batch MSM (K5), 0 per-signature pipeline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-reps", type=int, default=1000)
    ap.add_argument("--inflight", type=int, default=12,
                    help="resident batches in flight on separate streams (step s runs batch s %% K)")
    ap.add_argument("--keys", type=int, default=0,
                    help="distinct verifying keys (0: one per signature, the configs[1] worst case; "
                         "100: its committee variant, keyed batch MSM)")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C1 / C4 / C5 legs (other BASELINE.json configs, GPU and CPU)")
    ap.add_argument("--single-steps", type=int, default=8,
                    help="single-stream steps timed after the run (step latency, per-kernel times)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("NWV_BENCH_ONE_DEVICE") == "1":
        local = 0  # rehearsal of the multi-rank path on a one-GPU box (ranks share device 0)
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        # host-side barrier / max only: no data-path collective.  Gloo prints its connection
        # messages on fd 1; they go to stderr so stdout carries only the result line.
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    import narwhal_amd
    from narwhal_amd import _lib

    eng = narwhal_amd.Engine(device=local)
    pk, sg, msgs, offs, lens = synth(eng, args.n, args.msg_len, seed=1000 + rank, keys=args.keys)
    if args.keys:
        kidx = np.arange(args.n, dtype=np.uint32) % np.uint32(args.keys)
        stages = [eng.stage_keyed(pk[:32 * args.keys].copy(), kidx, sg, msgs, offs, lens)
                  for _ in range(max(1, args.inflight))]
    else:
        stages = [eng.stage(pk, sg, msgs, offs, lens) for _ in range(max(1, args.inflight))]
    seed = lambda s_: (bytes([(s_ * 7 + rank) % 256]) * 32)

    def sync_all():
        for s_ in stages:
            s_.sync()

    for w in range(args.warmup):
        stages[w % len(stages)].run(mode=args.mode, seed=seed(w))
    sync_all()

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    sync_all()
    t0 = time.perf_counter()
    for s in range(args.steps):
        stages[s % len(stages)].run(mode=args.mode, seed=seed(s))
    sync_all()
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    ok = 1
    for s_ in stages:
        all_valid, bits = s_.fetch()
        ok &= int(bool(all_valid) and bool(bits.all()))
    # single-stream pass: step latency and per-kernel device times without overlap
    st = stages[0]
    st.kernel_times(args.mode, reset=True)
    single = []
    for s in range(args.single_steps):
        ts = time.perf_counter()
        st.run(mode=args.mode, seed=seed(1000 + s), timed=True)
        st.sync()
        single.append((time.perf_counter() - ts) * 1e3)
    kt = st.kernel_times(args.mode, reset=True)
    ok &= int(st.fetch()[0])
    if dist is not None:
        import torch
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        o = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
        ok = int(o.item())
    for s_ in stages:
        s_.free()
    if not ok:
        raise SystemExit("verification of a valid synthetic batch failed")

    total = world * args.n * args.steps
    value = total / dt
    result = None
    if rank == 0:
        # latency: 1,024-signature batch, host buffers in -> verdict out (H2D + D2H included)
        n1 = 1024
        lat = []
        pk1, sg1 = pk[:32 * n1], sg[:64 * n1]
        bitsbuf = np.zeros(n1 // 64 + 1, dtype=np.uint64)
        allv = _lib._i32(0)
        for r in range(args.latency_reps + 5):
            t = time.perf_counter()
            rc = eng.lib.nwv_ed25519_verify_batch(eng._h, n1, pk1.ctypes.data, sg1.ctypes.data,
                                                  msgs.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                                  b"\x05" * 32, _lib.ctypes.byref(allv), bitsbuf.ctypes.data)
            if r >= 5:
                lat.append((time.perf_counter() - t) * 1e3)
            assert rc == 0 and allv.value == 1
        lat = np.array(lat)
        peak = valu_peak()
        peak_t = (peak["v_mad_u64_u32_per_s"] / 1e12) if peak else None
        npts = args.n + (args.keys or args.n)  # decompressed points: R_i and the A points
        if args.mode == 1:
            # k_msm_prep = SHA-512 challenge hashing + decompression in one grid; only the
            # decompression's multiply-adds are counted (the hash is add/rotate work), so this
            # is a lower bound on the kernel's VALU use
            roof = roofline_entry("k_msm_prep", kt, mads(OPS_MSM_POINTS) // 2 * npts, peak_t,
                                  f"{mads(OPS_MSM_POINTS) // 2} multiply-adds/point (decompression: "
                                  f"{OPS_MSM_POINTS[0] // 2} mul x 100 + {OPS_MSM_POINTS[1] // 2} sq x 55) x "
                                  f"{npts} points per launch; the SHA-512 hashing in the same grid "
                                  "is not counted", args.n)
            roof["kernel_ms"] = kt
            roof["valu_issue"] = {kn: valu_issue_entry(kn, kt, args.n, peak)
                                  for kn in ("k_msm_prep", "k_msm_bucket+fixup")}
            kt_split = split_prep_times(args, pk, sg, msgs, offs, lens)
            roof["decompression_alone"] = roofline_entry(
                "k_msm_points", kt_split, mads(OPS_MSM_POINTS) // 2 * npts, peak_t,
                "same multiply-adds, k_msm_points launched on its own (NWV_FLAG_MSM_SPLIT_PREP, "
                "single stream, timed pass)", args.n)
            roof["decompression_alone"]["kernel_ms"] = kt_split
        else:
            roof = roofline_entry("k_ed_straus", kt, mads(OPS_STRAUS) * args.n, peak_t,
                                  f"{mads(OPS_STRAUS)} multiply-adds/signature ({OPS_STRAUS[0]} mul x 100 + "
                                  f"{OPS_STRAUS[1]} sq x 55) x {args.n} signatures per launch", args.n)
            roof["kernel_ms"] = kt
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(pk, sg, msgs, offs, lens, args.cpu_seconds)
        configs = None
        if not args.no_configs:
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import config_legs as CL
            configs, cdata = {}, {}
            configs["C1"], cdata["C1"] = CL.leg_c1(eng)
            configs["C4"], cdata["C4"] = CL.leg_c4(eng)
            configs["C5"], cdata["C5"] = CL.leg_c5(eng)
            if not args.no_cpu_baseline:
                threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)
                for k, v in cpu_baseline_configs(configs, cdata, threads).items():
                    configs[k]["cpu_baseline"] = v
            del cdata
        result = {
            "metric": "Ed25519 sigs verified/sec",
            "value": value,
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
                                   "(BASELINE.json configs[1]) per GPU",
                       "sigs_per_batch": args.n, "msg_len": args.msg_len,
                       "path": "batch MSM (K5)" if args.mode == 1 else "per-signature (K1-K4)",
                       "distinct_keys": args.keys or args.n,
                       "parallelism": f"signature-index shards x{world}",
                       "inflight_batches": len(stages)},
            "single_stream": {"ms_per_step": float(np.median(single)),
                              "sigs_per_s": args.n / (float(np.median(single)) * 1e-3) * world},
            "latency_1k_batch_ms": {"p50": float(np.percentile(lat, 50)),
                                    "p99": float(np.percentile(lat, 99)), "reps": len(lat)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "configs": configs,
            "valu_ubench": peak,
        }
        print(json.dumps(result), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
