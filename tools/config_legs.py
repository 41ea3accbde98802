"""GPU legs of BASELINE.json's other configs, measured beside the headline (bench.py --configs):

  C1  Certificate::verify of a 4-node committee (header signature + 3 votes), host -> host, and
      verify_batch of 1,024 random signatures over 32-byte messages (p50 / p99);
  C4  a 65,536-signature batch with 1 % adversarial entries: the batch MSM rejects, the
      per-signature pipeline returns the exact verdict bits (time per batch, bad set);
  C5  a 100-node committee DAG round: validate_certificates over 100 certificates (header
      signature + 67 votes each), Header::verify of the 100 headers, Vote::verify of 99 votes, and
      BLAKE2b-256 of the 100 worker batches (500,224 B each), streamed over many rounds.

Fixtures are built with the product only (GPU signer, GPU digests, nwv_certificate_new); the CPU
legs that time the oracle live in bench.py (cpu_baseline_configs)."""
import ctypes
import os
import hashlib
import time

import numpy as np

from narwhal_amd import _lib
from narwhal_amd import types as T

L_ORDER = 2**252 + 27742317777372353535851937790883648493


def _seed(tag, i):
    return hashlib.sha256(tag + i.to_bytes(4, "little")).digest()


def _pcts(xs):
    a = np.array(xs) * 1e3
    return {"p50_ms": float(np.percentile(a, 50)), "p99_ms": float(np.percentile(a, 99)), "reps": len(xs)}


def committee_fixture(eng, n, tag=b"nwv-bench-committee"):
    seeds = [_seed(tag, i) for i in range(n)]
    pk, _ = eng.sign_many(seeds, [b""] * n)
    keys = [pk[32 * i:32 * i + 32].tobytes() for i in range(n)]
    return seeds, keys, T.Committee(list(keys), [1] * n, 0, [[0, 1, 2, 3]] * n)


def worker_batch(author, n_tx=977, tx_len=512):
    """node/src/benchmark_client.rs:153-168 transactions: [tag u8][counter u64 BE][zero pad]"""
    out = bytearray()
    for c in range(n_tx):
        tx = bytearray(tx_len)
        tx[0] = 1 if c == 0 else 0  # sample transaction tag on the first one
        tx[1:9] = (author * 1_000_000 + c).to_bytes(8, "big")
        out += tx
    return bytes(out)


def dag_round(eng, seeds, keys, committee, payload_digests=None, parents=None):
    """one round: every authority's header (signed), the quorum's votes, the certificates"""
    n = len(keys)
    q = committee.quorum_threshold()
    if parents is None:
        parents = T.certificate_digests(eng, T.Certificate.genesis(committee))
    headers = []
    for a in range(n):
        pay = [(payload_digests[a], a % 4)] if payload_digests else []
        headers.append(T.Header(author=keys[a], round=1, epoch=0, payload=pay, parents=list(parents)))
    for h, d in zip(headers, T.header_digests(eng, headers)):
        h.id = d
    _, hs = eng.sign_many(seeds, [h.id for h in headers])
    for a, h in enumerate(headers):
        h.signature = hs[64 * a:64 * a + 64].tobytes()
    voters = [[i for i in range(n) if i != a][:q] for a in range(n)]
    votes = [T.Vote(headers[a].id, 1, 0, keys[a], keys[v]) for a in range(n) for v in voters[a]]
    vd = T.vote_digests(eng, votes)
    vseeds = [seeds[v] for a in range(n) for v in voters[a]]
    _, vs = eng.sign_many(vseeds, vd)
    for k, v in enumerate(votes):
        v.signature = vs[64 * k:64 * k + 64].tobytes()
    certs = []
    for a in range(n):
        vv = votes[a * q:(a + 1) * q]
        certs.append(T.Certificate.new(committee, headers[a], [(v.author, v.signature) for v in vv]))
    return headers, votes, certs


def leg_c1(eng, reps=1000):
    seeds, keys, com = committee_fixture(eng, 4, b"nwv-bench-c1")
    headers, votes, certs = dag_round(eng, seeds, keys, com)
    cert = certs[-1]
    T.verify(eng, com, cert)  # raises on any DagError
    keep = T._Keep()
    cc = com._c(keep)
    carr = (T._Certificate * 1)(cert._c(keep))
    res = (ctypes.c_int32 * 1)()
    lib = T.lib()
    lat = []
    for r in range(reps + 5):
        t = time.perf_counter()
        rc = lib.nwv_certificate_verify_many(eng._h, ctypes.byref(cc), 1, carr, res)
        if r >= 5:
            lat.append(time.perf_counter() - t)
        assert rc == 0 and res[0] == 0
    # verify_batch of 1,024 random signatures, 32-byte messages, distinct keys
    rng = np.random.default_rng(11)
    n = 1024
    bseeds = [rng.bytes(32) for _ in range(n)]
    msgs = [rng.bytes(32) for _ in range(n)]
    pk, sg = eng.sign_many(bseeds, msgs)
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    apk, asg, arena, offs, lens = _lib.soa(items)
    allv = _lib._i32(0)
    blat = []
    for r in range(reps + 5):
        t = time.perf_counter()
        _lib._check(eng.lib.nwv_ed25519_verify_batch(eng._h, n, _lib._ptr(apk), _lib._ptr(asg), _lib._ptr(arena),
                                                     _lib._ptr(offs), _lib._ptr(lens), bytes([r % 256]) * 32,
                                                     ctypes.byref(allv), None))
        assert allv.value == 1
        if r >= 5:
            blat.append(time.perf_counter() - t)
    return {"certificate_verify_n4": _pcts(lat), "verify_batch_1024_m32": _pcts(blat)}, \
        {"committee": com, "cert": cert, "items": items}


def _golden_adversarial():
    """every non-honest category of the committed fixtures (B1-B8, built and
    pinned by oracle/gen_golden.py) and the 196-case ZIP-215 small-order table, as
    {category: [(pk, sig, msg, expected verdict)]}"""
    import json
    import os
    gdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")
    out = {}
    with open(os.path.join(gdir, "ed25519_vectors.json")) as f:
        for v in json.load(f)["vectors"]:
            if v["category"] != "honest":
                out.setdefault(v["category"], []).append(
                    (bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]), bool(v["expect"])))
    with open(os.path.join(gdir, "zip215_small_order.json")) as f:
        for v in json.load(f)["vectors"]:
            out.setdefault("B5_zip215_table", []).append(
                (bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"]), bool(v["expect"])))
    return out


# categories applied to the batch's own honest entries (512-byte messages)
INPLACE = ("B1_flip_R_inplace", "B1_flip_s_inplace", "B1_flip_msg_inplace", "B2_s_plus_l_inplace",
           "B5_identity_A_R_s0_inplace")


def adversarial_batch(eng, n=65536, frac=0.01, seed=4, mlen=512):
    """C4: n honest signatures over mlen-byte messages, frac of them replaced at seeded positions
    by adversarial entries, the categories taken in turn: bit-flipped R / s / message, s + l, the
    identity A = R with s = 0 (accepted by the cofactored equation), and every Appendix-B category
    of the golden fixtures (non-canonical R / A, small-order and mixed-order A / R, undecodable R /
    A, negative zero, with the entries that the cofactored equation accepts and rejects).
    Returns (items, positions, categories, expected bad indices by construction)."""
    rng = np.random.default_rng(seed)
    seeds = [rng.bytes(32) for _ in range(n)]
    msgs = [rng.bytes(mlen) for _ in range(n)]
    pk, sg = eng.sign_many(seeds, msgs)
    pk, sg = pk.copy(), sg.copy()
    pos = np.sort(rng.choice(n, size=int(n * frac), replace=False))
    gold = _golden_adversarial()
    cats = list(INPLACE) + sorted(gold)
    ident = np.zeros(32, dtype=np.uint8)
    ident[0] = 1
    items = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    used, expect_bad, turn = [], [], {}
    for j, i in enumerate(pos):
        i = int(i)
        c = cats[j % len(cats)]
        used.append(c)
        p, s, m = items[i]
        if c in gold:
            k = turn.get(c, 0)
            turn[c] = k + 1
            p, s, m, ok = gold[c][k % len(gold[c])]
        else:
            s = bytearray(s)
            ok = False
            if c == "B1_flip_R_inplace":
                s[3] ^= 0x10
            elif c == "B1_flip_s_inplace":
                s[40] ^= 0x01
            elif c == "B1_flip_msg_inplace":
                m = bytes([m[0] ^ 0x80]) + m[1:]
            elif c == "B2_s_plus_l_inplace":
                v = int.from_bytes(bytes(s[32:]), "little") + L_ORDER
                s[32:] = v.to_bytes(32, "little")
            else:
                p = ident.tobytes()
                s = bytearray(ident.tobytes() + bytes(32))
                ok = True
            s = bytes(s)
        items[i] = (p, s, m)
        if not ok:
            expect_bad.append(i)
    return items, [int(i) for i in pos], used, expect_bad


def leg_c4(eng, reps=5):
    """host arrays already packed (as a Rust caller holds them): the timed region is the C call,
    H2D + batch MSM + per-signature fallback + D2H"""
    items, pos, cats, expect_bad = adversarial_batch(eng)
    n = len(items)
    pk, sig, arena, offs, lens = _lib.soa(items)
    bitsbuf = np.zeros((n + 63) // 64 + 1, dtype=np.uint64)
    allv = _lib._i32(0)
    ts = []
    for r in range(reps + 1):
        t = time.perf_counter()
        _lib._check(eng.lib.nwv_ed25519_verify_batch(eng._h, n, _lib._ptr(pk), _lib._ptr(sig), _lib._ptr(arena),
                                                     _lib._ptr(offs), _lib._ptr(lens), bytes([r + 1]) * 32,
                                                     ctypes.byref(allv), _lib._ptr(bitsbuf)))
        if r >= 1:
            ts.append(time.perf_counter() - t)
    ok = bool(allv.value)
    bits = list(_lib.unpack_bits(bitsbuf, n))
    bad = [i for i, b in enumerate(bits) if not b]
    med = float(np.median(ts))
    return {"n": n, "adversarial": len(pos), "categories": len(set(cats)), "batch_verdict": ok, "bad": len(bad),
            "bad_set_equals_injected": bad == expect_bad, "ms_per_batch_host_to_host": med * 1e3,
            "sigs_per_s": n / med}, {"items": items, "pos": pos, "bits": bits}


def leg_c5_service(eng, com, cc, harr, varr, carr, nsig, rounds=20):
    """C5 the way a Core loop would run it (primary/src/core.rs:614-714): ONE
    consumer thread takes messages off a queue (Core's channels) with the drain pattern of
    narwhal_amd.service.CoreDrain / rust core_drain.rs -- on a message, take whatever else is
    queued (<= 512 messages, <= 1 ms) and verify the lot with one nwv_verify_mixed_many call -- while
    a producer thread delivers each round's 299 messages (the network).  Reports the round time,
    per-message latency (enqueue -> own verdict), flush sizes; then the same messages through the
    in-library service with asynchronous submission, and one engine call per message."""
    import queue
    import threading
    from narwhal_amd import service as S
    lib = S.bind(T.lib())
    msgs = [("header", harr[i]) for i in range(len(harr))] + [("vote", varr[i]) for i in range(len(varr))] + \
           [("certificate", carr[i]) for i in range(len(carr))]
    out = {"messages_per_round": len(msgs), "rounds": rounds}
    drain = S.CoreDrain(eng, com, max_items=512, max_wait_us=1000, min_items=64)
    q = queue.Queue()
    lat, rtimes, sizes = [], [], []

    stop = []

    def producer(r0):
        for r in range(r0):
            go.wait()
            go.clear()
            if stop:
                return
            t = time.perf_counter()
            for i, m in enumerate(msgs):
                q.put((t, i, m))

    go = threading.Event()
    th = threading.Thread(target=producer, args=(rounds + 1,))
    th.start()
    try:
        for r in range(rounds + 1):
            go.set()
            t0 = time.perf_counter()
            seen = 0
            while seen < len(msgs):
                batch = drain.drain(q)
                codes = drain.verify([m for _, _, m in batch])
                t1 = time.perf_counter()
                assert not any(codes), codes[:8]
                seen += len(batch)
                if r:
                    sizes.append(len(batch))
                    lat += [t1 - te for te, _, _ in batch]
            if r:  # the first round warms up
                rtimes.append(time.perf_counter() - t0)
    finally:
        stop.append(1)
        go.set()
        th.join()
    a = np.array(lat) * 1e3
    out.update({"consumer": "one thread, CoreDrain(max_items=512, max_wait_us=1000, min_items=64)",
                "ms_per_round": float(np.median(rtimes)) * 1e3, "sigs_per_s": nsig / float(np.median(rtimes)),
                "latency_ms_p50": float(np.percentile(a, 50)), "latency_ms_p99": float(np.percentile(a, 99)),
                "engine_calls": len(sizes), "largest_flush": int(max(sizes)),
                "mean_flush": float(np.mean(sizes))})
    # asynchronous submission: one thread submits a whole round's messages (a Core loop that
    # hands every message to the service instead of verifying it inline), each completion
    # callback records its latency; the service coalesces the round into one or two engine calls
    h2 = ctypes.c_void_p()
    _lib._check(lib.nwv_service_create(eng._h, ctypes.byref(cc), 512, 200, ctypes.byref(h2)))
    sub_fns = [lib.nwv_service_submit_header] * len(harr) + [lib.nwv_service_submit_vote] * len(varr) + \
              [lib.nwv_service_submit_certificate] * len(carr)
    structs = [harr[i] for i in range(len(harr))] + [varr[i] for i in range(len(varr))] + \
              [carr[i] for i in range(len(carr))]
    t_sub = np.zeros(len(structs))
    t_done = np.zeros(len(structs))
    codes = np.zeros(len(structs), dtype=np.int32)
    ev = threading.Event()
    left = [0]
    lk = threading.Lock()

    def on_done(user, code):
        i = user or 0
        t_done[i] = time.perf_counter()
        codes[i] = code
        with lk:
            left[0] -= 1
            if left[0] == 0:
                ev.set()

    cb = S.DONE_FN(on_done)
    lat2, rtimes = [], []
    try:
        for r in range(rounds + 1):
            ev.clear()
            left[0] = len(structs)
            t0 = time.perf_counter()
            for i, (fn, st) in enumerate(zip(sub_fns, structs)):
                t_sub[i] = time.perf_counter()
                _lib._check(fn(h2, ctypes.byref(st), cb, ctypes.c_void_p(i)))
            ev.wait(30)
            if r:  # the first round warms up
                rtimes.append(time.perf_counter() - t0)
                lat2.append(t_done - t_sub)
            assert not codes.any()
        stats2 = np.zeros(6, dtype=np.uint64)
        lib.nwv_service_stats(h2, stats2.ctypes.data)
    finally:
        lib.nwv_service_free(h2)
    a2 = np.concatenate(lat2) * 1e3
    out["async_submit"] = {"latency_ms_p50": float(np.percentile(a2, 50)), "latency_ms_p99": float(np.percentile(a2, 99)),
                           "ms_per_round": float(np.median(rtimes)) * 1e3,
                           "sigs_per_s": nsig / float(np.median(rtimes)),
                           "engine_calls": int(stats2[0]), "items": int(stats2[1]), "largest_batch": int(stats2[2])}
    try:  # bench tooling (tools/libsvcbench.so, built by `make tools`): its absence costs only this field
        out["native"] = leg_c5_service_native(eng, cc, harr, varr, carr, nsig, rounds)
    except OSError as e:
        out["native"] = {"error": str(e)}
    # the same messages, one engine call per message, serially (the reference's Core loop shape)
    tl = T.lib()
    one = []
    r = ctypes.c_int32(0)
    for fn_many, arr in ((tl.nwv_header_verify_many, harr), (tl.nwv_vote_verify_many, varr),
                         (tl.nwv_certificate_verify_many, carr)):
        for i in range(len(arr)):
            t1 = time.perf_counter()
            assert fn_many(eng._h, ctypes.byref(cc), 1, ctypes.byref(arr[i]), ctypes.byref(r)) == 0 and r.value == 0
            one.append(time.perf_counter() - t1)
    out["one_call_per_message"] = {"latency_ms_p50": float(np.median(one)) * 1e3,
                                   "ms_per_round": float(np.sum(one)) * 1e3}
    return out


def _svcbench():
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "libsvcbench.so")
    lib = ctypes.CDLL(path)
    vp, sz, i32, u32, dp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p
    lib.svcbench_service.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, i32, i32, sz, u32, u32, dp, dp, dp, dp]
    lib.svcbench_drain.argtypes = [vp, vp, sz, vp, sz, vp, sz, vp, i32, sz, u32, sz, u32, dp, dp, dp, dp]
    return lib


def leg_c5_service_native(eng, cc, harr, varr, carr, nsig, rounds=20):
    """The C5 service leg driven from C++ threads (tools/svcbench.cpp), as a Rust Core would run it
    (rust/narwhal-gpu-crypto/src/core_drain.rs): no Python queue, no ctypes call per message.
    'drain_idle*': a producer thread delivers the round's 299 messages one at a time into a channel
    and ONE consumer drains and verifies (CoreDrain's pattern, max_items 512, max_wait 1000 us,
    min_items 64; idle_us 50: past min_items wait up to 50 us for each next message);
    'service_k_idle*': k threads submit the round to nwv_service asynchronously (idle 50: the
    burst flush, nwv_service_set_idle)."""
    sb = _svcbench()
    n = len(harr) + len(varr) + len(carr)
    args = (eng._h, ctypes.byref(cc), len(harr), ctypes.cast(harr, ctypes.c_void_p), len(varr),
            ctypes.cast(varr, ctypes.c_void_p), len(carr), ctypes.cast(carr, ctypes.c_void_p))
    out = {"messages_per_round": n, "rounds": rounds}
    rt = np.zeros(rounds)
    lat = np.zeros(rounds * n)
    calls = np.zeros(rounds, dtype=np.uint32)
    big = np.zeros(rounds, dtype=np.uint32)
    for idle in (0, 50):
        rc = sb.svcbench_drain(*args, rounds, 512, 1000, 64, idle, rt.ctypes.data, lat.ctypes.data, calls.ctypes.data,
                               big.ctypes.data)
        assert rc == 0, rc
        out[f"drain_idle{idle}"] = {
            "max_items": 512, "max_wait_us": 1000, "min_items": 64, "idle_us": idle,
            "ms_per_round": float(np.median(rt)), "sigs_per_s": nsig / (float(np.median(rt)) * 1e-3),
            "latency_ms_p50": float(np.percentile(lat, 50)), "latency_ms_p99": float(np.percentile(lat, 99)),
            "engine_calls_per_round": float(np.mean(calls)), "largest_flush": int(big.max())}
    for k, wait, idle in ((1, 200, 0), (8, 200, 0), (1, 1000, 50), (8, 1000, 50)):
        st = np.zeros(6, dtype=np.uint64)
        sub = np.zeros(rounds)
        rc = sb.svcbench_service(*args, k, rounds, 512, wait, idle, rt.ctypes.data, sub.ctypes.data, lat.ctypes.data,
                                 st.ctypes.data)
        assert rc == 0, rc
        out[f"service_{k}_idle{idle}"] = {
            "submitter_threads": k, "max_batch": 512, "max_wait_us": wait, "idle_us": idle,
            "ms_per_round": float(np.median(rt)), "sigs_per_s": nsig / (float(np.median(rt)) * 1e-3),
            "submit_ms_per_round": float(np.median(sub)),
            "latency_ms_p50": float(np.percentile(lat, 50)), "latency_ms_p99": float(np.percentile(lat, 99)),
            "engine_calls_per_round": float(st[0]) / (rounds + 1), "largest_batch": int(st[2])}
    return out


def leg_c5(eng, rounds=50):
    seeds, keys, com = committee_fixture(eng, 100, b"nwv-bench-c5")
    batches = [worker_batch(a) for a in range(100)]
    pd = eng.blake2b256_many(batches)
    headers, votes, certs = dag_round(eng, seeds, keys, com, payload_digests=pd)
    vsample = votes[:99]
    # the C structs are built once (a Rust caller passes its own objects by pointer); the timed
    # region is the three C calls and the digest call, each host -> host
    ok, bad = T.validate_certificates(eng, com, certs)
    assert ok and not bad and not any(T.verify_headers(eng, com, headers)) and not any(T.verify_votes(eng, com, vsample))
    keep = T._Keep()
    cc = com._c(keep)
    carr = (T._Certificate * len(certs))(*[c._c(keep) for c in certs])
    harr = (T._Header * len(headers))(*[h._c(keep) for h in headers])
    varr = (T._Vote * len(vsample))(*[v._c(keep) for v in vsample])
    hres = (ctypes.c_int32 * len(headers))()
    vres = (ctypes.c_int32 * len(vsample))()
    nbad = ctypes.c_size_t(0)
    idx = (ctypes.c_size_t * len(certs))()
    lib = T.lib()
    blens = np.array([len(b) for b in batches], dtype=np.uint64)
    boffs = np.zeros(len(batches), dtype=np.uint64)
    boffs[1:] = np.cumsum(blens[:-1], dtype=np.uint64)
    barena = np.frombuffer(b"".join(batches) + bytes(16), dtype=np.uint8)
    bout = np.zeros(32 * len(batches), dtype=np.uint8)
    cres = (ctypes.c_int32 * len(certs))()
    t_sig, t_dig, t_mix = [], [], []
    for r in range(rounds + 2):
        t0 = time.perf_counter()
        rc = lib.nwv_validate_certificates(eng._h, ctypes.byref(cc), len(certs), carr, ctypes.byref(nbad), idx)
        rh = lib.nwv_header_verify_many(eng._h, ctypes.byref(cc), len(headers), harr, hres)
        rv = lib.nwv_vote_verify_many(eng._h, ctypes.byref(cc), len(vsample), varr, vres)
        t1 = time.perf_counter()
        rb = eng.lib.nwv_blake2b256_many(eng._h, len(batches), _lib._ptr(barena), _lib._ptr(boffs),
                                         _lib._ptr(blens), _lib._ptr(bout))
        t2 = time.perf_counter()
        d = [bout[32 * i:32 * i + 32].tobytes() for i in range(len(batches))]
        assert rc == rh == rv == rb == 0 and nbad.value == 0 and not any(hres) and not any(vres) and d == pd
        # the same round as ONE coalesced call (Core::sanitize_* batched): one digest launch,
        # one batch MSM for all 6,999 signatures
        t3 = time.perf_counter()
        rm = lib.nwv_verify_mixed_many(eng._h, ctypes.byref(cc), len(headers), harr, hres, len(vsample), varr, vres,
                                       len(certs), carr, cres)
        t4 = time.perf_counter()
        assert rm == 0 and not any(hres) and not any(vres) and not any(cres)
        if r >= 2:
            t_sig.append(t1 - t0)
            t_dig.append(t2 - t1)
            t_mix.append(t4 - t3)
    nsig = sum(1 + len(c.aggregated_signature) for c in certs) + len(headers) + len(vsample)
    svc = leg_c5_service(eng, com, cc, harr, varr, carr, nsig)
    ms = float(np.median(t_sig)) * 1e3
    return {"rounds": rounds, "signatures_per_round": nsig,
            "verify_ms_per_round": ms, "verify_sigs_per_s": nsig / (ms * 1e-3),
            "verify_coalesced_ms_per_round": float(np.median(t_mix)) * 1e3,
            "verify_coalesced_sigs_per_s": nsig / float(np.median(t_mix)),
            "worker_batch_digests_ms_per_round": float(np.median(t_dig)) * 1e3,
            "service": svc,
            "note": "one round = validate_certificates(100 certs x (1 + 67) sigs) + 100 Header::verify + "
                    "99 Vote::verify (three C calls on prepared structs, host -> host; 'coalesced': the same round as one "
                    "nwv_verify_mixed_many call) and BLAKE2b-256 of 100 x 500,224 B "
                    "worker batches (one GPU call)"}, \
        {"committee": com, "certs": certs, "headers": headers, "votes": vsample, "batches": batches}


def _bls_committee(b, n, rnd):
    r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001
    sks = [(int.from_bytes(rnd.bytes(32), "big") % r or 1).to_bytes(32, "big") for _ in range(n)]
    return sks, b.keygen(sks)


def _bls_round_items(b, sks, rnd, certs, quorum):
    """`certs` certificates of the committee: each an aggregate of `quorum` signatures over its
    32-byte digest (made on the GPU) -> (aggregates, signer lists, digests)"""
    committee = len(sks)
    digests = [rnd.bytes(32) for _ in range(certs)]
    signers = [sorted(rnd.choice(committee, quorum, replace=False).tolist()) for _ in range(certs)]
    flat = b.sign([sks[k] for s in signers for k in s], [d for d, s in zip(digests, signers) for _ in s])
    aggs = []
    for c in range(certs):
        rc, agg, _ = b.aggregate(flat[quorum * c:quorum * (c + 1)])
        assert rc == 0
        aggs.append(agg)
    return aggs, signers, digests


def bls_pairing_products(fixed_lines=True):
    """Fp products of one pairing check on the wave engine (narwhal_amd/csrc/bls_wave.h
    pairing_check + final_exp, the program counts tools/gen_bls_wave.py writes to
    bls_wave_counts.json; multiplications by one of combination lanes not counted), and the
    v_mad_u64_u32 of one product (14 x 14 limb products + 14 reduction rows of 14)"""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "narwhal_amd", "csrc",
                           "bls_wave_counts.json")) as f:
        meta = json.load(f)
    pc = {k: v["products"] for k, v in meta["programs"].items()}
    kind = "fixed" if fixed_lines else "step"
    ml = sum(pc[f"ml_{'add' if c == 'a' else 'dbl'}_{kind}"] for c in meta["steps"])
    xbits = bin(meta["x_abs"])[3:]  # below the top bit
    exp_x = len(xbits) * pc["cyc_sqr_F"]
    fe = (pc["inv_a"] + pc["inv_b"] + pc["easy1"] + pc["easy2"] + 5 * exp_x
          + xbits.count("1") * (pc["mul_F_M"] + 2 * pc["mul_F_A"] + pc["mul_F_B"] + pc["mul_F_C"])
          + pc["mulconj_F_M"] + pc["mulconj_F_A"] + pc["conjmulfrob_F_A"] + pc["conjmulfrob2_F_B"]
          + pc["mulconj2_F_B"] + pc["cycsqr_M_to_G"] + pc["mul_G_M"] + pc["mul_F_G"])
    return {"miller_loop": ml, "final_exp": fe, "total": ml + fe, "mads_per_product": meta["mads_per_product"]}


def bls_pmc(n_items, kernel="k_blsw_pair"):
    """(counters, source) of `kernel` from the newest committed BLS rocprofv3 --pmc summary
    (tools/gpurun/r4_bls_prof.sh -> profiles/*bls_pmc*.json) whose bls_source_hash is HEAD's and
    whose size is n_items; else (None, None)"""
    import glob
    import json
    import os
    from narwhal_amd._lib import bls_source_hash
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    want = bls_source_hash()
    for f in sorted(glob.glob(os.path.join(root, "profiles", "*bls_pmc*.json")), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        if d.get("n") == n_items and d.get("bls_source_hash") == want and kernel in d.get("kernels", {}):
            return d["kernels"][kernel], os.path.relpath(f, root)
    return None, None


def bls_pack():
    """items per pairing wave of large calls (nwv_bls.hip: NWV_BLS_PACK, default 3, 1..4)"""
    import os
    try:
        v = int(os.environ.get("NWV_BLS_PACK", "3"))
    except ValueError:
        v = 3
    return min(4, max(1, v))


def bls_roofline(n_items, pairing_ms, peak, fixed_lines=True):
    """the dominant BLS kernel (k_blsw_pair_k: the pairing checks, bls_pack() items per wave; with
    NWV_BLS_PACK=1 k_blsw_pair, one per wave) against the measured v_mad_u64_u32 rate; with a
    committed PMC pass of HEAD's BLS sources also its VALU issue floor (instructions at the
    measured rates) and HBM traffic"""
    mad_peak_ts = (peak["v_mad_u64_u32_per_s"] / 1e12) if peak else None
    c = bls_pairing_products(fixed_lines)
    mads = c["total"] * c["mads_per_product"] * n_items
    a = mads / (pairing_ms * 1e-3) / 1e12 if pairing_ms > 0 else None
    kernel = "k_blsw_pair_k" if bls_pack() > 1 else "k_blsw_pair"
    pmc, src = bls_pmc(n_items, kernel)
    floor = traffic = None
    if pmc and peak and "SQ_INSTS_VALU" in pmc and "SQ_INSTS_VALU_INT64" in pmc and pairing_ms > 0:
        v, i64 = pmc["SQ_INSTS_VALU"], pmc["SQ_INSTS_VALU_INT64"]
        fs = i64 * 64 / peak["v_mad_u64_u32_per_s"] + (v - i64) * 64 / peak["v_add_u32_per_s"]
        floor = {"valu_insts_per_launch": v, "int64_insts": i64, "floor_ms": fs * 1e3, "frac": fs / (pairing_ms * 1e-3),
                 "source": src}
    if pmc and "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        traffic = 2 * pmc["FETCH_SIZE"] * 1024 + pmc["WRITE_SIZE"] * 1024
    return {"kernel": kernel, "items_per_wave": bls_pack(), "bound": "valu", "achieved": a, "unit": "T v_mad_u64_u32/s",
            "peak": mad_peak_ts, "frac": (a / mad_peak_ts) if (a and mad_peak_ts) else None, "kernel_ms": pairing_ms,
            "mads_per_launch": mads, "items": n_items, "issue_floor": floor, "traffic": traffic,
            "pmc_source": src,
            "algorithmic": f"{c['total']} Fp products per pairing check ({c['miller_loop']} Miller loop with "
                           f"{'precomputed' if fixed_lines else 'computed'} key lines, {c['final_exp']} final "
                           f"exponentiation; tools/gen_bls_wave.py counts) x {c['mads_per_product']} multiply-adds x "
                           f"{n_items} items"}


def leg_bls(eng, threads=1, certs=100, quorum=67, committee=100, reps=20, throughput_n=16384, single_reps=200,
            dag_rounds=20, concurrency=8, cpu=True, peak=None):
    """SURVEY §8 row f4, the reference's default scheme (crypto/src/lib.rs:29-33 -> BLS12-381
    min_sig), host -> host, synthetic keys / messages (signatures and aggregates made on the GPU),
    the committee registered in the key cache (epoch start):
      round       `certs` certificates x `quorum` signers of a `committee`-key committee, ONE
                  nwv_bls_verify_many call (CertificatesResponse::validate_certificates; item =
                  AggregateAuthenticator::verify = fast_aggregate_verify)
      single      one Verifier::verify (Header::verify / Vote::verify's check) p50 / p99
      concurrent  `concurrency` threads issuing single verifies at once vs one thread
      throughput  `throughput_n` single-key items in one call
      dag_round   the C5 shape under BLS: 100 headers + 99 votes + 100 certificates through ONE
                  nwv_bls_verify_mixed_many call (types layer: digests + every signature check)
    Statuses are checked against the oracle (oracle/bls_oracle.c, keys validated once per call as
    fastcrypto validates a key at deserialization); the CPU baseline times that oracle on the host
    cores over the same round (kind: port)."""
    import sys
    import threading
    sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
        __import__("os").path.abspath(__file__))), "tests"))
    from narwhal_amd.bls import Bls
    b = Bls(eng)
    rnd = np.random.default_rng(77)
    sks, pks = _bls_committee(b, committee, rnd)
    b.register_keys(pks)
    aggs, signers, digests = _bls_round_items(b, sks, rnd, certs, quorum)
    # the C call on prepared arrays, as a Rust caller holds them (packing the round's lists in
    # Python is ~0.35 ms of interpreter time on its own)
    from narwhal_amd import bls as BL
    r_keys, r_sigs = BL._arr(b"".join(pks)), BL._arr(b"".join(aggs))
    r_cnt = np.array([len(k) for k in signers], dtype=np.uint32)
    r_off = np.zeros(len(signers), dtype=np.uint32)
    r_off[1:] = np.cumsum(r_cnt[:-1], dtype=np.uint32)
    r_idx = np.array([k for ks in signers for k in ks] or [0], dtype=np.uint32)
    r_arena, r_offs, r_lens = BL._msgs(digests)
    r_st = np.zeros(len(signers), dtype=np.int32)
    ts = []
    for i in range(reps + 2):
        t0 = time.perf_counter()
        st = b.verify_many_arrays(r_keys, r_sigs, r_off, r_cnt, r_idx, r_arena, r_offs, r_lens, r_st)
        dt = time.perf_counter() - t0
        assert not st.any(), st[:8]
        if i >= 2:
            ts.append(dt)
    # per-stage device times of the per-call paths come from a second context that records the
    # timing events (NWV_FLAG_BLS_STAGE_TIMES; they cost a single verification ~0.1 ms, so the
    # timed calls above and below run without them)
    eng_t = type(eng)(device=getattr(eng, "device", 0) or 0, flags=_lib.NWV_FLAG_BLS_STAGE_TIMES)
    b_t = Bls(eng_t)
    b_t.register_keys(pks)
    kms = []
    for i in range(5):
        st = b_t.verify_many_arrays(r_keys, r_sigs, r_off, r_cnt, r_idx, r_arena, r_offs, r_lens, r_st)
        assert not st.any(), st[:8]
        if i >= 2:
            kms.append(b_t.last_kernel_ms())
    out = {"round": {"certificates": certs, "quorum": quorum, "committee": committee, **_pcts(ts),
                     "certs_per_s": certs / float(np.median(ts)), "path": b.last_path(),
                     "kernel_ms": {k: float(np.median([x[k] for x in kms])) for k in kms[0]},
                     "kernel_ms_source": "3 calls on a NWV_FLAG_BLS_STAGE_TIMES context"}}
    m = rnd.bytes(32)
    s1 = b.sign([sks[0]], [m])[0]
    t1 = []
    for i in range(single_reps + 3):
        t0 = time.perf_counter()
        rc = b.verify(pks[0], m, s1)
        if i >= 3:
            t1.append(time.perf_counter() - t0)
        assert rc == 0
    assert b.verify(pks[0], m + b"!", s1) == _lib.NWV_ERR_SIGNATURE
    for _ in range(3):
        assert b_t.verify(pks[0], m, s1) == 0
    out["single_verify"] = dict(_pcts(t1), kernel_ms=b_t.last_kernel_ms())
    eng_t.close()
    # AggregateAuthenticator::aggregate of a quorum's votes (Certificate::new_unsafe,
    # types/src/primary.rs:476-477): `quorum` compressed signatures -> their sum.  The Core
    # aggregates votes it has verified on receipt (one verify call here), so their points come from
    # the device's verified-signature ring; "cold": votes never verified (decode + G1 check each)
    def time_agg(vs):
        ta = []
        for i in range(single_reps + 3):
            t0 = time.perf_counter()
            rc, agg_sig, _ = b.aggregate(vs)
            if i >= 3:
                ta.append(time.perf_counter() - t0)
            assert rc == 0
        return ta, agg_sig
    m_cold = rnd.bytes(32)
    vs_cold = b.sign(sks[:quorum], [m_cold] * quorum)
    ta_cold, agg_cold = time_agg(vs_cold)
    assert b.aggregate_verify(agg_cold, pks[:quorum], m_cold) == 0
    vs = b.sign(sks[:quorum], [m] * quorum)
    assert not b.verify_many(pks, vs, [[k] for k in range(quorum)], [m] * quorum).any()
    ta, agg_sig = time_agg(vs)
    assert b.aggregate_verify(agg_sig, pks[:quorum], m) == 0
    out["aggregate"] = dict(_pcts(ta), signatures=quorum, votes="verified first (one verify call)",
                            cold=dict(_pcts(ta_cold), votes="never verified"))
    # concurrent single verifies: one thread, then `concurrency` threads, for the same wall time
    sig_k = b.sign(sks[:concurrency], [m] * concurrency)

    def rate(nthreads, seconds=1.5):
        cnt, stop, err = [0] * nthreads, time.perf_counter() + seconds, []

        def work(k):
            while time.perf_counter() < stop:
                if b.verify(pks[k], m, sig_k[k]) != 0:
                    err.append(k)
                    return
                cnt[k] += 1
        th = [threading.Thread(target=work, args=(k,)) for k in range(nthreads)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not err
        return sum(cnt) / (time.perf_counter() - t0)
    r1, rn = rate(1), rate(concurrency)
    out["concurrent_single_verify"] = {"threads": concurrency, "verifies_per_s_1_thread": r1,
                                       f"verifies_per_s_{concurrency}_threads": rn, "speedup": rn / r1}
    if throughput_n:
        n = throughput_n
        msgs = [rnd.bytes(32) for _ in range(n)]
        kidx = (np.arange(n) % committee).tolist()
        sigs = b.sign([sks[k] for k in kidx], msgs)
        # the C call on prepared arrays, as a Rust caller holds them (the C4 leg does the same):
        # packing 16,384 items from Python lists costs ~8 ms of interpreter time on its own
        from narwhal_amd import bls as BL
        a_keys = BL._arr(b"".join(pks))
        a_sigs = BL._arr(b"".join(sigs))
        a_cnt = np.ones(n, dtype=np.uint32)
        a_off = np.arange(n, dtype=np.uint32)
        a_idx = np.asarray(kidx, dtype=np.uint32)
        a_arena, a_offs, a_lens = BL._msgs(msgs)
        a_st = np.zeros(n, dtype=np.int32)
        t2, km2 = [], []
        for i in range(3):
            t0 = time.perf_counter()
            st = b.verify_many_arrays(a_keys, a_sigs, a_off, a_cnt, a_idx, a_arena, a_offs, a_lens, a_st)
            dt = time.perf_counter() - t0
            assert not st.any()
            if i:
                t2.append(dt)
                km2.append(b.last_kernel_ms())
        out["throughput"] = {"items": n, "ms_host_to_host": float(np.median(t2)) * 1e3,
                             "verifies_per_s": n / float(np.median(t2)), "path": b.last_path(),
                             "kernel_ms": {k: float(np.median([x[k] for x in km2])) for k in km2[0]}}
        out["roofline"] = bls_roofline(n, out["throughput"]["kernel_ms"]["pairing_check"], peak)
        sample = sorted(rnd.choice(n, 48, replace=False).tolist())
        tp_check = ([sigs[k] for k in sample], [[kidx[k]] for k in sample], [msgs[k] for k in sample])
    out["dag_round"], arrs = leg_bls_dag(eng, b, sks, pks, rnd, dag_rounds)
    # the same round through the batching service with concurrent submitters (SURVEY §8 f1 + f4)
    out["service"] = leg_bls_service(eng, *arrs[:4])
    del arrs
    # the oracle: statuses of the round (and a throughput sample) + the CPU baseline
    import bls_ffi as B  # checker / CPU baseline only
    t0 = time.perf_counter()
    want = B.verify_items(pks, aggs, signers, digests, threads=threads)
    cpu_round_s = time.perf_counter() - t0
    assert want == [0] * certs
    got_bad = b.verify_many(pks, [aggs[0], aggs[1]], [signers[0], signers[0]], [digests[0], digests[0]])
    want_bad = B.verify_items(pks, [aggs[0], aggs[1]], [signers[0], signers[0]], [digests[0], digests[0]], threads=2)
    oracle = {"round_statuses_equal": True, "forged_pair_equal": list(got_bad) == want_bad}
    if throughput_n:
        oracle["throughput_sample_equal"] = B.verify_items(pks, *tp_check, threads=threads) == [0] * len(sample)
    out["oracle_check"] = oracle
    assert all(oracle.values()), oracle
    if cpu:
        t0 = time.perf_counter()
        rounds = 0
        while True:
            B.verify_items(pks, aggs, signers, digests, threads=threads)
            rounds += 1
            if time.perf_counter() - t0 >= 8.0:
                break
        cdt = (time.perf_counter() - t0) / rounds
        t0 = time.perf_counter()
        ns = 0
        while time.perf_counter() - t0 < 2.0:
            assert B.verify(pks[0], m, s1) == 0
            ns += 1
        out["cpu_baseline"] = {
            "value": certs / cdt, "unit": "certificates/s", "cores": threads, "kind": "port",
            "round_ms": cdt * 1e3, "single_verify_ms_1core": (time.perf_counter() - t0) / ns * 1e3,
            "sample": f"{rounds} x the same {certs}-certificate round ({quorum} of {committee} signers each), "
                      f"items split over {threads} threads; oracle/bls_oracle.c (plain C restatement of blst "
                      "fast_aggregate_verify), each key decoded and validated once per call"}
        out["round"]["gpu_speedup_over_cpu"] = out["round"]["certs_per_s"] / out["cpu_baseline"]["value"]
    out["note"] = ("BLS12-381 min_sig (48 B G1 signatures, 96 B G2 keys), fastcrypto's DST, committee keys "
                   "registered in the device key cache; item = sig decode + G1 check, key sum, hash to G1, "
                   "pairing check")
    return out


def leg_bls_dag(eng, b, sks, pks, rnd, rounds=20):
    """C5 under BLS: a 100-node DAG round (100 headers, 99 votes, 100 certificates x 67 signers)
    through ONE nwv_bls_verify_mixed_many call per round (host -> host)"""
    n = len(pks)
    sk_of = dict(zip(pks, sks))
    com = T.Committee(list(pks), [1] * n, 0, [[0, 1, 2, 3]] * n)
    q = com.quorum_threshold()
    parents = T.bls_certificate_digests(eng, T.BlsCertificate.genesis(com))
    headers = [T.Header(author=k, round=1, epoch=0, payload=[(rnd.bytes(32), a % 4)], parents=list(parents),
                        signature=bytes(48)) for a, k in enumerate(com.keys)]
    for h, d in zip(headers, T.bls_header_digests(eng, headers)):
        h.id = d
    for h, s_ in zip(headers, b.sign([sk_of[h.author] for h in headers], [h.id for h in headers])):
        h.signature = s_
    voters = [[i for i in range(n) if i != a][:q] for a in range(n)]
    votes = [T.Vote(headers[a].id, 1, 0, com.keys[a], com.keys[v], bytes(48)) for a in range(n) for v in voters[a]]
    for v, s_ in zip(votes, b.sign([sk_of[v.author] for v in votes], T.bls_vote_digests(eng, votes))):
        v.signature = s_
    certs = [T.BlsCertificate.new(eng, com, headers[a], [(v.author, v.signature) for v in votes[a * q:(a + 1) * q]])
             for a in range(n)]
    vsample = votes[:99]
    keep = T._Keep()
    cc = com._c(keep)
    harr = (T._Header * n)(*[h._c(keep) for h in headers])
    varr = (T._Vote * len(vsample))(*[v._c(keep) for v in vsample])
    carr = (T._BlsCertificate * n)(*[c._c(keep) for c in certs])
    hres, vres, cres = (ctypes.c_int32 * n)(), (ctypes.c_int32 * len(vsample))(), (ctypes.c_int32 * n)()
    lib = T.lib()
    ts = []
    for r in range(rounds + 2):
        t0 = time.perf_counter()
        rc = lib.nwv_bls_verify_mixed_many(eng._h, ctypes.byref(cc), n, harr, hres, len(vsample), varr, vres, n, carr,
                                           cres)
        dt = time.perf_counter() - t0
        assert rc == 0 and not any(hres) and not any(vres) and not any(cres)
        if r >= 2:
            ts.append(dt)
    out = dict(_pcts(ts), headers=n, votes=len(vsample), certificates=n, quorum=q,
               items_per_round=2 * n + len(vsample),
               note="one nwv_bls_verify_mixed_many call per round: every digest in one BLAKE2b launch, every "
                    "signature check (200 single-key, 100 aggregates of 67) in one BLS verification call")
    return out, (cc, harr, varr, carr, keep)


def leg_bls_service(eng, cc, harr, varr, carr, rounds=10, submitters=8):
    """The BLS round through the in-library batching service (nwv_service_create_bls), the way the
    Core loop's producers feed it (primary/src/core.rs:614-714): `submitters` threads each hand
    their share of a round's 299 headers, votes and certificates to the service asynchronously
    (nwv_service_submit_bls_*); each message's completion callback records its latency (submit ->
    own DagError code).  Reports the round time, p50 / p99 per message and the engine calls the
    service made (each flush = one nwv_bls_verify_mixed_many).  Then the same with blocking
    submitters (nwv_service_verify_bls_*: each thread waits for its message's code before the next)."""
    import threading
    from narwhal_amd import service as S
    lib = S.bind(T.lib())
    fns = [lib.nwv_service_submit_bls_header] * len(harr) + [lib.nwv_service_submit_bls_vote] * len(varr) + \
        [lib.nwv_service_submit_bls_certificate] * len(carr)
    vfns = [lib.nwv_service_verify_bls_header] * len(harr) + [lib.nwv_service_verify_bls_vote] * len(varr) + \
        [lib.nwv_service_verify_bls_certificate] * len(carr)
    structs = [harr[i] for i in range(len(harr))] + [varr[i] for i in range(len(varr))] + \
        [carr[i] for i in range(len(carr))]
    m = len(structs)
    out = {"messages_per_round": m, "rounds": rounds, "submitters": submitters}
    h = ctypes.c_void_p()
    _lib._check(lib.nwv_service_create_bls(eng._h, ctypes.byref(cc), 512, 1000, ctypes.byref(h)))
    t_sub, t_done = np.zeros(m), np.zeros(m)
    codes = np.zeros(m, dtype=np.int32)
    ev, lk, left = threading.Event(), threading.Lock(), [0]

    def on_done(user, code):
        i = user or 0
        t_done[i] = time.perf_counter()
        codes[i] = code
        with lk:
            left[0] -= 1
            if left[0] == 0:
                ev.set()

    cb = S.DONE_FN(on_done)
    try:
        # asynchronous submitters
        lat, rtimes, calls = [], [], []
        for r in range(rounds + 1):
            ev.clear()
            left[0] = m
            st0 = np.zeros(6, dtype=np.uint64)
            lib.nwv_service_stats(h, st0.ctypes.data)
            go = threading.Barrier(submitters + 1)

            def submit(lo):
                go.wait()
                for i in range(lo, m, submitters):
                    t_sub[i] = time.perf_counter()
                    _lib._check(fns[i](h, ctypes.byref(structs[i]), cb, ctypes.c_void_p(i)))

            th = [threading.Thread(target=submit, args=(lo,)) for lo in range(submitters)]
            for t in th:
                t.start()
            go.wait()
            t0 = time.perf_counter()
            for t in th:
                t.join()
            assert ev.wait(60), "service round timed out"
            dt = time.perf_counter() - t0
            assert not codes.any(), [int(c) for c in codes if c][:8]
            st1 = np.zeros(6, dtype=np.uint64)
            lib.nwv_service_stats(h, st1.ctypes.data)
            if r:  # the first round warms up
                rtimes.append(dt)
                lat.append(t_done - t_sub)
                calls.append(int(st1[0] - st0[0]))
        a = np.concatenate(lat) * 1e3
        out["async_submitters"] = {"ms_per_round": float(np.median(rtimes)) * 1e3,
                                   "latency_ms_p50": float(np.percentile(a, 50)),
                                   "latency_ms_p99": float(np.percentile(a, 99)),
                                   "engine_calls_per_round": float(np.mean(calls)),
                                   "max_engine_calls_per_round": int(max(calls))}
        # blocking submitters: each thread has one message outstanding at a time
        blat, brt, bcalls = [], [], []
        for r in range(3):
            st0 = np.zeros(6, dtype=np.uint64)
            lib.nwv_service_stats(h, st0.ctypes.data)
            per = [[] for _ in range(submitters)]
            bad = []

            def blocking(lo):
                res = ctypes.c_int32(0)
                for i in range(lo, m, submitters):
                    t1 = time.perf_counter()
                    rc = vfns[i](h, ctypes.byref(structs[i]), ctypes.byref(res))
                    per[lo].append(time.perf_counter() - t1)
                    if rc or res.value:
                        bad.append((i, rc, res.value))

            th = [threading.Thread(target=blocking, args=(lo,)) for lo in range(submitters)]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            dt = time.perf_counter() - t0
            assert not bad, bad[:4]
            st1 = np.zeros(6, dtype=np.uint64)
            lib.nwv_service_stats(h, st1.ctypes.data)
            if r:
                brt.append(dt)
                blat += [x for p in per for x in p]
                bcalls.append(int(st1[0] - st0[0]))
        b = np.array(blat) * 1e3
        out["blocking_submitters"] = {"ms_per_round": float(np.median(brt)) * 1e3,
                                      "latency_ms_p50": float(np.percentile(b, 50)),
                                      "latency_ms_p99": float(np.percentile(b, 99)),
                                      "engine_calls_per_round": float(np.mean(bcalls))}
    finally:
        lib.nwv_service_free(h)
    out["note"] = ("nwv_service_create_bls(max_batch 512, max_wait 1000 us); async: each submitter thread "
                   "submits its share of the round at once and the callbacks record each message's latency; "
                   "blocking: one message outstanding per thread")
    return out
