"""Child process of tests/test_gpu_shard.py: run with NWV_DEVICE_REPLICAS=3 (read by nwv_init), so
one GPU carries three independent device objects (lanes, key caches, basepoint tables) and an
all-devices context (nwv_init(ctx, 0, 0), the Rust crate's context) splits every Ed25519 call by
index over them exactly as over three GPUs (narwhal_amd/csrc/shard.h, nwv_host.hip for_shards).

  --part batch   n = 65,536 + 37 signatures (not a multiple of 64 x 3) with the C4 adversarial mix
                 plus forgeries on both sides of every shard boundary: verify_each, verify_batch
                 with and without bits, verify_batch_keyed (100 keys, with and without bits) --
                 verdict bits and the exact bad set equal the oracle's; a clean batch accepts;
                 the 1K batch's p50 on this context and on a one-device context
  --part types   a 100-node DAG round (run with a small NWV_SHARD_MIN so its 6,800-signature
                 batch splits): validate_certificates' exact invalid set and verify_mixed's codes
                 equal the oracle restatement (primary/src/block_synchronizer/responses.rs:115-138,
                 types/src/primary.rs:150-183, 307-328, 487-537)

Prints one JSON line."""
import argparse
import ctypes
import json
import os
import random
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import oracle_ffi as of  # noqa: E402  (checker)


def _threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def _ranges(n, ndev, min_per):
    """shard.h ed_shard_ranges restated (the CPU test pins the C++ against the same rules)"""
    units = (n + 63) // 64
    k = max(1, min(ndev, n // min_per, units))
    return [(min(n, units * j // k * 64), min(n, units * (j + 1) // k * 64)) for j in range(k)]


def _oracle_bits(items):
    pk, sig, msg, offs, lens = of.pack(items)
    words = of.verify_each_mt(pk, sig, msg, offs, lens, _threads())
    return np.unpackbits(words.view(np.uint8), bitorder="little")[:len(items)].astype(bool)


def part_batch(out):
    import config_legs as CL
    import narwhal_amd
    from narwhal_amd import _lib
    eng = narwhal_amd.Engine(device=None, n_devices=0)
    nd = eng.device_count
    out["devices"] = nd
    n = 65536 + 37
    smin = int(os.environ.get("NWV_SHARD_MIN", "16384"))
    rg = _ranges(n, nd, smin)
    out["ranges"] = rg
    items, pos, cats, expect_bad = CL.adversarial_batch(eng, n=n, frac=0.01, seed=66, mlen=64)
    # forgeries on both sides of every shard boundary (and the ends): flip a bit of s
    edge = sorted({0, n - 1} | {i for lo, _ in rg[1:] for i in (lo - 2, lo - 1, lo, lo + 1)})
    for i in edge:
        p, s, m = items[i]
        s = bytearray(s)
        s[45] ^= 0x04
        items[i] = (p, bytes(s), m)
    want = _oracle_bits(items)
    out["n"] = n
    out["want_bad"] = int((~want).sum())
    out["edge_bad"] = all(not want[i] for i in edge)
    got = np.array(eng.verify_each(items), dtype=bool)
    out["verify_each_equal"] = bool((got == want).all())
    ok, bits = eng.verify_batch(items)
    out["verify_batch_bits_equal"] = bool((np.array(bits, dtype=bool) == want).all()) and not ok
    out["bad_set_exact"] = sorted(np.flatnonzero(~np.array(bits, dtype=bool)).tolist()) == \
        sorted(np.flatnonzero(~want).tolist())
    ok2, _ = eng.verify_batch(items, want_bits=False)
    out["verify_batch_nobits_rejects"] = not ok2
    good = [it for it, w in zip(items, want) if w]
    okg, bg = eng.verify_batch(good)
    out["clean_batch_accepts"] = bool(okg and all(bg))
    # keyed: 100 committee keys, forged entries on both sides of every boundary
    rng = np.random.default_rng(7)
    kseeds = [rng.bytes(32) for _ in range(100)]
    kidx = [i % 100 for i in range(n)]
    msgs = [rng.bytes(32) for _ in range(n)]
    _, sg = eng.sign_many([kseeds[k] for k in kidx], msgs)
    kpk, _ = eng.sign_many(kseeds, [b""] * 100)
    keys = [kpk[32 * k:32 * k + 32].tobytes() for k in range(100)]
    sigs = [sg[64 * i:64 * i + 64].tobytes() for i in range(n)]
    forged = sorted(set(edge) | {int(x) for x in rng.choice(n, size=40, replace=False)})
    for j, i in enumerate(forged):
        s = bytearray(sigs[i])
        if j % 3 == 0:
            s[5] ^= 0x20  # R
        elif j % 3 == 1:
            s[40] ^= 0x01  # s
        else:
            v = int.from_bytes(bytes(s[32:]), "little") + CL.L_ORDER  # s + l (non-canonical)
            s[32:] = v.to_bytes(32, "little")
        sigs[i] = bytes(s)
    kitems = [(keys[kidx[i]], sigs[i], msgs[i]) for i in range(n)]
    kwant = _oracle_bits(kitems)
    okk, kbits = eng.verify_batch_keyed(keys, kidx, sigs, msgs)
    kb = np.array(kbits, dtype=bool)
    out["keyed_bits_equal"] = bool((kb == kwant).all()) and not okk
    out["keyed_bad_set_exact"] = np.flatnonzero(~kb).tolist() == forged == np.flatnonzero(~kwant).tolist()
    okk2, _ = eng.verify_batch_keyed(keys, kidx, sigs, msgs, want_bits=False)
    out["keyed_nobits_rejects"] = not okk2
    good_k = [i for i in range(n) if kwant[i]]
    okk3, kb3 = eng.verify_batch_keyed(keys, [kidx[i] for i in good_k], [sigs[i] for i in good_k],
                                       [msgs[i] for i in good_k])
    out["keyed_clean_accepts"] = bool(okk3 and all(kb3))
    # the 1K batch (32-byte messages, batch verdict only) on this context vs a one-device context
    one = narwhal_amd.Engine(device=0)

    def p50(e, reps=300):
        rng2 = np.random.default_rng(11)
        bseeds = [rng2.bytes(32) for _ in range(1024)]
        bm = [rng2.bytes(32) for _ in range(1024)]
        pk, sgb = e.sign_many(bseeds, bm)
        its = [(pk[32 * i:32 * i + 32].tobytes(), sgb[64 * i:64 * i + 64].tobytes(), bm[i]) for i in range(1024)]
        apk, asg, arena, offs, lens = _lib.soa(its)
        allv = _lib._i32(0)
        lat = []
        for r in range(reps + 10):
            t = time.perf_counter()
            _lib._check(e.lib.nwv_ed25519_verify_batch(e._h, 1024, _lib._ptr(apk), _lib._ptr(asg), _lib._ptr(arena),
                                                       _lib._ptr(offs), _lib._ptr(lens), bytes([r % 256]) * 32,
                                                       ctypes.byref(allv), None))
            assert allv.value == 1
            if r >= 10:
                lat.append(time.perf_counter() - t)
        return float(np.percentile(np.array(lat) * 1e3, 50))

    a = [p50(one), p50(eng)]
    b = [p50(one), p50(eng)]
    out["p50_1k_one_device_ms"] = min(a[0], b[0])
    out["p50_1k_replicated_ms"] = min(a[1], b[1])
    one.close()
    eng.close()


def part_types(out):
    import narwhal_amd
    import types_util as tu
    from types_util import nt
    from narwhal_amd import types as T
    eng = narwhal_amd.Engine(device=None, n_devices=0)
    out["devices"] = eng.device_count
    rnd = random.Random(101)
    fx = nt.CommitteeFixture(100, of.pubkey, of.sign, seed=101)
    c = tu.committee(fx.committee)
    q = fx.committee.quorum_threshold()
    parents = [rnd.randbytes(32) for _ in range(q)]
    certs = []
    for a in range(100):
        h = fx.header(author_idx=a, parents=parents, payload=[(rnd.randbytes(32), a % 4)])
        signers = [i for i in range(100) if i != a][:q]
        certs.append(tu.oracle_certificate(fx, h, signers))
    # every 6th certificate gets one bad vote at a varying position, every 13th a bad header
    # signature: some of them straddle the split of the round's 6,800-signature batch
    bad = set()
    for i in range(0, 100, 6):
        x = certs[i]
        j = (i * 7) % q
        s = x["sigs"][j]
        certs[i] = dict(x, sigs=x["sigs"][:j] + [s[:10] + bytes([s[10] ^ 8]) + s[11:]] + x["sigs"][j + 1:])
        bad.add(i)
    for i in range(5, 100, 13):
        certs[i] = dict(certs[i], header=dict(certs[i]["header"], signature=bytes(64)))
        bad.add(i)
    want = [nt.certificate_verify(fx.committee, x, of.verify) for x in certs]
    out["want_bad"] = sorted(i for i, w in enumerate(want) if w)
    ok, idx = T.validate_certificates(eng, c, [tu.certificate(x) for x in certs])
    out["validate_exact"] = (not ok) and idx == sorted(bad) == out["want_bad"]
    good = [x for i, x in enumerate(certs) if i not in bad]
    ok2, idx2 = T.validate_certificates(eng, c, [tu.certificate(x) for x in good])
    out["validate_clean"] = ok2 and idx2 == []
    # a mixed call: the round's headers, a vote per header, the certificates
    heads = [x["header"] for x in certs]
    hw = [nt.header_verify(fx.committee, h, of.verify) for h in heads]
    vs = []
    for a in range(0, 100, 3):
        v = fx.vote((a + 1) % 100, certs[a]["header"])
        if a % 9 == 0:
            v = dict(v, signature=v["signature"][:20] + bytes([v["signature"][20] ^ 1]) + v["signature"][21:])
        vs.append(v)
    vw = [nt.vote_verify(fx.committee, v, of.verify) for v in vs]
    gh, gv, gc = T.verify_mixed(eng, c, [tu.header(h) for h in heads], [tu.vote(v) for v in vs],
                                [tu.certificate(x) for x in certs])
    out["mixed_equal"] = gh == hw and gv == vw and gc == want
    out["mixed_nonzero"] = [sum(1 for x in hw if x), sum(1 for x in vw if x), sum(1 for x in want if x)]
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", choices=["batch", "types"], required=True)
    a = ap.parse_args()
    out = {"part": a.part, "replicas": int(os.environ.get("NWV_DEVICE_REPLICAS", "1")),
           "shard_min": int(os.environ.get("NWV_SHARD_MIN", "16384"))}
    (part_batch if a.part == "batch" else part_types)(out)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
