"""Re-entrancy: the reference calls its verifier from many tokio tasks at once (Core, the block
synchronizer, the workers; SURVEY.md §8(b) "Threading": Send + Sync, re-entrant).  Host threads
here drive one context (and a second context on the same device) concurrently with batch, keyed,
per-signature and digest calls; every result must equal the serial answer and the oracle's."""
import hashlib
import random
from concurrent.futures import ThreadPoolExecutor

import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    yield e
    e.close()


def _signed(eng, n, mlen, seed):
    rnd = random.Random(seed)
    seeds = [rnd.randbytes(32) for _ in range(n)]
    msgs = [rnd.randbytes(mlen) for _ in range(n)]
    pk, sg = eng.sign_many(seeds, msgs)
    return [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]


def _corrupt(items, idx):
    out = list(items)
    for i in idx:
        p, s, m = out[i]
        out[i] = (p, s[:5] + bytes([s[5] ^ 4]) + s[6:], m)
    return out


def test_concurrent_calls_one_context(eng):
    good = _signed(eng, 3000, 64, 1)
    bad = _corrupt(_signed(eng, 2500, 200, 2), [7, 1234, 2499])
    each = _corrupt(_signed(eng, 300, 32, 3), [0, 150])
    digests = [random.Random(4).randbytes(k * 37) for k in range(200)]
    want_bad = [of.verify(*it) for it in bad]
    want_each = [of.verify(*it) for it in each]
    want_dig = [hashlib.blake2b(m, digest_size=32).digest() for m in digests]
    assert want_bad.count(False) == 3 and want_each.count(False) == 2

    jobs = {
        "good": lambda r: eng.verify_batch(good, seed=bytes([r]) * 32),
        "bad": lambda r: eng.verify_batch(bad, seed=bytes([r + 64]) * 32),
        "each": lambda r: eng.verify_each(each),
        "digest": lambda r: eng.blake2b256_many(digests),
    }
    names = [k for k in jobs for _ in range(4)]
    with ThreadPoolExecutor(8) as ex:
        results = list(ex.map(lambda a: (a[1], jobs[a[1]](a[0])), enumerate(names)))
    for name, res in results:
        if name == "good":
            assert res[0] is True and all(res[1])
        elif name == "bad":
            assert res[0] is False and res[1] == want_bad
        elif name == "each":
            assert res == want_each
        else:
            assert res == want_dig


def test_concurrent_contexts_same_device(eng):
    import narwhal_amd
    other = narwhal_amd.Engine(device=0)
    try:
        a = _corrupt(_signed(eng, 1500, 48, 5), [99])
        b = _signed(eng, 1700, 48, 6)
        want_a = [of.verify(*it) for it in a]
        with ThreadPoolExecutor(4) as ex:
            fa = [ex.submit(eng.verify_batch, a, bytes([r]) * 32) for r in range(3)]
            fb = [ex.submit(other.verify_batch, b, bytes([r + 9]) * 32) for r in range(3)]
            for f in fa:
                ok, bits = f.result()
                assert ok is False and bits == want_a
            for f in fb:
                ok, bits = f.result()
                assert ok is True and all(bits)
    finally:
        other.close()


def test_concurrent_large_stagings(eng):
    """calls large enough for the piped staging (>= 16 MB of pk, sig and messages: msm_launch's
    early form, the fallback's speculative tables, the gated Straus pass) from four threads at once:
    all but one find the staging pool busy and copy with helper threads of their own.  Verdict bits
    of a forged and a valid batch against the oracle, every call"""
    import numpy as np
    from narwhal_amd import _lib
    n, mlen = 40000, 400
    rnd = random.Random(11)
    seeds = [rnd.randbytes(32) for _ in range(n)]
    msgs = [rnd.randbytes(mlen) for _ in range(n)]
    pk, sg = eng.sign_many(seeds, msgs)
    good = [(pk[32 * i:32 * i + 32].tobytes(), sg[64 * i:64 * i + 64].tobytes(), msgs[i]) for i in range(n)]
    bad = _corrupt(good, [3, 17000, 39999])
    want = {}
    for name, items in (("good", good), ("bad", bad)):
        apk, asg, arena, offs, lens = _lib.soa(items)
        words = of.verify_each_mt(bytes(apk[:32 * n]), bytes(asg[:64 * n]), bytes(arena), offs.copy(), lens.copy(), 8)
        want[name] = list(np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool))
    assert want["good"].count(False) == 0 and want["bad"].count(False) == 3
    names = ["good", "bad"] * 3
    with ThreadPoolExecutor(4) as ex:
        res = list(ex.map(lambda a: (a[1], eng.verify_batch(good if a[1] == "good" else bad,
                                                            seed=bytes([a[0] + 1]) * 32)), enumerate(names)))
    for name, (ok, bits) in res:
        assert ok == (name == "good")
        assert list(bits) == want[name]
