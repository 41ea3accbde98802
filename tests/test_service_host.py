"""The batching service's host logic (narwhal_amd/csrc/nwv_service.cpp) on the
CPU, over a stand-in engine (tests/hostemu/service_stub.cpp: epoch mismatch -> InvalidEpoch,
signature byte 0 = 0xFF -> InvalidSignature, else Ok).  Checks that concurrent submitters each
get their own item's code, that items are coalesced into few engine calls, the max_batch /
max_wait_us / flush triggers, committee replacement (items keep the committee current at their
submission), engine errors reaching every submitter, and draining on free."""
import ctypes
import os
import random
import threading
import time

import pytest

from narwhal_amd import service as S
from narwhal_amd import types as T

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    path = os.path.join(ROOT, "tests", "_build", "libsvcstub.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.run(["make", "-C", ROOT, "tests/_build/libsvcstub.so"], check=True)
    lib_ = ctypes.CDLL(path)
    lib_.stub_reset.argtypes = [ctypes.c_long, ctypes.c_long]
    lib_.stub_counts.argtypes = [ctypes.c_void_p]
    return S.bind(lib_)


def _committee(epoch=0, n=4):
    keys = sorted(bytes([i + 1]) * 32 for i in range(n))
    return T.Committee(keys, [1] * n, epoch, [[0, 1]] * n)


def _header(rnd, epoch, bad):
    sig = bytes([0xFF if bad else 1]) + rnd.randbytes(63)
    return T.Header(rnd.randbytes(32), 1, epoch, [(rnd.randbytes(32), 0)], [rnd.randbytes(32) for _ in range(3)],
                    rnd.randbytes(32), sig)


def _vote(rnd, epoch, bad):
    sig = bytes([0xFF if bad else 2]) + rnd.randbytes(63)
    return T.Vote(rnd.randbytes(32), 1, epoch, rnd.randbytes(32), rnd.randbytes(32), sig)


def _cert(rnd, epoch, bad):
    c = T.Certificate(_header(rnd, epoch, bad))
    c.signed_authorities = [0, 1, 2]
    c.aggregated_signature = [rnd.randbytes(64) for _ in range(3)]
    return c


def _counts(lib):
    import numpy as np
    out = np.zeros(3, dtype=np.int64)
    lib.stub_counts(out.ctypes.data)
    return [int(x) for x in out]


def _expect(item, epoch):
    sig = item.header.signature if isinstance(item, T.Certificate) else item.signature
    ep = item.header.epoch if isinstance(item, T.Certificate) else item.epoch
    if ep != epoch:
        return T.InvalidEpoch.code
    return T.InvalidSignature.code if sig[0] == 0xFF else 0


def _verify(svc, item):
    if isinstance(item, T.Header):
        return svc.verify_header(item)
    if isinstance(item, T.Vote):
        return svc.verify_vote(item)
    return svc.verify_certificate(item)


def test_concurrent_submitters_get_their_own_codes_and_are_coalesced(lib):
    lib.stub_reset(2000, 0)  # each engine call takes 2 ms: submitters pile up behind it
    rnd = random.Random(1)
    items = []
    for k in range(600):
        make = (_header, _vote, _cert)[k % 3]
        items.append(make(rnd, 0 if k % 7 else 1, k % 5 == 0))
    got = [None] * len(items)
    svc = S.Service(None, _committee(0), max_batch=64, max_wait_us=500, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        def worker(t):
            for i in range(t, len(items), 12):
                got[i] = _verify(svc, items[i])
        th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        st = svc.stats()
    finally:
        svc.close()
    assert got == [_expect(it, 0) for it in items]
    calls, n_items, largest = _counts(lib)
    assert n_items == len(items) == st["items"]
    # 12 blocking submitters keep at most 12 items pending: coalesced about 4-12 per engine call
    assert calls == st["calls"] < len(items) // 2, (calls, st)
    assert largest > 1


def test_max_batch_and_deadline_triggers(lib):
    lib.stub_reset(0, 0)
    rnd = random.Random(2)
    svc = S.Service(None, _committee(0), max_batch=8, max_wait_us=400_000, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        done = []
        ev = threading.Event()

        def cb(code):
            done.append(code)
            if len(done) == 8:
                ev.set()

        t0 = time.perf_counter()
        for _ in range(8):
            svc.submit_vote(_vote(rnd, 0, False), cb)
        assert ev.wait(5) and time.perf_counter() - t0 < 0.3  # a full batch goes at once (deadline 0.4 s)
        assert svc.stats()["by_count"] >= 1
        one = threading.Event()
        t0 = time.perf_counter()
        svc.submit_header(_header(rnd, 0, True), lambda c: (done.append(c), one.set()))
        assert one.wait(5)
        waited = time.perf_counter() - t0
        assert 0.38 < waited < 3.0  # a lone item waits for its deadline
        assert done[-1] == T.InvalidSignature.code
        assert svc.stats()["by_deadline"] >= 1
    finally:
        svc.close()


def test_idle_gap_flushes_a_burst_as_one_call(lib):
    """nwv_service_set_idle: a burst of submissions goes out as ONE engine call once nothing has
    arrived for idle_us -- long before max_wait_us -- and a second burst after a pause is a second
    call; with the gap off the same burst waits out max_wait_us"""
    lib.stub_reset(0, 0)
    rnd = random.Random(12)
    svc = S.Service(None, _committee(0), max_batch=1000, max_wait_us=3_000_000, lib=lib, ctx=ctypes.c_void_p(1),
                    idle_us=40_000)
    try:
        for burst in range(2):
            items = [_vote(rnd, 0, k == 5) for k in range(40)]
            codes, ev = [], threading.Event()

            def cb(code, codes=codes, ev=ev):
                codes.append(code)
                if len(codes) == 40:
                    ev.set()
            t0 = time.perf_counter()
            for it in items:
                svc.submit_vote(it, cb)
            assert ev.wait(5)
            waited = time.perf_counter() - t0
            assert 0.04 <= waited < 1.5, waited  # the idle gap, not the 3 s deadline
            assert sorted(codes) == [0] * 39 + [T.InvalidSignature.code]
            st = svc.stats()
            assert st["calls"] == burst + 1 and st["by_deadline"] == burst + 1 and st["max_batch"] == 40, st
            time.sleep(0.1)
    finally:
        svc.close()
    svc = S.Service(None, _committee(0), max_batch=1000, max_wait_us=300_000, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        ev = threading.Event()
        t0 = time.perf_counter()
        for k in range(10):
            svc.submit_vote(_vote(rnd, 0, False), lambda c, k=k: ev.set() if k == 9 else None)
        assert ev.wait(5) and time.perf_counter() - t0 >= 0.29  # no gap: the deadline
    finally:
        svc.close()


def test_flush_completes_everything_submitted_before(lib):
    lib.stub_reset(0, 0)
    rnd = random.Random(3)
    svc = S.Service(None, _committee(0), max_batch=1000, max_wait_us=10_000_000, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        codes = []
        for k in range(10):
            svc.submit_certificate(_cert(rnd, 0, k == 3), codes.append)
        svc.flush()
        assert sorted(codes) == [0] * 9 + [T.InvalidSignature.code]
        assert svc.stats()["by_flush"] >= 1
    finally:
        svc.close()


def test_committee_change_applies_to_later_submissions(lib):
    lib.stub_reset(0, 0)
    rnd = random.Random(4)
    svc = S.Service(None, _committee(0), max_batch=1000, max_wait_us=10_000_000, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        a, b = [], []
        for _ in range(5):
            svc.submit_vote(_vote(rnd, 1, False), a.append)  # epoch 1 under the epoch-0 committee
        svc.set_committee(_committee(1))
        for _ in range(5):
            svc.submit_vote(_vote(rnd, 1, False), b.append)
        svc.flush()
        assert a == [T.InvalidEpoch.code] * 5 and b == [0] * 5
    finally:
        svc.close()


def test_engine_error_reaches_every_submitter_and_free_drains(lib):
    lib.stub_reset(0, 1)  # the engine call fails
    rnd = random.Random(5)
    svc = S.Service(None, _committee(0), max_batch=4, max_wait_us=1000, lib=lib, ctx=ctypes.c_void_p(1))
    codes = []
    for _ in range(3):
        svc.submit_header(_header(rnd, 0, False), codes.append)
    with pytest.raises(Exception):
        svc.verify_vote(_vote(rnd, 0, False))
    lib.stub_reset(0, 0)
    svc.submit_vote(_vote(rnd, 0, False), codes.append)
    svc.close()  # drains the pending item first
    assert codes[:3] == [-2] * 3 and codes[3] == 0


def test_callbacks_may_submit_but_blocking_calls_from_them_fail_fast(lib):
    """a completion callback that calls nwv_service_flush or a blocking verify would wait
    on the flusher running it; the service returns NWV_ERR_REENTRANT instead, and an asynchronous
    submit from a callback still completes"""
    from narwhal_amd import _lib
    lib.stub_reset(0, 0)
    rnd = random.Random(6)
    svc = S.Service(None, _committee(0), max_batch=1, max_wait_us=0, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        seen, chained = [], threading.Event()

        def cb(code):
            for call in (svc.flush, lambda: svc.verify_vote(_vote(rnd, 0, False))):
                try:
                    call()
                    seen.append("returned")
                except _lib.NwvError as e:
                    seen.append(e.code)
            svc.submit_vote(_vote(rnd, 0, True), lambda c: (seen.append(("chained", c)), chained.set()))

        svc.submit_header(_header(rnd, 0, False), cb)
        assert chained.wait(5)
        svc.flush()
        assert seen == [_lib.NWV_ERR_REENTRANT, _lib.NWV_ERR_REENTRANT, ("chained", T.InvalidSignature.code)]
    finally:
        svc.close()


def test_callback_may_block_on_another_service(lib):
    """the reentrancy refusal is per service -- a callback of service A may make a
    blocking call on service B (B's flushers are free), and A's own blocking calls still fail fast"""
    from narwhal_amd import _lib
    lib.stub_reset(0, 0)
    rnd = random.Random(7)
    a = S.Service(None, _committee(0), max_batch=1, max_wait_us=0, lib=lib, ctx=ctypes.c_void_p(1))
    b = S.Service(None, _committee(0), max_batch=1, max_wait_us=0, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        seen, done = [], threading.Event()

        def cb(code):
            seen.append(b.verify_vote(_vote(rnd, 0, False)))
            try:
                a.flush()
                seen.append("returned")
            except _lib.NwvError as e:
                seen.append(e.code)
            done.set()

        a.submit_header(_header(rnd, 0, True), cb)
        assert done.wait(5)
        assert seen == [0, _lib.NWV_ERR_REENTRANT]
    finally:
        a.close()
        b.close()


def test_core_drain_policy():
    """CoreDrain.drain (no engine call): takes what is queued up to max_items, waits at most
    max_wait_us for more, keeps arrival order"""
    import queue
    import threading
    import time
    from narwhal_amd import service as S
    from narwhal_amd import types as T
    com = T.Committee([bytes([i]) * 32 for i in range(4)], [1] * 4)
    d = S.CoreDrain(None, com, max_items=5, max_wait_us=0)
    q = queue.Queue()
    for i in range(12):
        q.put(i)
    assert d.drain(q) == [0, 1, 2, 3, 4]
    assert d.drain(q, first="x") == ["x", 5, 6, 7, 8]
    assert d.drain(q) == [9, 10, 11]  # nothing more queued, no wait
    d3 = S.CoreDrain(None, com, max_items=100, max_wait_us=200_000, min_items=3)
    for i in range(4):
        q.put(i)
    t0 = time.perf_counter()
    assert d3.drain(q) == [0, 1, 2, 3] and time.perf_counter() - t0 < 0.1  # >= min_items: no wait
    d2 = S.CoreDrain(None, com, max_items=100, max_wait_us=200_000)
    q.put(0)
    threading.Timer(0.02, lambda: q.put(1)).start()
    t0 = time.perf_counter()
    assert d2.drain(q) == [0, 1]  # a late message within the deadline joins the flush
    assert 0.15 < time.perf_counter() - t0 < 2.0  # then the deadline ends the drain
    # idle_us: past min_items, a message arriving within the gap still joins; then the gap ends it
    d4 = S.CoreDrain(None, com, max_items=100, max_wait_us=2_000_000, min_items=2, idle_us=150_000)
    for i in range(3):
        q.put(i)
    threading.Timer(0.03, lambda: q.put(3)).start()
    t0 = time.perf_counter()
    assert d4.drain(q) == [0, 1, 2, 3]
    assert 0.15 < time.perf_counter() - t0 < 1.5  # the gap after the last arrival, not the 2 s deadline


def test_blocking_wait_that_closes_a_cycle_is_refused(lib):
    """a callback of A blocks on B (edge A -> B); a callback of B that then blocks on A
    would close the cycle A -> B -> A (with every flusher of both inside such callbacks nothing
    would ever verify) -- it gets NWV_ERR_REENTRANT, while A's wait on B completes normally"""
    from narwhal_amd import _lib
    lib.stub_reset(200_000, 0)  # each engine call takes 200 ms: A's callback is inside B meanwhile
    rnd = random.Random(8)
    a = S.Service(None, _committee(0), max_batch=1, max_wait_us=0, lib=lib, ctx=ctypes.c_void_p(1))
    b = S.Service(None, _committee(0), max_batch=1, max_wait_us=0, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        a_inside, seen_a, seen_b, done = threading.Event(), [], [], threading.Event()

        def cb_a(code):
            a_inside.set()
            seen_a.append(b.verify_vote(_vote(rnd, 0, False)))

        def cb_b(code):
            assert a_inside.wait(5)
            time.sleep(0.05)
            try:
                a.verify_vote(_vote(rnd, 0, False))
                seen_b.append("returned")
            except _lib.NwvError as e:
                seen_b.append(e.code)
            done.set()

        a.submit_header(_header(rnd, 0, False), cb_a)
        b.submit_header(_header(rnd, 0, False), cb_b)
        assert done.wait(10)
        a.flush()
        assert seen_b == [_lib.NWV_ERR_REENTRANT] and seen_a == [0]
    finally:
        lib.stub_reset(0, 0)
        a.close()
        b.close()


def test_bls_service_codes_and_scheme_checks(lib):
    """a BLS12-381 service (nwv_service_create_bls): concurrent submitters of 96-byte-key headers,
    votes and certificates get their own codes through one nwv_bls_verify_mixed_many per flush (the
    stub's rule; an aggregate holding no signature -> InvalidSignature), and the other scheme's
    calls are refused on each kind of service"""
    from narwhal_amd import _lib
    lib.stub_reset(2000, 0)
    rnd = random.Random(9)
    keys = sorted(bytes([i + 1]) * 96 for i in range(4))
    com = T.Committee(keys, [1] * 4, 0, [[0, 1]] * 4)

    def header(epoch, bad):
        return T.Header(rnd.randbytes(96), 1, epoch, [(rnd.randbytes(32), 0)], [rnd.randbytes(32)],
                        rnd.randbytes(32), bytes([0xFF if bad else 1]) + rnd.randbytes(47))

    def item(k):
        kind = k % 3
        epoch, bad = (1 if k % 7 == 0 else 0), (k % 5 == 0)
        if kind == 0:
            h = header(epoch, bad)
            return h, (T.InvalidEpoch.code if epoch else T.InvalidSignature.code if bad else 0)
        if kind == 1:
            v = T.Vote(rnd.randbytes(32), 1, epoch, rnd.randbytes(96), rnd.randbytes(96),
                       bytes([0xFF if bad else 2]) + rnd.randbytes(47))
            return v, (T.InvalidEpoch.code if epoch else T.InvalidSignature.code if bad else 0)
        none = k % 11 == 0
        c = T.BlsCertificate(header(epoch, bad), [0, 1, 2], None if none else rnd.randbytes(48))
        return c, (T.InvalidSignature.code if none else T.InvalidEpoch.code if epoch else
                   T.InvalidSignature.code if bad else 0)

    svc = S.Service(None, com, max_batch=16, max_wait_us=500, lib=lib, ctx=ctypes.c_void_p(1), scheme="bls")
    ed = S.Service(None, _committee(0), max_batch=4, max_wait_us=0, lib=lib, ctx=ctypes.c_void_p(1))
    try:
        items = [item(k) for k in range(120)]
        got = [None] * len(items)

        def worker(lo):
            for k in range(lo, len(items), 8):
                got[k] = _verify(svc, items[k][0])

        th = [threading.Thread(target=worker, args=(lo,)) for lo in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert got == [w for _, w in items]
        st = svc.stats()
        assert st["items"] == 120 and st["calls"] < 120
        r = ctypes.c_int32(0)  # an Ed25519 item on the BLS service, a BLS item on the Ed25519 one
        keep = T._Keep()
        assert lib.nwv_service_verify_vote(svc._h, ctypes.byref(_vote(rnd, 0, False)._c(keep)),
                                           ctypes.byref(r)) == _lib.NWV_ERR_ARG
        assert lib.nwv_service_verify_bls_vote(ed._h, ctypes.byref(_vote(rnd, 0, False)._c(keep)),
                                               ctypes.byref(r)) == _lib.NWV_ERR_ARG
    finally:
        lib.stub_reset(0, 0)
        svc.close()
        ed.close()
