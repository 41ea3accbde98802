"""GPU parity of the batching service (include/nwv_service.h): threads submit
headers, votes and certificates of every DagError kind concurrently, the library coalesces them
into few nwv_verify_mixed_many calls, and every submitter gets the code the reference's
Header::verify / Vote::verify / Certificate::verify (types/src/primary.rs:150-183, :307-328,
:487-537; oracle/narwhal_types.py) returns for its own item."""
import random
import threading

import pytest

import oracle_ffi as of
import types_util as tu
from types_util import nt

from narwhal_amd import service as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    yield e
    e.close()


def _cases(seed):
    from test_gpu_types import _mutations
    rnd = random.Random(seed)
    fx = nt.CommitteeFixture(10, of.pubkey, of.sign, seed=seed)
    cases = _mutations(fx, rnd)
    items, want = [], []
    for h, cert in cases:
        if h is not None:
            items.append(tu.header(h))
            want.append(nt.header_verify(fx.committee, h, of.verify))
        items.append(tu.certificate(cert))
        want.append(nt.certificate_verify(fx.committee, cert, of.verify))
    h = fx.header()
    vs = fx.votes(h)
    vs[1] = dict(vs[1], epoch=5)
    vs[2] = dict(vs[2], author=of.pubkey(b"\x03" * 32))
    vs[3] = dict(vs[3], signature=bytes(64))
    for v in vs:
        items.append(tu.vote(v))
        want.append(nt.vote_verify(fx.committee, v, of.verify))
    return fx, items, want


def _verify(svc, item):
    from narwhal_amd import types as T
    if isinstance(item, T.Header):
        return svc.verify_header(item)
    if isinstance(item, T.Vote):
        return svc.verify_vote(item)
    return svc.verify_certificate(item)


@pytest.mark.parametrize("max_batch,max_wait_us", [(64, 300), (1, 0), (1000, 2000)])
def test_concurrent_submitters_match_oracle(eng, max_batch, max_wait_us):
    fx, items, want = _cases(31)
    assert len(set(want)) >= 6  # every DagError path is present
    reps = 4
    got = {}
    with S.Service(eng, tu.committee(fx.committee), max_batch=max_batch, max_wait_us=max_wait_us) as svc:
        def worker(t):
            for r in range(reps):
                for i in range(t, len(items), 8):
                    got[(r, i)] = _verify(svc, items[i])
        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        st = svc.stats()
    assert all(got[(r, i)] == want[i] for r in range(reps) for i in range(len(items)))
    assert st["items"] == reps * len(items)
    if max_batch > 1:
        assert st["calls"] < st["items"]  # coalesced


def test_async_callbacks_and_flush(eng):
    fx, items, want = _cases(32)
    codes = {}
    lock = threading.Lock()
    with S.Service(eng, tu.committee(fx.committee), max_batch=10_000, max_wait_us=5_000_000) as svc:
        for i, it in enumerate(items):
            def done(code, i=i):
                with lock:
                    codes[i] = code
            from narwhal_amd import types as T
            if isinstance(it, T.Header):
                svc.submit_header(it, done)
            elif isinstance(it, T.Vote):
                svc.submit_vote(it, done)
            else:
                svc.submit_certificate(it, done)
        svc.flush()  # one engine call for everything, long before the deadline
        assert [codes[i] for i in range(len(items))] == want
        assert svc.stats()["calls"] == 1


def _kind(item):
    from narwhal_amd import types as T
    return {T.Header: "header", T.Vote: "vote", T.Certificate: "certificate"}[type(item)]


@pytest.mark.parametrize("max_items,max_wait_us", [(512, 1000), (7, 0), (1, 0)])
def test_core_drain_single_consumer_matches_oracle(eng, max_items, max_wait_us):
    """the Core-side drain (service.CoreDrain, rust core_drain.rs): one consumer thread takes the
    messages a producer thread queues, flushes <= max_items per engine call, and every message's
    code equals the oracle's, in arrival order"""
    import queue
    fx, items, want = _cases(33)
    order = list(range(len(items)))
    random.Random(34).shuffle(order)
    q = queue.Queue()

    def producer():
        for i in order:
            q.put((i, (_kind(items[i]), items[i])))

    d = S.CoreDrain(eng, tu.committee(fx.committee), max_items=max_items, max_wait_us=max_wait_us)
    th = threading.Thread(target=producer)
    th.start()
    got, seen = {}, []
    while len(got) < len(items):
        batch = d.drain(q)
        assert 1 <= len(batch) <= max_items
        codes = d.verify([m for _, m in batch])
        for (i, _), c in zip(batch, codes):
            got[i] = c
            seen.append(i)
    th.join()
    assert seen == order  # arrival order kept
    assert [got[i] for i in range(len(items))] == want
    assert d.items == len(items) and d.largest <= max_items
    if max_items == 1:
        assert d.calls == len(items)


def test_core_drain_prepared_structs(eng):
    """CoreDrain.verify on prepared C structs (the bench's form) gives the same codes"""
    from narwhal_amd import types as T
    fx, items, want = _cases(35)
    keep = T._Keep()
    d = S.CoreDrain(eng, tu.committee(fx.committee))
    assert d.verify([(_kind(it), it._c(keep)) for it in items]) == want
    assert d.calls == 1
