"""GPU parity of the BLAKE2b-256 kernels: fastcrypto::blake2b_256 known answers
(RFC 7693 / hashlib, committed in tests/golden) and serialized_batch_digest
(types/src/worker.rs:44-80) on the reference's golden bincode layout."""
import hashlib
import random
import struct

import pytest

import oracle_ffi as of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import narwhal_amd
    e = narwhal_amd.Engine(device=0)
    yield e
    e.close()


def test_known_answers(eng):
    g = of.load_golden("hash_vectors.json")
    msgs = [bytes.fromhex(v["msg"]) for v in g["blake2b256"]]
    got = eng.blake2b256_many(msgs)
    assert [d.hex() for d in got] == [v["digest"] for v in g["blake2b256"]]


def test_many_random_lengths(eng):
    rnd = random.Random(1)
    msgs = [bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(0, 700))) for _ in range(500)]
    assert eng.blake2b256_many(msgs) == [hashlib.blake2b(m, digest_size=32).digest() for m in msgs]


def test_many_short_messages_one_lane_form(eng):
    """above NWV_B2_QUAD_MAX_M (4,096) short messages take the one-lane kernel (k_blake2b_many),
    below it the quad kernel: both against hashlib, lengths 0..300 (0, 1, 2 and 3 blocks)"""
    rnd = random.Random(77)
    for m in (5000, 3000):
        msgs = [rnd.randbytes(rnd.randrange(0, 300)) for _ in range(m)]
        msgs[0], msgs[1], msgs[2] = b"", rnd.randbytes(128), rnd.randbytes(256)
        assert eng.blake2b256_many(msgs) == [hashlib.blake2b(x, digest_size=32).digest() for x in msgs]


def test_serialized_batches_golden(eng):
    g = of.load_golden("worker_batches.json")
    bufs = [bytes.fromhex(b["serialized"]) for b in g["batches"] if "serialized" in b]
    exp = [b["digest"] for b in g["batches"] if "serialized" in b]
    got = eng.batch_digest_serialized(bufs)
    assert [d.hex() for d, e in got] == exp
    assert all(e == -1 for _, e in got)
    bad = [bytes.fromhex(m["hex"]) for m in g["malformed"]]
    got = eng.batch_digest_serialized(bad)
    assert [e for _, e in got] == [m["err_offset"] for m in g["malformed"]]


def test_worker_batch_500kb(eng):
    # config 5 worker batch: 977 txs x 512 B (node/src/benchmark_client.rs:153-168 layout)
    rnd = random.Random(5)
    txs = [(bytes([1]) + struct.pack(">Q", rnd.getrandbits(64))).ljust(512, b"\0") for _ in range(977)]
    ser = struct.pack("<IQ", 0, len(txs)) + b"".join(struct.pack("<Q", len(t)) + t for t in txs)
    want = hashlib.blake2b(b"".join(txs), digest_size=32).digest()
    (d, e), = eng.batch_digest_serialized([ser])
    assert e == -1 and d == want
    assert eng.blake2b256_many([b"".join(txs)]) == [want]


def test_quad_kernel_mixed_lengths(eng):
    """a call whose longest message is >= 1 KiB runs 4 lanes per message (k_blake2b_quad):
    block-boundary lengths, empty, unaligned offsets inside the arena, and ~500 KB batches"""
    rnd = random.Random(9)
    lens = [0, 1, 111, 127, 128, 129, 255, 256, 257, 1023, 1024, 1025, 4096, 65537, 500224]
    lens += [rnd.randrange(0, 3000) for _ in range(40)]
    msgs = [rnd.randbytes(n) for n in lens]
    assert eng.blake2b256_many(msgs) == [hashlib.blake2b(m, digest_size=32).digest() for m in msgs]


def test_hundred_worker_batches_dag_round(eng):
    """configs[4]: 100 worker batches of 977 x 512 B serialized, digested in one call"""
    rnd = random.Random(55)
    bufs, want = [], []
    for b in range(100):
        txs = [(bytes([b % 2]) + struct.pack(">Q", rnd.getrandbits(64))).ljust(512, b"\0") for _ in range(977)]
        bufs.append(struct.pack("<IQ", 0, len(txs)) + b"".join(struct.pack("<Q", len(t)) + t for t in txs))
        want.append(hashlib.blake2b(b"".join(txs), digest_size=32).digest())
    got = eng.batch_digest_serialized(bufs)
    assert [d for d, _ in got] == want
