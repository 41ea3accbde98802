"""Pins the C oracle (oracle/nwv_oracle.c) against the committed golden fixtures
(tests/golden/*.json, produced by oracle/gen_golden.py and cross-checked there against
libsodium / OpenSSL / hashlib and the reference's Docker key fixtures)."""
import hashlib

import pytest

import oracle_ffi as of


def _vec(v):
    return bytes.fromhex(v["pk"]), bytes.fromhex(v["sig"]), bytes.fromhex(v["msg"])


def test_ed25519_vectors_per_signature():
    g = of.load_golden("ed25519_vectors.json")
    bad = [(i, v["category"]) for i, v in enumerate(g["vectors"]) if of.verify(*_vec(v)) != v["expect"]]
    assert not bad


def test_zip215_small_order_all_accept():
    g = of.load_golden("zip215_small_order.json")
    assert len(g["vectors"]) == 196
    assert all(of.verify(*_vec(v)) for v in g["vectors"])


def test_ed25519_batches():
    g = of.load_golden("ed25519_vectors.json")
    vecs = [_vec(v) for v in g["vectors"]]
    for b in g["batches"]:
        items = [vecs[i] for i in b["items"]]
        assert of.verify_batch(items) == b["expect"]


def test_batch_equals_and_of_individual_mt():
    g = of.load_golden("ed25519_vectors.json")
    vecs = [_vec(v) for v in g["vectors"]]
    pk, sig, msg, offs, lens = of.pack(vecs)
    bits = of.verify_each_mt(pk, sig, msg, offs, lens, threads=4)
    for i, v in enumerate(g["vectors"]):
        assert bool((int(bits[i // 64]) >> (i % 64)) & 1) == v["expect"]
    good = [x for x, v in zip(vecs, g["vectors"]) if v["expect"]]
    pk, sig, msg, offs, lens = of.pack(good * 2)
    assert of.verify_batch_mt(pk, sig, msg, offs, lens, threads=3)


def test_pippenger_regime_batch():
    # >= 190 points takes dalek's Pippenger branch in the oracle
    g = of.load_golden("ed25519_vectors.json")
    good = [_vec(v) for v in g["vectors"] if v["expect"]]
    items = (good * 4)[:200]
    assert of.verify_batch(items)
    bad = [_vec(v) for v in g["vectors"] if not v["expect"] and v["category"].startswith("B1")]
    assert not of.verify_batch(items[:150] + [bad[0]] + items[150:])


def test_keys_docker_fixtures():
    g = of.load_golden("keys.json")
    for k in g["keys"]:
        assert of.pubkey(bytes.fromhex(k["seed"])).hex() == k["pk"]


def test_rfc8032_signing_matches_golden():
    g = of.load_golden("ed25519_vectors.json")
    keys = of.load_golden("keys.json")["keys"]
    seed = bytes.fromhex(keys[0]["seed"])
    for n in (0, 32, 112, 512):
        m = bytes(range(256)) * 2
        sig = of.sign(seed, m[:n])
        assert of.verify(of.pubkey(seed), sig, m[:n])
    assert g["meta"]["pins"]["libsodium"]


def test_hash_vectors():
    g = of.load_golden("hash_vectors.json")
    for v in g["sha512"]:
        assert of.sha512(bytes.fromhex(v["msg"])).hex() == v["digest"]
    for v in g["blake2b256"]:
        assert of.blake2b256(bytes.fromhex(v["msg"])).hex() == v["digest"]
    assert of.blake2b256(b"").hex() == g["blake2b256_empty"]
    for v in g["sc_reduce"]:
        assert of.sc_reduce(bytes.fromhex(v["in"])).hex() == v["out"]


def test_worker_batch_digests():
    g = of.load_golden("worker_batches.json")
    for b in g["batches"]:
        if "serialized" in b:
            d, err = of.batch_digest_serialized(bytes.fromhex(b["serialized"]))
            assert err == -1 and d.hex() == b["digest"]
    for m in g["malformed"]:
        d, err = of.batch_digest_serialized(bytes.fromhex(m["hex"]))
        assert d is None and err == m["err_offset"]
