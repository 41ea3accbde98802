"""Child process of tests/test_gpu_bls.py::test_verify_many_sharded_over_devices: run with
NWV_BLS_DEVICE_REPLICAS=3 and NWV_BLS_SHARD_MIN=8 (read once per process), so one GPU carries three
independent BLS shards (key caches, rings, lanes) and nwv_bls_verify_many splits its items by index
over them (narwhal_amd/csrc/bls_shard.h).  A 100-key committee round (registered keys on every
shard, then the cache reset so every shard decodes the keys itself) with every adversarial category
must give the oracle's statuses; prints one JSON line."""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import bls_cases as C  # noqa: E402
import bls_ffi as B  # noqa: E402

r = 0x73eda753299d7d483339d80809a1d80553bda402fffe5bfeffffffff00000001


def main():
    import narwhal_amd
    from narwhal_amd.bls import Bls
    e = narwhal_amd.Engine(device=0)
    bls = Bls(e)
    rnd = random.Random(61)
    sks = [rnd.randrange(1, r).to_bytes(32, "big") for _ in range(100)]
    pks = bls.keygen(sks)
    keys = pks + [C.not_in_g2(), C.IDENTITY_G2]
    items = []
    for q in [67] * 40 + [100, 68, 99]:
        d = rnd.randbytes(32)
        who = sorted(rnd.sample(range(100), q))
        _, agg = B.aggregate(bls.sign([sks[k] for k in who], [d] * q))
        items.append((agg, who, d))
    agg, who, d = items[0]
    items += [(agg, who, d + b"!"), (agg, who[:-1], d), (agg, [], d), (agg, who[:30] + [100] + who[30:], d),
              (agg, who + [101], d), (C.not_in_g1(), who, d), (C.IDENTITY_G1, who, d)]
    items += [(b, who, d) for b in C.bad_encodings_g1(agg)]
    rnd.shuffle(items)
    sig, kl, ms = [i[0] for i in items], [i[1] for i in items], [i[2] for i in items]
    want = [int(x) for x in B.verify_items(keys, sig, kl, ms)]
    out = {"items": len(items), "shards": int(os.environ.get("NWV_BLS_DEVICE_REPLICAS", "1"))}
    bls.register_keys(pks)
    out["registered_on_shard0"] = int(bls.lib.nwv_bls_keycache_size(bls._h))
    out["cached_equal"] = [int(x) for x in bls.verify_many(keys, sig, kl, ms)] == want
    bls.lib.nwv_bls_keycache_reset(bls._h)
    out["uncached_equal"] = [int(x) for x in bls.verify_many(keys, sig, kl, ms)] == want
    out["want_nonzero"] = sum(1 for x in want if x)
    e.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
