"""debugging aid: statuses of the BLS engine's stages on small cases (GPU)"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import narwhal_amd
from narwhal_amd.bls import Bls
g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "bls12381_kats.json")))
e = narwhal_amd.Engine(device=0)
b = Bls(e)
sks = [bytes.fromhex(k["sk"]) for k in g["keygen"]]
pks = [bytes.fromhex(k["pk"]) for k in g["keygen"]]
m = bytes(range(32))
sigs = b.sign(sks, [m] * 4)
for n in (1, 2, 64, 65):
    print("aggregate x", n, b.aggregate([sigs[0]] * n)[0::2], flush=True)
for k in range(4):
    print("verify", k, b.verify(pks[k], m, sigs[k]), flush=True)
for n in (1, 4, 64):
    st = b.verify_many(pks, [sigs[i % 4] for i in range(n)], [[i % 4] for i in range(n)], [m] * n)
    print("verify_many", n, list(st), flush=True)
