"""Conversions between the oracle's dict restatement (oracle/narwhal_types.py) and the product's
narwhal_amd.types objects, shared by the types tests."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import narwhal_types as nt  # noqa: E402  (checker)

from narwhal_amd import types as T  # noqa: E402


def committee(c: "nt.Committee") -> T.Committee:
    return T.Committee(list(c.keys), list(c.stakes), c.epoch, [list(w) for w in c.workers])


def header(h) -> T.Header:
    return T.Header(h["author"], h["round"], h["epoch"], list(h["payload"]), list(h["parents"]), h["id"],
                    h["signature"])


def vote(v) -> T.Vote:
    return T.Vote(v["id"], v["round"], v["epoch"], v["origin"], v["author"], v["signature"])


def certificate(c) -> T.Certificate:
    return T.Certificate(header(c["header"]), list(c["signed"]), list(c["sigs"]))


def oracle_certificate(fx, h, signer_idx):
    """CommitteeFixture::certificate over the votes of the given authorities (generation indices)"""
    votes = [(fx.authorities[i], fx.vote(i, h)["signature"]) for i in signer_idx]
    code, signed, sigs = nt.certificate_new(fx.committee, votes, check_stake=False)
    assert code == 0
    return {"header": h, "signed": signed, "sigs": sigs}
