"""narwhal_amd -- MI355X (gfx950) Ed25519 / BLAKE2b-256 verification engine for Narwhal.

Drop-in for the signature-verification and digest hot path of erwanor/narwhal (see
SURVEY.md §8).  The product is the C-ABI library narwhal_amd/lib/libnwv.so
(include/nwv.h); this package only binds it.
"""
from ._lib import Engine, NwvError, load  # noqa: F401

__all__ = ["Engine", "NwvError", "load"]
