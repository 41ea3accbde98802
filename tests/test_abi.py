"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every entry point
declared in include/nwv.h, and refuses to run without a gfx950 device (no CPU fallback)."""
import ctypes
import os
import subprocess

import pytest

import narwhal_amd
from narwhal_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    names = _lib.exported_symbols_from_header()
    assert len(names) >= 20
    lib = _lib.load()
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(names) <= exported


def test_abi_version():
    assert _lib.load().nwv_abi_version() == 1


def test_library_contains_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    raw = open(_lib.LIB_PATH, "rb").read()
    import re
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", raw))
    assert targets == {b"gfx950"}, targets  # gfx950 code objects only


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK),
                    reason="a GPU is present")
def test_no_cpu_fallback_without_gpu():
    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.nwv_init(ctypes.byref(h), 0, 0)
    assert rc == _lib.NWV_ERR_NODEV
    with pytest.raises(narwhal_amd.NwvError):
        narwhal_amd.Engine(device=0)


def test_batch_seed_defaults_to_os_entropy():
    """the batch coefficients z_i must be unpredictable (OsRng in the reference): every Python
    entry point defaults to seed=None, which passes NULL so the library keys them from OS entropy
    on each call; a caller-given seed must be exactly 32 bytes (the C side reads 32)"""
    import inspect
    assert _lib._seed(None) is None
    assert _lib._seed(b"\x01" * 32) == b"\x01" * 32
    for bad in (b"", b"\x01" * 31, b"\x01" * 33):
        with pytest.raises(ValueError):
            _lib._seed(bad)
    for fn in (_lib.Engine.verify_batch, _lib.Engine.verify_batch_keyed, _lib.Engine.verify_batch_keyed_digests,
               _lib.Staged.run):
        assert inspect.signature(fn).parameters["seed"].default is None, fn
