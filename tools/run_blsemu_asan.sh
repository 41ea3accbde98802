#!/bin/bash
# tests/test_bls_hostemu.py against the AddressSanitizer + UndefinedBehaviorSanitizer build of the
# gfx950 BLS code compiled for the host (make blsemu-asan).  CPU only.
set -euo pipefail
cd "$(dirname "$0")/.."
make -s tests/_build/libblsemu_asan.so
RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so 2>/dev/null || true)
[ -f "$RT" ] || RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
NWV_BLSEMU_LIB=$PWD/tests/_build/libblsemu_asan.so LD_PRELOAD=$RT python -m pytest tests/test_bls_hostemu.py -q -p no:cacheprovider "$@"
