"""Per-kernel register, spill, scratch and LDS figures of a built object (hipcc -c output or the
.so): the .hip_fatbin bundle's gfx950 code object, its AMDGPU metadata notes.  Usage:
  python3 tools/kernel_regs.py narwhal_amd/lib/nwv_bls.o [substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fatbin"), os.path.join(d, "co")
        subprocess.run([f"{B}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj, os.path.join(d, "x")],
                       check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--type=o", f"--input={fb}", f"--output={co}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--unbundle"], check=True)
        notes = subprocess.run([f"{B}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = []
    for blk in re.split(r"\n\s+- \.", notes):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m or ".kd" in m.group(1):
            continue

        def g(k):
            x = re.search(r"\." + k + r":\s+(\S+)", "." + blk)
            return x.group(1) if x else "-"
        out.append((m.group(1), g("vgpr_count"), g("agpr_count"), g("vgpr_spill_count"), g("sgpr_spill_count"),
                    g("private_segment_fixed_size"), g("group_segment_fixed_size")))
    return out


if __name__ == "__main__":
    subs = sys.argv[2:]
    print("kernel vgpr agpr vgpr_spill sgpr_spill scratch_bytes_per_lane lds_static")
    for k in kernels(sys.argv[1]):
        if not subs or any(s in k[0] for s in subs):
            print(*k)
