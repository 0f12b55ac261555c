"""Per-kernel resource usage (VGPR / AGPR / SGPR / LDS / scratch) of a built HIP object.

usage: python tools/kres.py build/_hopsx_ops/conv_mfma.hip.o [name-substring]
Extracts the gfx950 code object from the object's .hip_fatbin bundle and reads its AMDGPU metadata
notes (llvm-readelf), so occupancy can be checked without a GPU."""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(obj: str):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "k.hsaco")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
        names = subprocess.check_output(["c++filt"], input="\n".join(
            re.findall(r"\.name:\s+(\S+)", notes)), text=True).split("\n")
    out = []
    for i, blk in enumerate(re.split(r"\n\s+- \.agpr_count:", notes)[1:]):
        g = lambda k: int((re.search(rf"\.{k}:\s+(\d+)", blk) or [0, 0])[1])  # noqa: E731
        agpr = int(blk.split("\n")[0].strip() or 0)
        out.append((names[i] if i < len(names) else "?", g("vgpr_count"), agpr, g("sgpr_count"),
                    g("group_segment_fixed_size"), g("private_segment_fixed_size")))
    return out


if __name__ == "__main__":
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    for n, v, a, s, l, p in kernels(sys.argv[1]):
        if flt in n:
            print(f"vgpr {v:3d} agpr {a:3d} sgpr {s:3d} lds {l:6d} scratch {p:4d}  {n[:150]}")
