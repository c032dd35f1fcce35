"""Register / LDS / scratch use of the kernels in a built object (AMDGPU code-object metadata).

    python tools/kernel_resources.py [build/pt_runtime.o] [name-regex]

Extracts the gfx950 code object from the HIP fat object (llvm-objdump --offloading) and prints,
per kernel, VGPRs, AGPRs, SGPRs, spills, static LDS, scratch and the waves per SIMD the VGPR
count allows (512 VGPRs per lane per SIMD on CDNA3/4, in granules of 8).
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(__file__), "..", "project3-cuda-path-tracer-2025_amd", "build", "pt_runtime.o")
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    with tempfile.TemporaryDirectory() as d:
        obj = os.path.abspath(obj)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", obj], cwd=d, check=True, capture_output=True)
        cands = [f for f in os.listdir(os.path.dirname(obj)) if f.startswith(os.path.basename(obj) + ".") and "gfx950" in f]
        # llvm-objdump writes next to the input; move out of the build tree
        for f in os.listdir(os.path.dirname(obj)):
            if f.startswith(os.path.basename(obj) + ".0."):
                os.replace(os.path.join(os.path.dirname(obj), f), os.path.join(d, f))
        co = [os.path.join(d, f) for f in os.listdir(d) if "gfx950" in f][0]
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    kern = None
    rows = []
    for line in notes.splitlines():
        m = re.match(r"\s*- \.agpr_count:\s*(\d+)", line)
        if m:
            kern = {"agpr": int(m.group(1))}
            rows.append(kern)
            continue
        if kern is None:
            continue
        for key, name in ((".name:", "name"), (".vgpr_count:", "vgpr"), (".sgpr_count:", "sgpr"),
                          (".vgpr_spill_count:", "vspill"), (".group_segment_fixed_size:", "lds"),
                          (".private_segment_fixed_size:", "scratch")):
            m = re.match(r"\s*" + re.escape(key) + r"\s*(\S+)", line)
            if m and name not in kern:
                kern[name] = m.group(1) if name == "name" else int(m.group(1))
    for k in rows:
        if "name" not in k or not pat.search(k["name"]):
            continue
        v = max(8, (k.get("vgpr", 0) + k.get("agpr", 0) + 7) // 8 * 8)
        waves = min(8, 512 // v)
        print(f"{k['name'][:90]:90s} vgpr {k.get('vgpr', 0):3d} agpr {k['agpr']:2d} sgpr {k.get('sgpr', 0):3d} "
              f"spill {k.get('vspill', 0):3d} lds {k.get('lds', 0):6d} scratch {k.get('scratch', 0):4d} waves/SIMD {waves}")


if __name__ == "__main__":
    main()
