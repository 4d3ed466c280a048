#!/usr/bin/env python3
"""Register use of every gfx950 kernel in the built objects (dispersy_amd/csrc/build/*.o): VGPRs, spills, SGPRs,
static LDS and the waves per SIMD the VGPR count allows (512 VGPRs per SIMD lane, 8-register granules).  Reads the
code object's AMDGPU metadata notes with the ROCm LLVM tools; no GPU needed.

usage: python tools/kernel_regs.py [substring ...]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(obj):
    with tempfile.TemporaryDirectory() as tmp:
        fat, co = os.path.join(tmp, "f.fatbin"), os.path.join(tmp, "k.co")
        if subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, obj],
                          capture_output=True).returncode:
            return  # host-only object
        subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fat,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
        notes = subprocess.run([LLVM + "/llvm-readelf", "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    cur = {}
    for line in notes.splitlines():
        m = re.match(r"\s+(?:- )?\.(name|vgpr_count|sgpr_count|vgpr_spill_count|group_segment_fixed_size):\s+(\S+)",
                     line)
        if not m:
            continue
        key, val = m.groups()
        cur[key] = val
        if len(cur) == 5:
            yield cur
            cur = {}


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return out.splitlines()


def main():
    subs = sys.argv[1:]
    rows = []
    for obj in sorted(glob.glob(os.path.join(ROOT, "dispersy_amd", "csrc", "build", "*.o"))):
        for k in kernels(obj):
            rows.append(k)
    names = demangle([r["name"] for r in rows])
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*", "", n)
        if subs and not any(s in n for s in subs):
            continue
        v = int(r["vgpr_count"])
        waves = min(8, 512 // max(8, (v + 7) // 8 * 8))
        print("%-70s vgpr %3d spill %3s sgpr %3s lds %6s waves/SIMD %d" % (n[:70], v, r["vgpr_spill_count"],
                                                                          r["sgpr_count"],
                                                                          r["group_segment_fixed_size"], waves))


if __name__ == "__main__":
    main()
