#!/usr/bin/env python3
"""SHA-256 of one kernel's machine code inside a built library: the gfx950 code object is unbundled from the .so's
.hip_fatbin section with the ROCm LLVM tools (as tools/kernel_regs.py does) and the bytes of the kernel's function
symbol are hashed.  bench.py uses it to bind a committed PMC traffic figure (profiles/pmc_traffic_<hash>.json) to the
build it was measured on: a figure measured on another build of the kernel is not reported.  CPU only.

usage: python tools/kernel_hash.py LIB SYMBOL_SUBSTRING
"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib, tmp):
    """The gfx950 code objects of a library: its .hip_fatbin holds one offload bundle per linked object file."""
    fat = os.path.join(tmp, "f.fatbin")
    subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, lib], check=True, capture_output=True)
    raw = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), raw)]
    out = []
    for i, a in enumerate(starts):
        b = starts[i + 1] if i + 1 < len(starts) else len(raw)
        part, co = os.path.join(tmp, "b%d.fatbin" % i), os.path.join(tmp, "k%d.co" % i)
        with open(part, "wb") as fh:
            fh.write(raw[a:b])
        r = subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + part,
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co):
            out.append(co)
    return out


def kernel_sha(lib, symbol_substring):
    """sha256 hex of the bytes of the first function symbol whose mangled name contains every '|'-separated part of
    symbol_substring, or None when the tools or the symbol are missing."""
    parts = symbol_substring.split("|")
    try:
        with tempfile.TemporaryDirectory() as tmp:
            for co in code_objects(lib, tmp):
                secs = subprocess.run([LLVM + "/llvm-readelf", "-S", "-W", co], check=True, capture_output=True,
                                      text=True).stdout
                text = None
                for line in secs.splitlines():
                    m = re.search(r"\]\s+\.text\s+PROGBITS\s+([0-9a-f]+)\s+([0-9a-f]+)", line)
                    if m:
                        text = (int(m.group(1), 16), int(m.group(2), 16))
                syms = subprocess.run([LLVM + "/llvm-readelf", "-s", "-W", co], check=True, capture_output=True,
                                      text=True).stdout
                for line in syms.splitlines():
                    f = line.split()
                    if len(f) >= 8 and f[3] == "FUNC" and all(p in f[7] for p in parts) and text:
                        addr, size = int(f[1], 16), int(f[2])
                        with open(co, "rb") as fh:
                            fh.seek(addr - text[0] + text[1])
                            return hashlib.sha256(fh.read(size)).hexdigest()
    except (OSError, subprocess.CalledProcessError):
        return None
    return None


# the headline kernel: k_pair_test<Md5, 2, DMA=true, DIAG=0, POOL=false, PADDED=true>
HEADLINE = "k_pair_testINS_3Md5ELi2ELb1ELi0ELb0ELb1E"

if __name__ == "__main__":
    print(kernel_sha(sys.argv[1], sys.argv[2]))
