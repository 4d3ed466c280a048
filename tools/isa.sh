#!/bin/bash
# Disassemble one built object's gfx950 code (dispersy_amd/csrc/build/<name>.o) to /tmp/isa/<name>.s; with a
# second argument, also extract the first kernel whose demangled name contains it into /tmp/isa/kernel.s
set -e
o=/root/repo/dispersy_amd/csrc/build/$1.o
mkdir -p /tmp/isa && cd /tmp/isa
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section=.hip_fatbin=$1.fatbin $o
$L/clang-offload-bundler --unbundle --type=o --input=$1.fatbin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$1.co
$L/llvm-objdump -d --demangle $1.co > $1.s
if [ -n "$2" ]; then
  n=$(grep -n "^[0-9a-f]* <.*$2" $1.s | head -1 | cut -d: -f1)
  awk -v n=$n 'NR>=n' $1.s | awk '/^$/{exit} {print}' > kernel.s
  echo "$(wc -l < kernel.s) lines; scratch: $(grep -c scratch_ kernel.s)"
fi
