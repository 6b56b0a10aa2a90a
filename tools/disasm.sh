#!/bin/bash
# Disassemble the gfx950 code object that actually ships in a built object
# file (the -S output of hipcc predates device-library linking).
# Usage: tools/disasm.sh path/to/file.o out.dis
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb "$1" $T/dummy.o
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --input=$T/fb --output=$T/co --unbundle
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 $T/co > "$2"
rm -rf $T
