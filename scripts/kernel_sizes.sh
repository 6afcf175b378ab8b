#!/bin/bash
# Code size (bytes) of every gfx950 kernel of one source file (device-only compile, the product's
# flags), from the code object's symbol table.  Usage: kernel_sizes.sh [csrc/npr_kernels.hip] [name-filter]
set -eu
SRC="${1:-$(dirname "$0")/../net-parser-rs_amd/csrc/npr_kernels.hip}"; PAT="${2:-.}"
T=$(mktemp -d); trap 'rm -rf "$T"' EXIT
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds --cuda-device-only \
  -c "$SRC" -o "$T/dev.o"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$T/dev.o" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="$T/gfx950.co"
/opt/rocm/lib/llvm/bin/llvm-readelf -s -W "$T/gfx950.co" | awk '$4=="FUNC"{print $3, $8}' | sort -u | sort -n | grep -E "$PAT"
