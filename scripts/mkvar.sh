#!/bin/bash
# Build lib/libnpr_NAME.so from the working tree's sources with a python edit applied to
# csrc/FILE (default npr_kernels.hip; the variable `s` holds the file; the snippet rewrites it):
# A/B builds for scripts/ab_c2.sh and friends.  Usage: mkvar.sh NAME SNIPPET.py [FILE]
set -eu
cd "$(dirname "$0")/../net-parser-rs_amd"
NAME="$1"; SNIP="$2"; FILE="${3:-npr_kernels.hip}"
rm -rf "build/v$NAME"; mkdir -p "build/v$NAME/csrc" "build/v$NAME/include" lib
cp csrc/* "build/v$NAME/csrc/"; cp ../include/npr.h "build/v$NAME/include/"
sed -i 's#../../include/npr.h#../include/npr.h#' build/v$NAME/csrc/*.hip build/v$NAME/csrc/*.hpp
python3 - "build/v$NAME/csrc/$FILE" "$SNIP" <<'PY'
import sys
p, snip = sys.argv[1], sys.argv[2]
s = open(p).read()
s0 = s
exec(open(snip).read())
assert s != s0, "the edit changed nothing"
open(p, "w").write(s)
PY
for f in build/v$NAME/csrc/*.hip; do /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -disable-promote-alloca-to-lds -c "$f" -o "${f%.hip}.o" & done; wait
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared build/v$NAME/csrc/*.o -o lib/libnpr_$NAME.so
echo "lib/libnpr_$NAME.so"
