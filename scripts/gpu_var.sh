#!/bin/bash
# C2 / C3 bench lines for the default build and each lib/libnpr_<NAME>.so variant given.
# Usage: gpu_var.sh TAG NAME...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"; shift
for V in default "$@"; do
  if [ "$V" = default ]; then L=""; else L="$PWD/net-parser-rs_amd/lib/libnpr_$V.so"; fi
  NPR_LIB="$L" timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/var_${TAG}_c2_$V.json 2>> gpurun_out/var_$TAG.err || exit $?
  NPR_LIB="$L" timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu > gpurun_out/var_${TAG}_c3_$V.json 2>> gpurun_out/var_$TAG.err || exit $?
done
exit 0
