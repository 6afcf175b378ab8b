#!/bin/bash
# A/B of in-tree library variants (lib/libnpr_*.so via NPR_LIB): bench + stamps each.
# Usage: bash scripts/ab.sh TAG lib1 lib2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG=$1; shift
for L in "$@"; do
  b=$(basename "$L" .so)
  NPR_LIB="$R/$L" timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu > "gpurun_out/ab_${TAG}_$b.json" 2>&1 || exit $?
  NPR_LIB="$R/$L" timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu --stats > "gpurun_out/ab_${TAG}_${b}_stats.log" 2>&1 || exit $?
  cp gpurun_out/stamps_rank0.npy "gpurun_out/stamps_${TAG}_$b.npy"
done
exit 0
