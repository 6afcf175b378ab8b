#!/bin/bash
# Bench the tile-size variants (lib/libnpr_t*.so) fused and two-launch.  Usage: variants.sh TAG [libs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
for L in "$@"; do
  for F in 1 0; do
    NPR_LIB="$R/net-parser-rs_amd/lib/$L" NPR_FUSED=$F timeout -k 10 200 python bench.py --steps 50 --warmup 10 --no-cpu \
      > "$R/gpurun_out/var_${TAG}_${L}_f$F.log" 2>&1
    rc=$?; echo "$L fused=$F rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
