#!/bin/bash
# k_convert_records over list sizes, interleaved against variants.  Usage: gpu_cvt_sizes.sh TAG ROUNDS "SIZES" V...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; SIZES="$3"; shift 3
L=$PWD/net-parser-rs_amd/lib
for r in $(seq 1 "$ROUNDS"); do for n in $SIZES; do for v in "$@"; do
  [ "$v" = base ] && lib=$L/libnpr.so || lib=$L/libnpr_$v.so
  NPR_LIB=$lib timeout -k 10 200 python scripts/cvt_breakdown.py 4 $n >> gpurun_out/${TAG}_sizes.txt 2>>gpurun_out/${TAG}_sizes.err || exit $?
done; done; done
exit 0
