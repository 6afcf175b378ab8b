#!/bin/bash
# Interleaved timing of k_convert_records variants (scripts/cvt_breakdown.py, cold and resident
# inputs).  Usage: gpu_cvtb.sh TAG ROUNDS V1 V2 ...   (base = the product library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
L=$PWD/net-parser-rs_amd/lib
for r in $(seq 1 "$ROUNDS"); do for v in "$@"; do for c in 4 1; do
  [ "$v" = base ] && lib=$L/libnpr.so || lib=$L/libnpr_$v.so
  NPR_LIB=$lib timeout -k 10 200 python scripts/cvt_breakdown.py $c >> gpurun_out/${TAG}_cvtb.txt 2>>gpurun_out/${TAG}_cvtb.err || exit $?
done; done; done
exit 0
