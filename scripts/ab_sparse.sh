#!/bin/bash
# Interleaved A/B of library variants (lib/libnpr_<V>.so, "" = the product build) on the C3 bench
# under rocprofv3 --kernel-trace.  Usage: ab_sparse.sh TAG ROUNDS V1 V2 ...   (extra bench args: BENCH_ARGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    [ "$v" = "base" ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
    (cd /tmp && export TMPDIR=/tmp && NPR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_${v}_$r" -o run --output-format csv \
       -- python3 "$R/bench.py" --config c3 --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$R/gpurun_out/${TAG}_${v}_$r.json" 2> "$R/gpurun_out/${TAG}_${v}_$r.err") || exit $?
  done
done
exit 0
