#!/bin/bash
# Interleaved C3 timing of library builds (lib/libnpr_<V>.so; "base" = the product build):
# rocprofv3 --kernel-trace --stats of the C3 bench per variant and round, per-kernel averages printed.
# Usage: ab_c3.sh TAG ROUNDS V1 V2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    [ "$v" = "base" ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
    (cd /tmp && export TMPDIR=/tmp && NPR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_${v}_$r" -o run --output-format csv \
       -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/${TAG}_${v}_$r.json" 2> "$R/gpurun_out/${TAG}_${v}_$r.err") || exit $?
    grep -E "k_sparse" "gpurun_out/${TAG}_${v}_$r/run_kernel_stats.csv" | cut -d, -f1,4 | sed "s/^/$v $r /"
  done
done
exit 0
