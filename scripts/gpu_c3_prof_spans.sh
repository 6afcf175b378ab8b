#!/bin/bash
# Per-kernel times of the C3 sparse step at given lane spans: rocprofv3 --kernel-trace --stats of the
# C3 bench with the sparse walk forced at each span.  Usage: gpu_c3_prof_spans.sh TAG SPAN...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
for sp in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_s$sp" -o run --output-format csv \
     -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu --sparse-span "$sp" > "$R/gpurun_out/${TAG}_s$sp.json" 2> "$R/gpurun_out/${TAG}_s$sp.err") || exit $?
  grep -E "k_sparse" "gpurun_out/${TAG}_s$sp/run_kernel_stats.csv" | cut -d, -f1-4 | sed "s/^/$sp /"
done
exit 0
