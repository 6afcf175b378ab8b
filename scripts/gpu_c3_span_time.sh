#!/bin/bash
# C3 lane-span timing, interleaved: ROUNDS x (each SPAN) C3 bench lines with the sparse walk forced.
# Usage: gpu_c3_span_time.sh TAG ROUNDS SPAN...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for sp in "$@"; do
    timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 2 --no-cpu --sparse-span "$sp" > "gpurun_out/${TAG}_s${sp}_$r.json" 2> "gpurun_out/${TAG}_s${sp}_$r.err" || exit $?
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_s${sp}_$r.json')); print('$sp $r', d['roofline']['kernel_ms'])"
  done
done
exit 0
