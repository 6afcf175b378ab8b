#!/bin/bash
# bench --stats (diagnostic stamps of the default launch) -> gpurun_out/stamps_TAG.npy
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-s}"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --stats > "gpurun_out/stats_$TAG.log" 2>&1 || exit $?
cp gpurun_out/stamps_rank0.npy "gpurun_out/stamps_$TAG.npy"
python scripts/res_stamps.py "gpurun_out/stamps_$TAG.npy" > "gpurun_out/res_stamps_$TAG.txt" 2>&1
exit 0
