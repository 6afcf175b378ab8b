#!/bin/bash
# Per-wave phase stamps of the C2 resident launch (the DIAG build: bench.py --stats), summarised by
# scripts/res_stamps.py.  Usage: gpu_stamps.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"; shift
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --stats "$@" > "gpurun_out/${TAG}_stats_bench.json" 2> "gpurun_out/${TAG}_stats.err" || exit $?
python scripts/res_stamps.py gpurun_out/stamps_rank0.npy > "gpurun_out/${TAG}_stamps.txt" || exit $?
cp gpurun_out/stamps_rank0.npy "gpurun_out/${TAG}_stamps.npy"
