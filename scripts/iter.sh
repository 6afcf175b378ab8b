#!/bin/bash
# Iteration loop on the GPU box: parity tests, then (only if green) the bench and a stamps run.
# Usage: bash scripts/iter.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-it}"
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$R/gpurun_out/$log" 2>&1; local rc=$?
        echo "[$(date +%T)] $* -> rc=$rc" | tee -a "$R/gpurun_out/steps.log"; return $rc; }
run 600 "gpu_tests_$TAG.log" python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
run 300 "bench_$TAG.json" python bench.py --steps 100 --warmup 10 --no-cpu || exit $?
run 300 "stats_$TAG.log" python bench.py --steps 10 --warmup 3 --no-cpu --stats || exit $?
cp gpurun_out/stamps_rank0.npy "gpurun_out/stamps_$TAG.npy"
exit 0
