#!/bin/bash
# Parity tests + bench (defaults: two launches, parked flows) + stamps runs of the default, the
# decode-in-pass-2 (NPR_LIGHT=0) and the fused variants.  Usage: gpu_quick.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-q}"
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$R/gpurun_out/$log" 2>&1; local rc=$?
        echo "[$(date +%T)] $* -> rc=$rc" | tee -a "$R/gpurun_out/steps.log"; return $rc; }
run 900 "gpu_tests_$TAG.log" python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; [ $rc -eq 0 ] || exit $rc   # any failure may be a device fault: run nothing more
run 300 "bench_${TAG}.log" python bench.py --steps 100 --warmup 10 --no-cpu || exit $?
run 300 "bench_${TAG}_stats.log" python bench.py --steps 20 --warmup 5 --no-cpu --stats || exit $?
cp gpurun_out/stamps_rank0.npy gpurun_out/stamps_${TAG}.npy
NPR_LIGHT=0 run 300 "bench_${TAG}_decode.log" python bench.py --steps 100 --warmup 10 --no-cpu || exit $?
NPR_FUSED=1 run 300 "bench_${TAG}_fused.log" python bench.py --steps 100 --warmup 10 --no-cpu || exit $?
exit 0
