#!/bin/bash
# Resident single pass: its parity tests first (fail fast), the rest of the GPU suite, then the
# bench (resident default / two-pass) and a rocprofv3 kernel-trace of the default bench.
# Usage: gpu_res.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r}"
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$R/gpurun_out/$log" 2>&1; local rc=$?
        echo "[$(date +%T)] $* -> rc=$rc" | tee -a "$R/gpurun_out/steps.log"; return $rc; }
run 600 "gpu_res_tests_$TAG.log" python -u -m pytest tests/test_gpu_parity.py -k "resident" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
run 300 "bench_${TAG}.json" python bench.py --steps 100 --warmup 10 --no-cpu || exit $?
NPR_RESIDENT=0 run 300 "bench_${TAG}_twopass.json" python bench.py --steps 100 --warmup 10 --no-cpu || exit $?
run 900 "gpu_tests_$TAG.log" python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
exit 0
