#!/bin/bash
# Parity tests + bench of both kernel variants (+ stamps of the default one).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-q}"
run() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$R/gpurun_out/$log" 2>&1; local rc=$?
        echo "[$(date +%T)] $* -> rc=$rc" | tee -a "$R/gpurun_out/steps.log"; return $rc; }
run 900 "gpu_tests_$TAG.log" python -m pytest tests -m gpu -q -x -p no:cacheprovider
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
run 300 "bench_${TAG}_pipe.log" python bench.py --steps 50 --warmup 10 --no-cpu --stats || exit $?
NPR_KERNEL=tile run 300 "bench_${TAG}_tile.log" python bench.py --steps 50 --warmup 10 --no-cpu || exit $?
exit $rc
