#!/bin/bash
# One gpurun call: GPU parity tests, then (only if the tests did not crash) a short bench and a
# rocprofv3 kernel-trace profile of the same bench command.  Every GPU step has its own time
# limit; a crash / fault / time-out ends the script before anything else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
TAG="${1:-r01}"
run() {  # run <limit-seconds> <log> <cmd...>
  local lim=$1 log=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$R/gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $* -> rc=$rc" | tee -a "$R/gpurun_out/steps.log"
  return $rc
}
run 900 "gpu_tests_$TAG.log" python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?
if [ $rc -ne 0 ]; then echo "tests failed (rc=$rc): stop"; exit $rc; fi
run 600 "bench_$TAG.json" python bench.py --steps 50 --warmup 10 || exit $?
cd /tmp && export TMPDIR=/tmp
run 600 "rocprof_$TAG.log" rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu || exit $?
exit $rc
