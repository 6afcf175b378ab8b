#!/bin/bash
# Round-3 check on one GPU: every -m gpu test, then the C2 bench with / without the cross-context
# launch ordering (A/B, interleaved), the per-record API timings.  Usage: gpu_r03.sh TAG [tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-r03}"
TESTS="${2:-tests}"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu > gpurun_out/bench_c2_${TAG}_on$i.json 2> gpurun_out/bench_c2_${TAG}_on$i.err || exit $?
  NPR_LAUNCH_ORDER=0 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu > gpurun_out/bench_c2_${TAG}_off$i.json 2> gpurun_out/bench_c2_${TAG}_off$i.err || exit $?
done
timeout -k 10 200 python scripts/bench_records_api.py > gpurun_out/records_api_$TAG.json 2> gpurun_out/records_api_$TAG.err || exit $?
exit 0
