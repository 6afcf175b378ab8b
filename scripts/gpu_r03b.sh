#!/bin/bash
# Round-3 check on one GPU: every -m gpu test, then the C2 bench line (with the batched field) and
# its rocprofv3 kernel-trace summary.  Usage: gpu_r03b.sh TAG [tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r03}"
TESTS="${2:-tests}"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-budget 4 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/prof_$TAG.log" 2>&1) || exit $?
exit 0
