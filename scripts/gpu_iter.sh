#!/bin/bash
# One GPU iteration: the -m gpu suite (optionally -k EXPR), then the C2 and C3 bench lines.
# Usage: gpu_iter.sh TAG [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-it}"; K="${2:-}"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > gpurun_out/tests_$TAG.log 2>&1 || exit $?
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
exit 0
