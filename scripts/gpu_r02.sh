#!/bin/bash
# Round-2 check on one GPU: every -m gpu test (incl. the full-size configs), then the bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-r02}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || exit $?
exit 0
