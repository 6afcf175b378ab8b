#!/bin/bash
# Pipelined-pass check on one GPU: parity tests, then the C2 / C3 bench lines (NPR_PIPE=0: the
# contiguous-range resident pass, for comparison).  Usage: gpu_pipe.sh TAG [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-pipe}"; K="${2:-}"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > gpurun_out/tests_$TAG.log 2>&1 || exit $?
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
fi
NPR_PIPE=1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || exit $?
NPR_PIPE=0 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu > gpurun_out/bench_c2_$TAG.old.json 2>> gpurun_out/bench_c2_$TAG.err || exit $?
NPR_PIPE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --stats > gpurun_out/bench_c2_$TAG.stats.json 2>> gpurun_out/bench_c2_$TAG.err || exit $?
python scripts/pipe_stamps.py > gpurun_out/pipe_stamps_$TAG.txt 2>&1 || exit $?
NPR_PIPE=1 timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c3_$TAG.json 2> gpurun_out/bench_c3_$TAG.err || exit $?
for per in 4; do
  NPR_CVT_PER=$per timeout -k 10 300 python scripts/bench_records_api.py > gpurun_out/records_api_$TAG.per$per.json 2>> gpurun_out/records_api_$TAG.err || exit $?
done
exit 0
