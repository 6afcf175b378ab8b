#!/bin/bash
# Per-record API: parity (device vs oracle), then convert_records A/B: the persistent pipelined
# kernel (default) vs the one-block-per-workgroup kernel (NPR_CVT=1), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-cvt}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_records_api.py tests/test_c_harness.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
NPR_CVT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_records_api.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests1_$TAG.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python scripts/bench_records_api.py > gpurun_out/rec_${TAG}_p$i.json 2>> gpurun_out/rec_$TAG.err || exit $?
  NPR_CVT=1 timeout -k 10 200 python scripts/bench_records_api.py > gpurun_out/rec_${TAG}_o$i.json 2>> gpurun_out/rec_$TAG.err || exit $?
done
exit 0
