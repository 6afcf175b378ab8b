#!/bin/bash
# convert_records rework check: its GPU tests, interleaved timing against the previous kernel, stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_records_api.py > gpurun_out/${TAG}_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash scripts/gpu_cvtb.sh $TAG 3 base cv_old || exit $?
L=$PWD/net-parser-rs_amd/lib
for c in 1 4; do
  NPR_LIB=$L/libnpr_cv_stamp1k.so timeout -k 10 200 python scripts/cvt_stamps.py $c 4096 >> gpurun_out/${TAG}_stamps.txt 2>>gpurun_out/${TAG}_stamps.err || exit $?
done
exit 0
