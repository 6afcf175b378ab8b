#!/bin/bash
# Per-record entry points: GPU tests, scripts/bench_records_api.py, its kernel trace, and the
# convert kernel's per-workgroup stamps (libnpr_cv_stamp1k.so).  Usage: gpu_records.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$PWD; mkdir -p gpurun_out
TAG="$1"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_records_api.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python scripts/bench_records_api.py > gpurun_out/${TAG}_records_api.json 2> gpurun_out/${TAG}_records_api.err || exit $?
for c in 1 4; do
  NPR_LIB=$R/net-parser-rs_amd/lib/libnpr_cv_stamp1k.so timeout -k 10 200 python scripts/cvt_stamps.py $c >> gpurun_out/${TAG}_stamps.txt 2>>gpurun_out/${TAG}_stamps.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run -- python3 $R/scripts/bench_records_api.py > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit $?
exit 0
