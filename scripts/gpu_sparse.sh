#!/bin/bash
# Sparse-walk iteration on the GPU box: the sparse parity tests, the C3 bit-exact test, the C3
# bench line and a rocprofv3 kernel-trace summary of it.  Usage: gpu_sparse.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r04}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "sparse" --timeout 120 --timeout-method thread -p no:cacheprovider > "gpurun_out/${TAG}_sparse_tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -v -k c3 --timeout 250 --timeout-method thread -p no:cacheprovider > "gpurun_out/${TAG}_c3.log" 2>&1 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_c3" -o run --output-format csv \
   -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/${TAG}_bench_c3.json" 2> "$R/gpurun_out/${TAG}_bench_c3.err") || exit $?
exit 0
