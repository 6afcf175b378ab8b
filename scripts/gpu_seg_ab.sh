#!/bin/bash
# The two-segment resident pass: parity (device vs oracle), then C2 bench A/B against the
# one-segment pass (NPR_SEGS=1), interleaved, and a rocprofv3 summary.  Usage: gpu_seg_ab.sh TAG [tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-seg}"
TESTS="${2:-tests/test_gpu_parity.py tests/test_gpu_scale.py::test_c2_bench_launch_bit_exact}"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --batch 1 > gpurun_out/bench_${TAG}_seg$i.json 2>> gpurun_out/bench_$TAG.err || exit $?
  NPR_SEGS=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --batch 1 > gpurun_out/bench_${TAG}_one$i.json 2>> gpurun_out/bench_$TAG.err || exit $?
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu --batch 1 > "$R/gpurun_out/prof_$TAG.log" 2>&1) || exit $?
exit 0
