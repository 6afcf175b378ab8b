#!/bin/bash
# Two-segment pass: parity subset, C2 A/B (seg vs one segment, interleaved), stamps of both.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-seg2}"
TESTS="${2:-tests/test_gpu_parity.py tests/test_gpu_records_api.py tests/test_gpu_scale.py::test_c2_bench_launch_bit_exact}"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
for i in 1 2; do
  NPR_SEGS=2 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --batch 1 > gpurun_out/bench_${TAG}_seg$i.json 2>> gpurun_out/bench_$TAG.err || exit $?
  NPR_SEGS=1 timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu --batch 1 > gpurun_out/bench_${TAG}_one$i.json 2>> gpurun_out/bench_$TAG.err || exit $?
done
NPR_SEGS=2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --batch 1 --stats > gpurun_out/stats_${TAG}.json 2>> gpurun_out/bench_$TAG.err || exit $?
python scripts/seg_stamps.py gpurun_out/stamps_rank0.npy > gpurun_out/seg_stamps_$TAG.txt 2>&1
mv gpurun_out/stamps_rank0.npy gpurun_out/stamps_seg_$TAG.npy
NPR_SEGS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --batch 1 --stats > gpurun_out/stats1_${TAG}.json 2>> gpurun_out/bench_$TAG.err || exit $?
python scripts/res_stamps.py gpurun_out/stamps_rank0.npy > gpurun_out/res_stamps_$TAG.txt 2>&1
timeout -k 10 200 python scripts/bench_records_api.py > gpurun_out/records_api_$TAG.json 2>> gpurun_out/bench_$TAG.err || exit $?
exit 0
