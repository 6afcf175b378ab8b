#!/bin/bash
# One iteration on the GPU box: full GPU test suite (stop on failure), bench, stamps, and one PMC
# pass of instruction counts.  Usage: gpu_iter.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-it}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "gpurun_out/tests_$TAG.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu > "gpurun_out/bench_$TAG.json" 2>&1 || exit $?
bash scripts/gpu_stats.sh "$TAG" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d "$R/gpurun_out/pmc_$TAG/p1" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/pmc_${TAG}_p1.log" 2>&1 || exit $?
exit 0
