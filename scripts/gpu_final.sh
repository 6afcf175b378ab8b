#!/bin/bash
# Round-end measurement set on the GPU box: the bench line (incl. cpu_baseline), a rocprofv3
# kernel-trace summary of the same command, and the PMC passes.  Usage: gpu_final.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r01}"
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > "gpurun_out/final_bench_$TAG.json" 2> "gpurun_out/final_bench_$TAG.err" || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final_prof_$TAG" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/final_prof_$TAG.log" 2>&1) || exit $?
bash scripts/pmc.sh "$TAG" > "gpurun_out/final_pmc_$TAG.log" 2>&1 || exit $?
exit 0
