#!/bin/bash
# Round-end measurement set on the GPU box: the bench lines (C2 headline incl. cpu_baseline, C3,
# C4 at N=1), a rocprofv3 kernel-trace summary of the C2 and C3 commands, the PMC passes (C2 and
# C3), and the per-record API bench.  Usage: gpu_final.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r02}"
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > "gpurun_out/final_bench_$TAG.json" 2> "gpurun_out/final_bench_$TAG.err" || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > "gpurun_out/final_bench_c3_$TAG.json" 2>> "gpurun_out/final_bench_$TAG.err" || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu > "gpurun_out/final_bench_c4_$TAG.json" 2>> "gpurun_out/final_bench_$TAG.err" || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final_prof_$TAG" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/final_prof_$TAG.log" 2>&1) || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final_prof_c3_$TAG" -o run --output-format csv \
   -- python3 "$R/bench.py" --config c3 --steps 5 --warmup 1 --no-cpu > "$R/gpurun_out/final_prof_c3_$TAG.log" 2>&1) || exit $?
bash scripts/pmc.sh "$TAG" > "gpurun_out/final_pmc_$TAG.log" 2>&1 || exit $?
bash scripts/pmc.sh "${TAG}_c3" --config c3 --steps 2 --warmup 1 > "gpurun_out/final_pmc_c3_$TAG.log" 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_records_api.py > "gpurun_out/final_records_api_$TAG.json" 2>> "gpurun_out/final_bench_$TAG.err" || exit $?
exit 0
