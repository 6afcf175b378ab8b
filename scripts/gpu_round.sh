#!/bin/bash
# Round measurement set on the GPU box: every -m gpu test; the bench lines (C2 headline with
# cpu_baseline, C3, C4 at N=1); rocprofv3 --kernel-trace --stats summaries of the C2 and C3 bench
# commands; the PMC passes (C2, C3; scripts/pmc.sh, summarised by scripts/pmc_json.py); the
# per-record API bench.  Usage: gpu_round.sh TAG [--no-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r04}"
if [ "${2:-}" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "gpurun_out/${TAG}_tests.log" 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err" || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > "gpurun_out/${TAG}_bench_c3.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu > "gpurun_out/${TAG}_bench_c4.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run --output-format csv \
   -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/${TAG}_prof.log" 2>&1) || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_c3" -o run --output-format csv \
   -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/${TAG}_prof_c3.log" 2>&1) || exit $?
bash scripts/pmc.sh "${TAG}" > "gpurun_out/${TAG}_pmc.log" 2>&1 || exit $?
bash scripts/pmc.sh "${TAG}_c3" --config c3 --steps 2 --warmup 1 > "gpurun_out/${TAG}_pmc_c3.log" 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_records_api.py > "gpurun_out/${TAG}_records_api.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
exit 0
