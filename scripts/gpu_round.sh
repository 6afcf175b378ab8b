#!/bin/bash
# Round measurement set on the GPU box, in phases (one gpurun call each):
#   tests  every -m gpu test
#   pmc    the PMC passes of the C2 and C3 bench commands (scripts/pmc.sh, one counter group per
#          rocprofv3 run, no trace domains), summarised by scripts/pmc_json.py into
#          gpurun_out/TAG_pmc_{c2,c3}.json (commit them as profiles/r04_pmc_{c2,c3}.json: bench.py
#          reads those as roofline.traffic)
#   bench  the bench lines (C2 headline with cpu_baseline, C3, C4 at N=1), rocprofv3 --kernel-trace
#          --stats summaries of the C2 and C3 bench commands, the per-record API bench
#   sharded  the C4 bench through the N > 1 path at N = 1 (--sharded)
# Usage: gpu_round.sh TAG PHASE...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
for PHASE in "$@"; do
  case "$PHASE" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "gpurun_out/${TAG}_tests.log" 2>&1 || exit $?
    ;;
  pmc)
    bash scripts/pmc.sh "${TAG}_c2" > "gpurun_out/${TAG}_pmc_c2.log" 2>&1 || exit $?
    python scripts/pmc_json.py "${TAG}_c2" "gpurun_out/${TAG}_pmc_c2.json" c2 || exit $?
    bash scripts/pmc.sh "${TAG}_c3" --config c3 --steps 2 --warmup 1 > "gpurun_out/${TAG}_pmc_c3.log" 2>&1 || exit $?
    python scripts/pmc_json.py "${TAG}_c3" "gpurun_out/${TAG}_pmc_c3.json" c3 || exit $?
    ;;
  bench)
    timeout -k 10 300 python bench.py --steps 50 --warmup 10 > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err" || exit $?
    timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 > "gpurun_out/${TAG}_bench_c3.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
    timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu > "gpurun_out/${TAG}_bench_c4.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
    timeout -k 10 300 python bench.py --config c4 --sharded --steps 20 --warmup 5 --no-cpu > "gpurun_out/${TAG}_bench_c4_sharded.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run --output-format csv \
       -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/${TAG}_prof.log" 2>&1) || exit $?
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_c3" -o run --output-format csv \
       -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/${TAG}_prof_c3.log" 2>&1) || exit $?
    timeout -k 10 300 python scripts/bench_records_api.py > "gpurun_out/${TAG}_records_api.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
    ;;
  sharded)  # the N > 1 code path (RCCL communicator, shared-memory exchange, RCCL flow gather) at N = 1
    timeout -k 10 300 python bench.py --config c4 --sharded --steps 20 --warmup 5 --no-cpu > "gpurun_out/${TAG}_bench_c4_sharded.json" 2> "gpurun_out/${TAG}_sharded.err" || exit $?
    ;;
  *) echo "unknown phase $PHASE"; exit 2 ;;
  esac
done
exit 0
