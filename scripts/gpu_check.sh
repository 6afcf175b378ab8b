#!/bin/bash
# One GPU pass over a candidate tree: every -m gpu test, the C2 bench (HIP events over 200 launches),
# one issue-counter PMC pass of the C2 bench, and optionally C3.  Usage: gpu_check.sh TAG [c3]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "gpurun_out/${TAG}_tests.log" 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > "gpurun_out/${TAG}_bench.json" 2> "gpurun_out/${TAG}_bench.err" || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES \
   --output-format csv -d "$R/gpurun_out/${TAG}_pmc" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu > "$R/gpurun_out/${TAG}_pmc.log" 2>&1) || exit $?
if [ "${2:-}" = "c3" ]; then
  timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > "gpurun_out/${TAG}_bench_c3.json" 2>> "gpurun_out/${TAG}_bench.err" || exit $?
fi
exit 0
