#!/bin/bash
# One PMC pass (instruction mix) over a short bench run.  Usage: pmc_quick.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d "$R/gpurun_out/pmcq_$TAG" -o run -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/pmcq_$TAG.log" 2>&1
