#!/bin/bash
# One PMC pass (LDS banking) over a short bench run.  Usage: pmc_lds.sh TAG [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES \
  --output-format csv -d "$R/gpurun_out/pmcl_$TAG" -o run -- python3 "$R/bench.py" --no-cpu "$@" > "$R/gpurun_out/pmcl_$TAG.log" 2>&1
