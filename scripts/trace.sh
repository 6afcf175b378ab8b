#!/bin/bash
# rocprofv3 kernel trace of the bench (env passes through: NPR_LIGHT, NPR_FUSED, ...).  Usage: trace.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace_$TAG" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu > "$R/gpurun_out/trace_$TAG.log" 2>&1
