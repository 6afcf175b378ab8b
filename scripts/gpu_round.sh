#!/bin/bash
# Round measurement set: every -m gpu test, then scripts/gpu_final.sh (bench lines, rocprofv3
# summaries, PMC passes, per-record API).  Usage: gpu_round.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-r03}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || exit $?
bash scripts/gpu_final.sh "$TAG" || exit $?
exit 0
