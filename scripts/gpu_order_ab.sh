#!/bin/bash
# A/B of the cross-context launch ordering's cost on the C2 bench (NPR_LAUNCH_ORDER modes 0..3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="${1:-order}"
for i in 1 2; do
  for m in 0 1 2 3; do
    NPR_LAUNCH_ORDER=$m timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu --batch 1 > gpurun_out/${TAG}_m${m}_$i.json 2> gpurun_out/${TAG}_m${m}_$i.err || exit $?
  done
done
exit 0
