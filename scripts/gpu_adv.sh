#!/bin/bash
# The 300-MB adversarial capture through the sparse walk and the resident pass (scripts/time_adversarial.py),
# then its kernel times under rocprofv3.  Usage: gpu_adv.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"
timeout -k 10 300 python scripts/time_adversarial.py > "gpurun_out/${TAG}_adv.json" 2> "gpurun_out/${TAG}_adv.err" || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_adv_prof" -o run \
   -- python3 "$R/scripts/time_adversarial.py" > "$R/gpurun_out/${TAG}_adv_prof.log" 2>&1) || exit $?
