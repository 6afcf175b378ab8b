#!/bin/bash
# req_size microbench: timings, then one rocprofv3 --pmc pass with the request-size counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"
timeout -k 10 120 scripts/microbench/req_size > gpurun_out/${TAG}_req_size.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
  --output-format csv -d "$R/gpurun_out/pmc_${TAG}_req" -o run -- "$R/scripts/microbench/req_size" > "$R/gpurun_out/pmc_${TAG}_req.log" 2>&1
exit $?
