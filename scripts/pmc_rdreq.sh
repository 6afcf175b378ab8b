#!/bin/bash
# L2 -> fabric read request sizes (TCC_EA0_RDREQ_{32B,64B,128B}) of the C2 and C3 bench kernels,
# one rocprofv3 --pmc pass each (no trace domains).  Usage: pmc_rdreq.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"
cd /tmp && export TMPDIR=/tmp
for cfg in c2 c3; do
  [ $cfg = c2 ] && A="--steps 10 --warmup 2" || A="--config c3 --steps 2 --warmup 1"
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum \
    --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$cfg" -o run -- python3 "$R/bench.py" $A --no-cpu \
    > "$R/gpurun_out/pmc_${TAG}_$cfg.log" 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
