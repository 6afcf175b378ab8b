#!/bin/bash
# PMC instruction counts of scripts/launch_only.py for each library variant.  Usage: abl_pmc.sh TAG lib...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  b=$(basename "$L" .so)
  NPR_LIB="$R/$L" timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$b/p1" -o run -- python3 "$R/scripts/launch_only.py" > "$R/gpurun_out/pmc_${TAG}_$b.log" 2>&1 || exit $?
  NPR_LIB="$R/$L" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/abl_${TAG}_$b" -o run \
      --output-format csv -- python3 "$R/scripts/launch_only.py" > "$R/gpurun_out/abl_${TAG}_$b.log" 2>&1 || exit $?
done
exit 0
