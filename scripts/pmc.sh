#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, no trace domains) over a short bench.
# Usage: bash scripts/pmc.sh TAG [extra bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM SQ_INSTS_VSKIPPED SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_$TAG/p$i" -o run \
      -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu "$@" > "$R/gpurun_out/pmc_${TAG}_p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
