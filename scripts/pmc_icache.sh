#!/bin/bash
# Instruction-cache counters of the C2 bench kernel, one rocprofv3 --pmc pass per library (no trace
# domains).  Usage: pmc_icache.sh TAG V...   (base = the product library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  [ "$v" = base ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
  NPR_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY \
    --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$v" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu \
    > "$R/gpurun_out/pmc_${TAG}_$v.log" 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
