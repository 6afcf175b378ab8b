#!/bin/bash
# Unaligned-window sparse walk (lib/libnpr_sp_unal.so): microbench check, sparse parity, C3 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"
for g in 1 6.4; do timeout -k 10 60 scripts/microbench/req_size $g x || exit 1; done > gpurun_out/${TAG}_win.txt 2>&1
L=$R/net-parser-rs_amd/lib
NPR_LIB=$L/libnpr_sp_unal.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "sparse or s256 or s4096 or s16384 or chunk" > gpurun_out/${TAG}_parity.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -1 gpurun_out/${TAG}_parity.log
for r in 1 2 3; do for v in base sp_unal; do
  [ $v = base ] && lib=$L/libnpr.so || lib=$L/libnpr_$v.so
  NPR_LIB=$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_c3_${v}_$r.json 2>>gpurun_out/${TAG}_c3.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_c3_${v}_$r.json')); print('$v $r', d['roofline']['kernel_ms'], d['ms_per_step'])"
done; done
exit 0
