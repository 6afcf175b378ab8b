#!/bin/bash
# Interleaved timing of library builds of other revisions (make variant NAME=X REV=<commit>): C2 x3 and C3 x1 each.
# Usage: gpu_variants.sh TAG X [Y ...]   (base = lib/libnpr.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
for i in 1 2 3; do
  for v in base "$@"; do
    if [ "$v" = base ]; then L=""; else L="$R/net-parser-rs_amd/lib/libnpr_$v.so"; fi
    NPR_LIB=$L timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu > gpurun_out/var_${TAG}_${v}_$i.json 2>> gpurun_out/var_$TAG.err || exit $?
    python -c "import json; d=json.load(open('gpurun_out/var_${TAG}_${v}_$i.json')); print('c2 $v $i', d['roofline']['kernel_ms'])"
  done
done
for v in base "$@"; do
  if [ "$v" = base ]; then L=""; else L="$R/net-parser-rs_amd/lib/libnpr_$v.so"; fi
  NPR_LIB=$L timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 --no-cpu > gpurun_out/var_${TAG}_${v}_c3.json 2>> gpurun_out/var_$TAG.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/var_${TAG}_${v}_c3.json')); print('c3 $v', d['roofline']['kernel_ms'])"
done
exit 0
