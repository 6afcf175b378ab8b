#!/bin/bash
# Interleaved C2 timing of library builds (lib/libnpr_<V>.so; "base" = the product build): ROUNDS x
# each variant, bench.py --steps 200 (HIP-event kernel time printed).  Usage: ab_c2.sh TAG ROUNDS V...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    [ "$v" = "base" ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
    NPR_LIB=$L timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > "gpurun_out/${TAG}_${v}_$r.json" 2>> "gpurun_out/${TAG}.err" || exit $?
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}_$r.json')); print('$v $r', d['roofline']['kernel_ms'])"
  done
done
exit 0
