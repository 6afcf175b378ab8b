#!/bin/bash
# Interleaved A/B of library variants (lib/libnpr_<V>.so; "base" = the product build) on the
# per-record API bench.  Usage: ab_records_api.sh TAG ROUNDS V1 V2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    [ "$v" = "base" ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
    NPR_LIB=$L timeout -k 10 300 python scripts/bench_records_api.py > "gpurun_out/${TAG}_${v}_$r.json" 2> "gpurun_out/${TAG}_${v}_$r.err" || exit $?
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}_$r.json')); print('$v $r', d['dev_convert_records']['kernel_ms'], d['dev_extract_flows']['kernel_ms'])"
  done
done
exit 0
