#!/bin/bash
# Interleaved A/B of library builds (lib/<name>.so, selected with NPR_LIB) on ONE box, so box-to-box
# variance cancels.  Usage: ab.sh TAG REPS lib... ; env LIGHT=0|1 (default 1), FUSED=0|1 (default 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; REPS="$2"; shift 2
OUT="$R/gpurun_out/ab_${TAG}.txt"; : > "$OUT"
for i in $(seq "$REPS"); do
  for L in "$@"; do
    NPR_LIB="$R/net-parser-rs_amd/lib/$L" NPR_LIGHT="${LIGHT:-1}" NPR_FUSED="${FUSED:-0}" \
      timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu > "$R/gpurun_out/ab_${TAG}_cur.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$L rc=$rc" >> "$OUT"; cat "$R/gpurun_out/ab_${TAG}_cur.log" >> "$OUT"; exit $rc; }
    python -c "import json,sys;d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1];print(sys.argv[2],d['ms_per_step']*1000)" \
      "$R/gpurun_out/ab_${TAG}_cur.log" "$L" >> "$OUT"
  done
done
exit 0
