#!/bin/bash
# Interleaved k_agg_insert timing of library builds (lib/libnpr_<V>.so; "base" = the product build):
# rocprofv3 --kernel-trace of scripts/bench_records_api.py, per-grid median of the flow-table kernels.
# Usage: ab_agg.sh TAG ROUNDS V1 V2 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    [ "$v" = "base" ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
    (cd /tmp && export TMPDIR=/tmp && NPR_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_$r" -o run --output-format csv \
       -- python3 "$R/scripts/bench_records_api.py" > "$R/gpurun_out/${TAG}_${v}_$r.json" 2> "$R/gpurun_out/${TAG}_${v}_$r.err") || exit $?
    python3 - "$R/gpurun_out/${TAG}_${v}_$r/run_kernel_trace.csv" "$v $r" <<'PY'
import csv, re, sys
from collections import defaultdict
d = defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"k_agg_insert", row["Kernel_Name"])
    if m:
        d[row.get("Grid_Size_X") or row.get("Grid_Size")].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
print(sys.argv[2], " ".join(f"grid{g}:{sorted(x)[len(x) // 2]:.1f}us" for g, x in sorted(d.items())))
PY
  done
done
exit 0
