#!/bin/bash
# C2 timing-only builds (lib/libnpr_<V>.so; "base" = the product build): for each, the bench's
# kernel time (gate off: an ablation's rows are not the reference's) and one PMC pass of issue
# counters.  Usage: abl_c2.sh TAG V...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
for v in "$@"; do
  [ "$v" = "base" ] && L=$R/net-parser-rs_amd/lib/libnpr.so || L=$R/net-parser-rs_amd/lib/libnpr_$v.so
  NPR_LIB=$L timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu --no-gate > "gpurun_out/${TAG}_${v}.json" 2>> "gpurun_out/${TAG}.err" || exit $?
  (cd /tmp && export TMPDIR=/tmp && NPR_LIB=$L timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM \
      --output-format csv -d "$R/gpurun_out/${TAG}_${v}_pmc" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu --no-gate > "$R/gpurun_out/${TAG}_${v}_pmc.log" 2>&1) || exit $?
  python - "$TAG" "$v" <<'PY'
import csv, glob, json, sys, collections
tag, v = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/{tag}_{v}.json"))
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/{tag}_{v}_pmc/run_counter_collection.csv"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_parse_resident" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for cs in per.values():
        for c, x in cs.items():
            acc[c].append(x)
print(v, "kernel_us %.2f" % (d["roofline"]["kernel_ms"] * 1e3), " ".join(f"{c}={sum(x)/len(x)/1e6:.2f}M" for c, x in sorted(acc.items())))
PY
done
exit 0
