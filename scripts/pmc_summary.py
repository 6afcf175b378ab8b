"""Average PMC counters per dispatch of the parse kernel from scripts/pmc.sh output."""
import csv
import glob
import sys
from collections import defaultdict

tag = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "k_parse"
vals = defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc_{tag}/p*/run_counter_collection.csv"):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    for d in per.values():
        for k, v in d.items():
            vals[k].append(v)
out = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(out):
    print(f"{k:28s} {out[k]:16.1f}   (n={len(vals[k])})")
if "FETCH_SIZE" in out:
    print("FETCH_SIZE x2 (gfx950 wide-read correction) MB/dispatch: %.1f" % (2 * out["FETCH_SIZE"] * 1024 / 1e6))
if "WRITE_SIZE" in out:
    print("WRITE_SIZE MB/dispatch: %.1f" % (out["WRITE_SIZE"] * 1024 / 1e6))
if "GRBM_GUI_ACTIVE" in out:
    print("GRBM_GUI_ACTIVE/8 cycles: %.0f" % (out["GRBM_GUI_ACTIVE"] / 8))
