"""Summarise scripts/pmc.sh output (gpurun_out/pmc_TAG/p*/) per kernel into a profiles/ JSON:
average counter values per dispatch, FETCH_SIZE doubled (gfx950 wide-read correction,
MI355X_MICROARCH.md), and traffic_bytes_per_step = sum over the step's kernels (each dispatched
once per step) of FETCH_SIZE x 2 + WRITE_SIZE (KiB units -> bytes).
Usage: pmc_json.py TAG OUT.json CONFIG [kernel-substr...]   (CONFIG: c2 | c3; bench.py PMC_SUMMARY)"""
import csv
import glob
import json
import sys
from collections import defaultdict

tag, out, config = sys.argv[1], sys.argv[2], sys.argv[3]
kerns = sys.argv[4:] or (["k_sparse_walk", "k_sparse_scan", "k_sparse_rows"] if config == "c3" else ["k_parse_resident"])
WORKLOAD = {"c2": "C2: 1M x 64-B Ethernet/IPv4/TCP records per GPU, device-resident",
            "c3": "C3: 8M records, frames U[64,1500] B, IPv4 TCP|UDP, device-resident (one step: every kernel once)"}
per = {k: defaultdict(list) for k in kerns}
for f in sorted(glob.glob(f"gpurun_out/pmc_{tag}/p*/run_counter_collection.csv")):
    acc = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        for k in kerns:
            if k in r["Kernel_Name"]:
                acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = k
    for d, cs in acc.items():
        for c, v in cs.items():
            per[names[d]][c].append(v)
res = {"tag": tag, "workload": WORKLOAD[config],
       "command": f"scripts/pmc.sh {tag}: rocprofv3 --pmc <group> -- python3 bench.py --config {config} ..., one pass per group",
       "note": "FETCH_SIZE doubled (gfx950 wide-read correction); FETCH counts L2 misses incl. Infinity-Cache hits",
       "per_kernel": {}}
traffic = 0.0
for k, cs in per.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in avg:
        avg["fetch_bytes_x2"] = 2 * avg["FETCH_SIZE"] * 1024
        traffic += avg["fetch_bytes_x2"]
    if "WRITE_SIZE" in avg:
        avg["write_bytes"] = avg["WRITE_SIZE"] * 1024
        traffic += avg["write_bytes"]
    avg["dispatches"] = max(len(v) for v in cs.values()) if cs else 0
    res["per_kernel"][k] = avg
res["traffic_bytes_per_step"] = round(traffic)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: {c: round(v, 1) for c, v in d.items() if c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "fetch_bytes_x2", "write_bytes")}
                  for k, d in res["per_kernel"].items()}), res["traffic_bytes_per_step"])
