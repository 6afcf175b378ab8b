"""Per-kernel durations and the gaps between consecutive dispatches from a rocprofv3 kernel trace."""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
gap = defaultdict(list)
prev = None
for r in rows:
    k = r["Kernel_Name"].split("(")[0][-40:]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    dur[k].append((e - s) / 1e3)
    if prev is not None:
        gap[(prev[0], k)].append((s - prev[1]) / 1e3)
    prev = (k, e)
for k, v in dur.items():
    v = np.array(v[-50:])
    print(f"{k:42s} n={len(dur[k]):4d} med {np.median(v):7.2f} us  mean {v.mean():7.2f}")
for (a, b), v in gap.items():
    v = np.array(v[-50:])
    if len(v) > 5:
        print(f"gap {a[-20:]:>20s} -> {b[-20:]:20s} med {np.median(v):6.2f} us")
