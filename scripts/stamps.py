"""Summarise per-tile phase stamps written by `bench.py --stats` (gpurun_out/stamps_rank0.npy)."""
import sys

import numpy as np

s = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps_rank0.npy").astype(np.int64)
# two-pass layout: [0] scan tile start [1] entry known [2] walked [3] counted [4] published (+group folds)
#                  [5] emit tile start [6] walked [7] written
t0 = s[:, 0].min()
us = (s - t0) / 100.0  # s_memrealtime = 100 MHz
print("tiles", len(s), "scan span us %.2f" % (us[:, 4].max() - us[:, 0].min()),
      "emit span us %.2f" % (us[:, 7].max() - us[:, 5].min()), "gap us %.2f" % (us[:, 5].min() - us[:, 4].max()))
for a, b, nm in ((0, 1, "entry"), (1, 2, "walk"), (2, 3, "count"), (3, 4, "pub+fold"), (5, 6, "walk"),
                 (6, 7, "decode+write"), (0, 4, "scan tile"), (5, 7, "emit tile")):
    d = us[:, b] - us[:, a]
    print(f"{nm:14s} mean {d.mean():6.2f} med {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
c0 = s[:, 8] != 0  # chunk-first tiles (stamps 8..12)
light = c0.any() and not s[:, 5].any()  # light mode: no per-tile emit stamps
if light:  # chunk stamps [8]=[9] emit start [10] prefix known [11] counts summed [12] copied
    u = lambda k: (s[c0, k] - t0) / 100.0
    print("light emit span us %.2f  gap us %.2f" % (u(12).max() - u(8).min(), u(8).min() - us[:, 4].max()))
    for a, b, nm in ((9, 10, "emit prefix"), (10, 11, "sum counts"), (11, 12, "copy"), (8, 12, "emit chunk")):
        d = u(b) - u(a)
        print(f"{nm:16s} mean {d.mean():6.2f} med {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    print("emit chunk entry pct", np.percentile(u(8), [0, 10, 50, 90, 100]).round(2))
elif c0.any():
    u = lambda k: (s[c0, k] - t0) / 100.0
    for a, b, nm in ((8, 9, "emit prologue"), (9, 10, "emit prefix"), (11, 12, "scan arrive+fold")):
        d = u(b) - u(a)
        print(f"{nm:16s} mean {d.mean():6.2f} med {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    print("emit chunk entry pct", np.percentile(u(8), [0, 10, 50, 90, 100]).round(2))
for c, nm in ((0, "scan"), (5, "emit")):
    e = c + 2 if c == 5 else 4
    ts = np.linspace(us[:, c].min(), us[:, e].max(), 12)
    print(nm, "active", [int(((us[:, c] <= x) & (us[:, e] > x)).sum()) for x in ts])
