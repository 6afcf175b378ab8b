"""Per-tile phase timings from bench.py --stats stamps (s_memrealtime, 100 MHz ticks).
count: [0] start [1] landed [8] entry [9] walked [10] offsets stored [11] counted [2] published [3] folded
emit:  [5] start [12] context+tile landed [6] prefix known [13] offsets ready [14] decoded+written [7] published"""
import sys

import numpy as np

s = np.load(sys.argv[1]).astype(np.int64)
t0 = s[:, 0].min()
S = lambda k: (s[:, k] - t0) / 100.0
med = lambda x: float(np.median(x))
def chain(name, ks, labels):
    parts = [f"{labels[i]} {med(S(ks[i+1]) - S(ks[i])):.2f}" for i in range(len(ks) - 1)]
    print(f"{name}: " + " | ".join(parts))
chain("count (median us)", [0, 1, 8, 9, 10, 11, 2, 3], ["load", "spec", "walk", "offs", "count", "publish", "fold"])
chain("emit  (median us)", [5, 12, 6, 13, 14, 7], ["load", "prefix", "offs", "decode+write", "publish"])
c0, c3, e5, e7 = S(0), S(3), S(5), S(7)
print(f"count span {c3.max():.2f} us, last start {c0.max():.2f}; emit span {e7.max() - e5.min():.2f} us")
for name, a, b in (("count", c0, c3), ("emit", e5, e7)):
    ts = np.linspace(a.min(), b.max(), 16)
    print(f"{name} live:", [int(((a <= x) & (b > x)).sum()) for x in ts])
