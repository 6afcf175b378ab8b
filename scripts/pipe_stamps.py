"""Timeline of one k_parse_pipe launch from its DIAG stamps (bench.py --stats -> gpurun_out/stamps_rank0.npy).
Parser row v: [0] start [1..6] round 0..5 aggregate published [7] drain start [8] done [9] ticks in blocking
flushes [10] rounds flushed before the drain [11] rounds.  Resolver row W + b: [q] round q's X posted
(q < 8), [12] / [13] G(0, b) / G(1, b) published, [14] / [8] every G(0, .) / G(1, .) seen, [10] / [9]
round 0 / 1 windows folded, [11] round 0 local fold done.
Usage: python scripts/pipe_stamps.py [path] [W]"""
import sys

import numpy as np

p = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps_rank0.npy"
W = int(sys.argv[2]) if len(sys.argv) > 2 else 3840
s = np.load(p).astype(np.int64)
par = s[:W]
res = s[W:W + W // 15]
t0 = par[:, 0][par[:, 0] > 0].min()
us = lambda x: (x - t0) / 100.0  # s_memrealtime: 100 MHz


def row(name, col, a=par, rel=True):
    v = a[:, col]
    v = v[v > 0]
    if not len(v):
        return
    v = us(v) if rel else v / 100.0
    print(f"{name:34s} min {v.min():8.2f}  med {np.median(v):8.2f}  p90 {np.percentile(v, 90):8.2f}  max {v.max():8.2f}")


row("parser start", 0)
for q in range(6):
    row(f"parser round {q} aggregate", 1 + q)
row("parser drain start", 7)
row("parser done", 8)
row("parser blocking-flush us", 9, rel=False)
print("rounds flushed before drain (median):", np.median(par[:, 10]), " rounds:", np.bincount(par[:, 11]))
row("resolver G(0,b) published", 12, res)
row("resolver G(0,.) all seen", 14, res)
row("resolver round0 windows folded", 10, res)
row("resolver round0 local fold", 11, res)
row("resolver G(1,b) published", 13, res)
row("resolver G(1,.) all seen", 8, res)
row("resolver round1 windows folded", 9, res)
for q in range(8):
    row(f"resolver round {q} X posted", q, res)
