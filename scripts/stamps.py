"""Summarise per-tile phase stamps written by `bench.py --stats` (gpurun_out/stamps_rank0.npy)."""
import sys

import numpy as np

s = np.load(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps_rank0.npy").astype(np.int64)
if len(sys.argv) > 2 and sys.argv[2] == "pipe":  # [0] iter start [1] decoded [2] resolved [3] written
    t0 = s[:, 0].min()
    st = (s[:, :4] - t0) / 100.0
    print("tiles", len(st), "span us %.2f" % st[:, 3].max())
    for i, nm in enumerate(["phase1", "until resolved", "outputs"]):
        d = st[:, i + 1] - st[:, i]
        print(f"{nm:15s} mean {d.mean():6.2f} med {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    sp = (s[:, 4] - s[:, 0]) / 100.0
    wk = (s[:, 5] - s[:, 4]) / 100.0
    dc = (s[:, 1] - s[:, 5]) / 100.0
    for nm, d in (("  spec", sp), ("  walk", wk), ("  decode+park", dc)):
        print(f"{nm:15s} mean {d.mean():6.2f} med {np.median(d):6.2f} p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f}")
    for q in np.linspace(0, len(st) - 1, 9).astype(int):
        print(q, "start %.2f decoded %.2f resolved %.2f written %.2f" % tuple(st[q]))
    sys.exit(0)
t0 = s[:, 0].min()
st = (s[:, :6] - t0) / 100.0  # us (s_memrealtime = 100 MHz)
print("tiles", len(st), "span us %.2f" % st[:, 5].max())
ph = np.diff(st, axis=1)
for i, nm in enumerate(["stage", "spec", "walk+count", "lookback", "output"]):
    print(f"{nm:12s} mean {ph[:, i].mean():6.2f} med {np.median(ph[:, i]):6.2f} p90 {np.percentile(ph[:, i], 90):6.2f}"
          f" max {ph[:, i].max():6.2f}")
print("life mean %.2f" % (st[:, 5] - st[:, 0]).mean(), " spins/tile %.2f" % (s[:, 7] & 0xFFFFF).mean())
for q in np.linspace(0, len(st) - 1, 9).astype(int):
    print(q, "start %.2f staged %.2f spec %.2f counted %.2f prefix %.2f end %.2f" % tuple(st[q]))
ts = np.arange(0, st[:, 5].max(), max(st[:, 5].max() / 30, 0.5))
print("active", [int(((st[:, 0] <= x) & (st[:, 5] > x)).sum()) for x in ts])
