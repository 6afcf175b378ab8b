"""Per-wave phase timings of k_parse_resident from bench.py --stats stamps (100 MHz ticks).
[0] start [1] first tile landed [2] phase A done [3] A published + group fold (wave 0 of each
workgroup only) [4] prefix known [5] kept flows written (fast path) [6] done; [8] tiles [9] kept
rounds [10] deferred tiles [11] fast; [12] look-back start [13] lower aggregates all landed
[14] workgroup prefix folded (wave 0 only); [15] ticks phase A spent waiting for its tiles to land,
[7] ticks walking the chain.  A stamp a wave does not write reads 0: every percentile below is
taken over the waves that wrote it (the round-4 version subtracted unset stamps)."""
import sys

import numpy as np

s = np.load(sys.argv[1]).astype(np.int64)
nw = int((s[:, 8] > 0).sum())
s = s[:nw]
t0 = s[:, 0][s[:, 0] > 0].min()


def S(k, rows=None):
    x = s[:, k] if rows is None else s[rows, k]
    x = x[x > 0]
    return (x - t0) / 100.0


def pc(x):
    if len(x) == 0:
        return "   (no stamps)"
    return " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))


def D(a, b, rows=None):  # per-wave b - a over the waves that wrote both
    x = s[:, [a, b]] if rows is None else s[rows][:, [a, b]]
    m = (x[:, 0] > 0) & (x[:, 1] > 0)
    return (x[m, 1] - x[m, 0]) / 100.0


w0 = np.arange(0, nw, 16)
print(f"waves {nw}; tiles/wave {np.bincount(s[:, 8])[1:]}; kept rounds {np.bincount(s[:, 9])}; "
      f"deferred tiles {int(s[:, 10].sum())}; fast {int(s[:, 11].sum())}")
print("pctl            0     10     50     90     99    100")
for k, nm, rows in [(0, "start", None), (1, "landed", None), (2, "A done", None), (3, "published", w0),
                    (4, "prefix", None), (6, "done", None)]:
    print(f"{nm:10s} {pc(S(k, rows))}")
print(f"{'A wait':10s} {pc(s[:, 15] / 100.0)}   (us waiting for tiles in phase A)")
print(f"{'A walk':10s} {pc(s[:, 7] / 100.0)}   (us walking the chain in phase A; general loop only)")
for a, b, nm, rows in [(0, 1, "first land", None), (1, 2, "phase A", None), (2, 3, "pub+fold", w0),
                       (3, 4, "prefix wait", w0), (4, 6, "write", None)]:
    print(f"{nm:10s} {pc(D(a, b, rows))}")
if len(w0):
    A = s[:, 2]
    last_a = A[A > 0].max()
    print("workgroup wave 0 (relative to the last phase A of the launch):")
    for k, nm in [(3, "arrived"), (12, "lookback"), (13, "G landed"), (14, "E folded"), (4, "prefix")]:
        x = s[w0, k]
        x = x[x > 0]
        print(f"  {nm:10s} {pc((x - last_a) / 100.0)}")
