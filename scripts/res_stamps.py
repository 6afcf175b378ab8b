"""Per-wave phase timings of k_parse_resident from bench.py --stats stamps (100 MHz ticks).
[0] start [1] first tile landed [2] phase A done [3] A published + group fold [4] prefix known
[5] kept flows written (fast path) [6] done; [8] tiles [9] kept rounds [10] deferred tiles [11] fast
[15] ticks phase A spent waiting for its tiles to land, [7] ticks walking the chain"""
import sys

import numpy as np

s = np.load(sys.argv[1]).astype(np.int64)
nw = int((s[:, 8] > 0).sum())
s = s[:nw]
t0 = s[:, 0].min()
S = lambda k: (s[:, k] - t0) / 100.0
pc = lambda x: " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
print(f"waves {nw}; tiles/wave {np.bincount(s[:, 8])[1:]}; kept rounds {np.bincount(s[:, 9])}; "
      f"deferred tiles {int(s[:, 10].sum())}; fast {int(s[:, 11].sum())}")
print("pctl            0     10     50     90     99    100")
for k, nm in [(0, "start"), (1, "landed"), (2, "A done"), (3, "published"), (4, "prefix"), (6, "done")]:
    print(f"{nm:10s} {pc(S(k))}")
print(f"{'A wait':10s} {pc(s[:, 15] / 100.0)}   (us waiting for tiles in phase A)")
print(f"{'A walk':10s} {pc(s[:, 7] / 100.0)}   (us walking the chain in phase A)")
for a, b, nm in [(0, 1, "first land"), (1, 2, "phase A"), (2, 3, "pub+fold"), (3, 4, "prefix wait"), (4, 6, "write")]:
    print(f"{nm:10s} {pc(S(b) - S(a))}")
w0 = np.arange(0, nw, 16)
if len(w0):
    A = S(2)
    amax = np.array([A[i:i + 16].max() for i in w0])
    print("workgroup wave 0 (last A in the workgroup = 0):")
    for k, nm in [(3, "arrived"), (12, "lookback"), (13, "G landed"), (14, "E folded"), (4, "prefix")]:
        print(f"  {nm:10s} {pc(S(k)[w0] - amax.max())}   (rel. to the last A of the launch)")
