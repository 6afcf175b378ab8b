"""Per-wave phase timings of k_parse_seg (the two-segment resident pass) from bench.py --stats
stamps (100 MHz ticks), µs from the launch's first wave start.  Stamps (npr_kernels.hip,
res_capture_seg): [0] start [1] first tile landed [2] segment 0 parsed [3] A(0) published (+ the
workgroup fold by the last arriver, [12] = 1) [4] phase A done [5] past the barrier [6] wave 0:
segment-0 prefixes + T0 [7] B0 starts [8] wave 0: segment-1 prefixes [9] B0 done [10] B1 starts
[11] done; [13] ticks waiting for tiles, [14] n0, [15] tiles."""
import sys

import numpy as np

s = np.load(sys.argv[1]).astype(np.int64)
nw = int((s[:, 15] > 0).sum())
s = s[:nw]
t0 = s[:, 0].min()
S = lambda k: (s[:, k] - t0) / 100.0
pc = lambda x: " ".join(f"{v:6.2f}" for v in np.percentile(x, [0, 10, 50, 90, 99, 100]))
print(f"physical waves {nw}; tiles/wave {np.bincount(s[:, 15])[1:]}; seg-0 tiles {np.bincount(s[:, 14])[1:]}")
print("pctl             0     10     50     90     99    100")
for k, nm in [(0, "start"), (1, "landed"), (2, "seg0 parsed"), (3, "A0 pub"), (4, "A done"), (5, "barrier"),
              (7, "B0 start"), (9, "B0 done"), (10, "B1 start"), (11, "done")]:
    print(f"{nm:11s} {pc(S(k))}")
w0 = np.arange(0, nw, 16)
for k, nm in [(6, "LB0+T0 (w0)"), (8, "LB1 (w0)")]:
    print(f"{nm:11s} {pc(S(k)[w0])}")
last = s[:, 12] == 1
print(f"{'fold (last)':11s} {pc(S(3)[last] - S(2)[last])}   (us: A(0) publish + workgroup fold, last arrivers)")
print(f"{'A wait':11s} {pc(s[:, 13] / 100.0)}   (us waiting for tiles in phase A)")
for a, b, nm in [(0, 1, "first land"), (1, 2, "seg0 parse"), (3, 4, "seg1 parse"), (4, 5, "barrier"),
                 (5, 7, "-> B0"), (7, 9, "B0"), (9, 10, "B0 -> B1"), (10, 11, "B1")]:
    print(f"{nm:11s} {pc(S(b) - S(a))}")
