"""Wave-0 publication timeline of the r6_finestamps DIAG variant (stamps [2] phase A done, [10]
after the publication barrier, [11] after the workgroup fold, [3] published, [12] look-back start),
per workgroup, relative to the workgroup's last phase A and to the launch's last phase A."""
import sys

import numpy as np

s = np.load(sys.argv[1]).astype(np.int64)
nw = int((s[:, 8] > 0).sum())
s = s[:nw]
nb = nw // 16
A = s[:, 2].reshape(nb, 16)
last_wg = A.max(axis=1)
w0 = s[np.arange(0, nw, 16)]
last_all = A.max()


def pc(x):
    return " ".join(f"{v:6.2f}" for v in np.percentile(x / 100.0, [0, 10, 50, 90, 99, 100]))


print("pctl (us)                          0     10     50     90     99    100")
print(f"barrier - WG's last A      {pc(w0[:, 10] - last_wg)}")
print(f"fold done - barrier        {pc(w0[:, 11] - w0[:, 10])}")
print(f"published - fold done      {pc(w0[:, 3] - w0[:, 11])}")
print(f"lookback start - published {pc(w0[:, 12] - w0[:, 3])}")
print(f"WG's last A - launch last A {pc(last_wg - last_all)}")
print(f"wave 0 A - WG's last A     {pc(w0[:, 2] - last_wg)}")
