"""Per-workgroup stamps of k_convert_records (library built with scripts/variants/cv_stamp.py:
NPR_LIB=.../libnpr_cv_stamp.so): for one launch after warm-up over COPIES rotated inputs, the
spread of {decoded, prefix known, rows issued} relative to the launch's first workgroup start, in
us (s_memrealtime, 100 MHz).  python scripts/cvt_stamps.py [COPIES [RECORDS_PER_WORKGROUP]]"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _oracle  # noqa: E402
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import device, synth  # noqa: E402

copies = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = 1_000_000
blob = synth.fixed64(n)
_, _, recs, _ = _oracle.capture_file_parse(blob)
dev = torch.device("cuda", 0)
bufs = [torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev) for _ in range(copies)]
drs = [torch.from_numpy(recs.view(np.uint8).copy()).to(dev) for _ in range(copies)]
out, out6 = (torch.empty(n * 32, dtype=torch.uint8, device=dev) for _ in range(2))
ctx = npr.context(0)
rpb = min(max(-(-(-(-n // 256)) // 256) * 256, 1024), 4096)  # launch_convert_records on 256 CUs
per = int(sys.argv[2]) if len(sys.argv) > 2 else rpb  # records per workgroup
nb = (n + per - 1) // per
res = {"copies": copies, "workgroups": nb}
stages = ("decoded", "prefix", "end")
acc = {k: [] for k in stages}
for it in range(3 * copies + 5):
    device.dev_convert_records(bufs[it % copies], drs[it % copies], cap=n, out=out, out_v6=out6, ctx=ctx)
    torch.cuda.synchronize()
    if it < 2 * copies:
        continue
    st = out6.view(torch.int64)[: nb * 4].view(nb, 4).cpu().numpy().astype(np.float64)
    t = (st - st[:, 0].min()) / 100.0  # us
    for k, col in zip(stages, (1, 2, 3)):
        acc[k].append(t[:, col])
    acc.setdefault("start", []).append(t[:, 0])
    acc.setdefault("wait", []).append(t[:, 2] - t[:, 1])
    last = t
j = np.arange(nb)
res["decoded_by_xcd_med"] = [round(float(np.median(last[j % 8 == x, 1])), 2) for x in range(8)]
res["decoded_by_j_octile_med"] = [round(float(np.median(last[(j * 8) // nb == q, 1])), 2) for q in range(8)]
res["decode_time_by_j_octile_med"] = [round(float(np.median(last[(j * 8) // nb == q, 1] - last[(j * 8) // nb == q, 0])), 2)
                                      for q in range(8)]
res["decoded_slowest_j"] = [int(x) for x in np.argsort(last[:, 1])[-16:]]
np.save(os.path.join(REPO, "gpurun_out", f"cvt_stamps_{copies}.npy"), last)
for k, v in acc.items():
    a = np.concatenate(v)
    res[k] = {p: round(float(np.percentile(a, q)), 2) for p, q in (("min", 0), ("p10", 10), ("med", 50), ("p90", 90), ("max", 100))}
print(json.dumps(res), flush=True)
