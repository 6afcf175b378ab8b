"""Device-to-device copy rate on this box (torch copy_ of uint8 buffers, read + write counted), the
floor k_sparse_rows (a permuting copy of C3's 32-B slots) is compared with in DESIGN.md §3.8.
python scripts/microbench/copy_bw.py"""
import json

import torch

dev = torch.device("cuda", 0)
out = {}
for mb in (64, 264, 1024):
    n = mb << 20
    k = max(2, 1024 // mb)  # rotate over buffers larger than the MALL together
    src = [torch.empty(n, dtype=torch.uint8, device=dev).fill_(1) for _ in range(k)]
    dst = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(k)]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    for i in range(3):
        dst[i % k].copy_(src[i % k])
    e0.record()
    for i in range(reps):
        dst[i % k].copy_(src[(i + 1) % k])
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    out[f"{mb}MB"] = {"us_per_copy": round(ms * 1e3, 1), "read_plus_write_TBps": round(2 * n / (ms * 1e-3) / 1e12, 2)}
print(json.dumps(out))
