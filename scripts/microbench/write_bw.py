"""Write-only and read-only HBM bandwidth on this box (torch fill_ / sum over uint8 buffers), the
numbers the C2 write tail is compared with in DESIGN.md §5.  python scripts/microbench/write_bw.py"""
import json

import torch

dev = torch.device("cuda", 0)
out = {}
for mb in (32, 128, 1024):
    n = mb << 20
    bufs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(max(1, 512 // mb))]  # rotate past the MALL
    for b in bufs:
        b.fill_(1)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 40
    e0.record()
    for i in range(reps):
        bufs[i % len(bufs)].fill_(i & 0xff)
    e1.record()
    torch.cuda.synchronize()
    w = n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    f32 = [b.view(torch.float32) for b in bufs]
    e0.record()
    for i in range(reps):
        f32[i % len(f32)].sum()
    e1.record()
    torch.cuda.synchronize()
    r = n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    out[f"{mb}MB"] = {"write_TBps": round(w, 2), "read_TBps": round(r, 2)}
print(json.dumps(out))
