"""Timing aid for k_convert_records on C2 (1M x 64-B records): npr_dev_convert_records with its
rows written (cap = n) and with none (cap = 0: decode + look-back only), beside
npr_dev_extract_flows, each over COPIES rotated capture + record copies (COPIES = 4: 416 MB, past
the 256 MiB Infinity Cache; COPIES = 1: the records API bench's resident case).  NPR_LIB selects a
library variant.  python scripts/cvt_breakdown.py [COPIES [RECORDS]]"""
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
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
steps = 40
blob = synth.fixed64(n)
rc, _, recs, _ = _oracle.capture_file_parse(blob)
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
bufs = [torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev) for _ in range(copies)]
drs = [torch.from_numpy(recs.view(np.uint8).copy()).to(dev) for _ in range(copies)]
out, out6 = (torch.empty(n * 32, dtype=torch.uint8, device=dev) for _ in range(2))
st = torch.empty(n, dtype=torch.uint8, device=dev)
ctx = npr.context(0)
want, _ = _oracle.convert_records(blob, recs)
_, _, k = device.dev_convert_records(bufs[0], drs[0], cap=n, out=out, out_v6=out6, ctx=ctx, stream=s)
torch.cuda.synchronize()
correct = int(k.item()) == len(want) and out.cpu().numpy().tobytes() == want.tobytes()


def timed(fn):
    for i in range(copies):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for i in range(steps):
        fn(i % copies)
    e1.record(s)
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / steps * 1e3, 2)


res = {"lib": os.path.basename(os.environ.get("NPR_LIB", "libnpr.so")), "copies": copies, "records": n, "rows_correct": correct,
       "convert_us": timed(lambda i: device.dev_convert_records(bufs[i], drs[i], cap=n, out=out, out_v6=out6, ctx=ctx,
                                                                stream=s)),
       "convert_cap0_us": timed(lambda i: device.dev_convert_records(bufs[i], drs[i], cap=0, out=out, out_v6=out6,
                                                                     ctx=ctx, stream=s)),
       "extract_us": timed(lambda i: device.dev_extract_flows(bufs[i], drs[i], out, out6, st, ctx=ctx, stream=s))}
print(json.dumps(res), flush=True)
