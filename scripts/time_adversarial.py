"""Timing aid: the 300-MB quirk corpus of tests/test_gpu_scale.py::test_adversarial_300mb_auto_sparse
(fake header chains inside payloads, jumbo and zero-length records, IPv6, VLANs, ARP) through the
sparse walk (the auto choice) and the resident pass, wall time per launch (synchronised), and the
sparse scan's re-walk count.  python scripts/time_adversarial.py [big]"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "net-parser-rs_amd"))
from net_parser_rs import _abi, device, synth  # noqa: E402

big = len(sys.argv) > 1 and sys.argv[1] == "big"
blob = synth.quirk_corpus(360_000, seed=71 + big, big=big, jumbo_every=60, fake_every=7, zero_every=11,
                          tail="truncated_payload")
a = np.frombuffer(blob, dtype=np.uint8)
buf = torch.empty(a.size, dtype=torch.uint8, device="cuda")
buf.copy_(torch.from_numpy(a.copy()))
n = 400_000
ws = device.Workspace(record_cap=n, flow_cap=n, records=False, offsets=False, status=False, flows=True,
                      flows_v6=True)
lib, h = ws.ctx.lib, ws.ctx.handle
endian = _abi.BIG if big else _abi.LITTLE
out = {"bytes": len(blob), "big": big}
for name, mode in (("sparse", 0), ("resident", 1)):
    ws.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, mode))
    ws.ctx.check(lib.npr_ctx_set_stats(h, 1))
    ts = []
    for i in range(6):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ws.launch(buf, start=24, endianness=endian)
        sm = ws.check()
        ts.append(time.perf_counter() - t0)
    st = (ctypes.c_uint32 * 8)()
    ws.ctx.check(lib.npr_ctx_read_stats(h, st, 8, 1))
    ws.ctx.check(lib.npr_ctx_set_stats(h, 0))
    out[name] = {"ms_median": round(float(np.median(ts[1:])) * 1e3, 3), "pass": lib.npr_ctx_last_pass(h),
                 "records": sm.n_records, "flows": sm.n_flows, "rewalks_per_launch": st[0] / 6,
                 "scan_rounds_per_launch": st[3] / 6}
ws.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, 0))
print(json.dumps(out))
