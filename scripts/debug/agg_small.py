# one-off: npr_dev_flow_aggregate at small row counts against the row-f4 checker
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "net-parser-rs_amd")
import numpy as np, torch
from net_parser_rs import _abi, device, synth
import _flowtable_ref
import test_gpu_flowtable as t
blob = synth.flow_mix(30_000, n_flows=700, seed=12)
fl, f6, n = t.device_table(blob)
for m in [100, 511, 512, 700, 712, 1024, 1025, 2000, 5000]:
    flows = fl[: m * 32].cpu().numpy().view(_abi.FLOW_DTYPE)
    v6 = f6[: m * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
    want, counts = _flowtable_ref.aggregate(flows, v6, None)
    res = []
    for w in (None, torch.ones(m, dtype=torch.int64, device="cuda")):
        out, out6, cnt, n_out = device.dev_flow_aggregate(fl[: m * 32].contiguous(), f6[: m * 32].contiguous(), n=m, weights=w)
        res.append(int(n_out.item()))
    print(m, len(want), res, flush=True)
