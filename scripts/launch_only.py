"""Launch the device parse N times on the C2 capture (no result checks): a rocprofv3 target for
timing ablation / variant libraries (NPR_LIB)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
from net_parser_rs import device, synth  # noqa: E402

n = int(os.environ.get("NPR_RECORDS", "1000000"))
blob = synth.fixed64(n)
dev = torch.device("cuda", 0)
bufs = [torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev) for _ in range(4)]
ws = device.Workspace(record_cap=n, flow_cap=n, device=0, records=False, offsets=False, status=False,
                      flows=True, flows_v6=True)
for i in range(60):
    ws.launch(bufs[i % 4], start=24)
torch.cuda.synchronize()
