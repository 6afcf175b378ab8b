"""A capture past 2 GiB through the device path (flows-only chunked resident pass, and the
two-pass kernels), checked against the oracle's counts."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import _oracle  # noqa: E402
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import _abi, device, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000
blob = synth.variable_mix(n)
rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
print("oracle", len(recs), cons, len(blob), flush=True)
buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
for mode in ("resident", "two_pass"):
    ctx = npr.context(0)
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 1 if mode == "resident" else 0))
    ws = device.Workspace(n + 1, n + 1, records=False, status=False)
    ws.launch(buf, start=24, endianness=hdr.endianness)
    try:
        sm = ws.check()
    except npr.DeviceError as e:
        sm = ws.last
        print(mode, "error", e)
    print(mode, sm.n_records, sm.n_flows, sm.consumed, sm.entry, sm.flags, flush=True)
