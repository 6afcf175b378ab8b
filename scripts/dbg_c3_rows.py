"""Debug aid: the C3 capture through the sparse walk, rows compared with the oracle row by row
(which rows, which words differ).  Usage: python scripts/dbg_c3_rows.py [n_records]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "net-parser-rs_amd"))
import _oracle  # noqa: E402
from net_parser_rs import _abi, device, synth  # noqa: E402

n_req = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000
blob = synth.variable_mix(n_req)
rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
flows, _ = _oracle.convert_records(blob, recs)
n = len(recs)
ws = device.Workspace(record_cap=n, flow_cap=n, records=False, offsets=False, status=False, flows=True, flows_v6=True)
a = np.frombuffer(blob, dtype=np.uint8)
buf = torch.empty(a.size, dtype=torch.uint8, device="cuda")
buf.copy_(torch.from_numpy(a))
ws.flows.zero_()
ws.launch(buf, start=24, endianness=hdr.endianness)
sm = ws.check()
print("pass", ws.ctx.lib.npr_ctx_last_pass(ws.ctx.handle), "n", sm.n_records, n, "flows", sm.n_flows, "cons", sm.consumed, cons)
got = np.frombuffer(ws.flows_np().tobytes(), dtype=np.uint32).reshape(-1, 8)
exp = np.frombuffer(flows.tobytes(), dtype=np.uint32).reshape(-1, 8)
bad = np.nonzero((got != exp).any(axis=1))[0]
print("rows", len(exp), "bad rows", len(bad))
if len(bad):
    print("first/last bad", bad[:20], bad[-5:])
    w = (got[bad] != exp[bad])
    print("words differing (count per word)", w.sum(axis=0))
    print("got all-zero rows", int((got[bad] == 0).all(axis=1).sum()))
    for r in bad[:6]:
        print(r, "exp", [hex(x) for x in exp[r]], "got", [hex(x) for x in got[r]])
    d = np.diff(bad)
    print("gaps between bad rows (hist of first 200)", np.unique(d[:200], return_counts=True))
