"""Where a bench step's time goes outside the kernels: host cost of one launch call, per-step event
overhead, and the GPU-side step period with and without events (C2 workload, as bench.py)."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import device, synth  # noqa: E402

n = 1_000_000
blob = synth.fixed64(n)
dev = torch.device("cuda", 0)
bufs = [torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev) for _ in range(4)]
hdr = npr.GlobalHeader.parse(blob[:24])[1]
ws = device.Workspace(record_cap=n, flow_cap=n, device=0, records=False, offsets=False, status=False,
                      flows=True, flows_v6=True)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
e = hdr.endianness
for i in range(20):
    ws.launch(bufs[i % 4], start=24, endianness=e)
torch.cuda.synchronize()
K = 200


def period(events):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a.record(stream)
    for i in range(K):
        if events:
            ev[i][0].record(stream)
        ws.launch(bufs[i % 4], start=24, endianness=e)
        if events:
            ev[i][1].record(stream)
    b.record(stream)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6, a.elapsed_time(b) / K * 1e3


for events in (True, False, True, False):
    host, wall, gpu = period(events)
    print(f"events={events!s:5s} host-submit {host:6.1f} us/step  wall {wall:6.1f} us/step  gpu-span {gpu:6.1f} us/step")
# host cost of the bare C call (queue kept shallow: sync every 8)
t = 0.0
for r in range(25):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(8):
        ws.launch(bufs[i % 4], start=24, endianness=e)
    t += time.perf_counter() - t0
print(f"host cost of ws.launch (shallow queue): {t / 200 * 1e6:.1f} us")
