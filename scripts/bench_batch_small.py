"""K small captures per npr_dev_parse_extract_batch call against K single launches (written for round 3's one-launch k_parse_batch, which it retired: DESIGN.md §3.2).

The batched launch pays the launch ramp and tail once per K captures; it should pay where those
dominate: many SMALL captures.  Times K x R-record C2-shaped captures (distinct buffers, 16 rounds
rotating over 4 sets so the working set exceeds the 256 MiB Infinity Cache at large R) both ways,
with HIP events on the stream, every capture gated against the first round's rows.
Prints one JSON line per R.  Usage: python scripts/bench_batch_small.py [R ...]"""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import device, synth  # noqa: E402

K, ROUNDS, SETS = 8, 16, 4


def run(records):
    dev = torch.device("cuda", 0)
    blobs = [synth.fixed64(records, seed=100 + i) for i in range(SETS * K)]
    bufs = [torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev) for b in blobs]
    hdr = npr.GlobalHeader.parse(blobs[0][:24])[1]
    wss = [device.Workspace(records, records, records=False, offsets=False, status=False, flows=True, flows_v6=True)
           for _ in range(K)]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def single(r):
        for i in range(K):
            wss[i].launch(bufs[(r % SETS) * K + i], start=24, endianness=hdr.endianness)

    def batched(r):
        device.launch_batch([(wss[i], bufs[(r % SETS) * K + i], 24, hdr.endianness) for i in range(K)], stream=stream)

    out = {"records_per_capture": records, "captures_per_launch": K}
    for name, fn in (("single", single), ("batched", batched), ("single_again", single), ("batched_again", batched)):
        for r in range(SETS):
            fn(r)
        torch.cuda.synchronize()
        for w in wss:
            sm = w.check()
            assert sm.n_records == records and sm.n_flows == records
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for r in range(ROUNDS):
            fn(r)
        ev1.record(stream)
        torch.cuda.synchronize()
        out[f"{name}_us_per_capture"] = round(ev0.elapsed_time(ev1) * 1e3 / (ROUNDS * K), 3)
    out["batched_gain"] = round(min(out["single_us_per_capture"], out["single_again_us_per_capture"]) /
                                min(out["batched_us_per_capture"], out["batched_again_us_per_capture"]), 3)
    return out


if __name__ == "__main__":
    for r in [int(x) for x in sys.argv[1:]] or [16_384, 65_536, 262_144, 1_000_000]:
        print(json.dumps(run(r)), flush=True)
        time.sleep(0.1)
