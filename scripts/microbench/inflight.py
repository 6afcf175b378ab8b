"""C2 steps with D launches in flight: D workspaces (contexts), each on its own stream, steps dealt
round-robin.  Consecutive batches are independent captures, so step k+1's workgroups may take the
CUs that step k's workgroups free as they finish their rows (its prefix and write tail).

python scripts/microbench/inflight.py --depth 1 2 3 --steps 400

Measured: depth 2 DEADLOCKS until the kernels' 1-s bounded waits abort them (the
call then fails with "tile hand-off timed out"): each XCD dispatches its share of a launch's
workgroups in order, so two resident launches can each hold CUs the other's lower workgroups need.
Kept as the record of that experiment; depth 1 is the bench's loop.
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import device, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--records", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    blob = synth.fixed64(args.records)
    host = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    bufs = [host.to(dev) for _ in range(args.copies)]
    n = args.records
    for D in args.depth:
        wss = [device.Workspace(record_cap=n, flow_cap=n, device=0, records=False, offsets=False, status=False,
                                flows=True, flows_v6=True) for _ in range(D)]
        streams = [torch.cuda.Stream(dev) for _ in range(D)]
        for i in range(20):
            wss[i % D].launch(bufs[i % args.copies], start=24, stream=streams[i % D])
        torch.cuda.synchronize()
        for ws in wss:
            sm = ws.check()
            assert sm.n_records == n and sm.n_flows == n
        res = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                wss[i % D].launch(bufs[i % args.copies], start=24, stream=streams[i % D])
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) / args.steps * 1e6)
        for ws in wss:
            sm = ws.check()
            assert sm.n_records == n and sm.n_flows == n
        us = min(res)
        print(json.dumps({"depth": D, "us_per_step": [round(r, 2) for r in res],
                          "Gpps": round(n / us / 1e3, 2), "frac": round(112e6 / (us * 1e-6) / 8e12, 4)}), flush=True)
        del wss


if __name__ == "__main__":
    main()
