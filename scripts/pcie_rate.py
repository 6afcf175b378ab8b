"""PCIe-inclusive rate of the host entry point npr_parse_extract (host capture in, host flow table
out), with and without the overlapped chunked copy (NPR_OPT_STREAM_CHUNK).  Not the bench value:
DESIGN.md §4 quotes it next to the device-resident rate.  Usage (GPU box):
    python scripts/pcie_rate.py [--records N] [--config c2|c3] [--reps R]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import _abi, device, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["c2", "c3"], default="c2")
    ap.add_argument("--records", type=int, default=None)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    n = args.records or (4_000_000 if args.config == "c2" else 2_000_000)
    blob = synth.fixed64(n) if args.config == "c2" else synth.variable_mix(n)
    a = np.frombuffer(blob, dtype=np.uint8)
    ctx = npr.context(0)
    out = {"config": args.config, "records": n, "capture_bytes": len(blob), "runs": {}}
    for kib in (0, 8 << 10, 32 << 10, 128 << 10):
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, kib))
        device.host_parse_extract(a, with_v6=False, ctx=ctx)  # warm-up (allocations)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            flows, _, n_flows, consumed, _ = device.host_parse_extract(a, with_v6=False, ctx=ctx)
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        out["runs"][f"chunk_{kib}KiB" if kib else "one_copy"] = {
            "s": round(t, 5), "Mpackets_per_s": round(n / t / 1e6, 1),
            "capture_GBps": round(len(blob) / t / 1e9, 2),
            "flows_out_GBps": round(32 * n_flows / t / 1e9, 2)}
        print(json.dumps({"chunk_KiB": kib, **out["runs"][f"chunk_{kib}KiB" if kib else "one_copy"]}), flush=True)
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, 0))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
