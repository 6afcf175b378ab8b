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
    # npr_parse_extract_pipelined: page-locked chunked H2D | chained launches | per-link D2H,
    # (a) from a pageable capture (registered per call), (b) from npr_host_alloc'ed buffers
    cap = n + 1
    pin_in = device.PinnedArray(len(blob))
    pin_in.array[:] = a
    pin_out = device.PinnedArray(cap * 32, _abi.FLOW_DTYPE)
    page_out = np.zeros(cap, dtype=_abi.FLOW_DTYPE)
    for label, src, dst in (("pipelined_pageable", a, page_out), ("pipelined_pinned", pin_in.array, pin_out.array)):
        for mib in (8, 32, 128):
            device.host_parse_extract_pipelined(src, dst, None, cap, mib << 20, ctx=ctx)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                flows, _, n_flows, consumed = device.host_parse_extract_pipelined(src, dst, None, cap, mib << 20, ctx=ctx)
                ts.append(time.perf_counter() - t0)
            t = min(ts)
            key = f"{label}_{mib}MiB"
            out["runs"][key] = {"s": round(t, 5), "Mpackets_per_s": round(n / t / 1e6, 1),
                                "capture_GBps": round(len(blob) / t / 1e9, 2),
                                "flows_out_GBps": round(32 * n_flows / t / 1e9, 2)}
            print(json.dumps({"run": key, **out["runs"][key]}), flush=True)
    # the same from page-locked buffers through a bounded device window (NPR_OPT_DEVICE_WINDOW):
    # W chunk slots + 3 flow-row slots on the device, a host sync per link
    for mib, win in ((8, 4), (8, 8), (32, 3), (32, 8)):
        run = lambda: device.host_parse_extract_pipelined(pin_in.array, pin_out.array, None, cap, mib << 20, ctx=ctx,
                                                          window=win)
        run()
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            flows, _, n_flows, consumed = run()
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        key = f"windowed_pinned_{mib}MiB_x{win}"
        out["runs"][key] = {"s": round(t, 5), "Mpackets_per_s": round(n / t / 1e6, 1),
                            "capture_GBps": round(len(blob) / t / 1e9, 2),
                            "flows_out_GBps": round(32 * n_flows / t / 1e9, 2),
                            "device_window_MB": round((win * (mib << 20) + (260 << 10)) / 1e6, 1)}
        print(json.dumps({"run": key, **out["runs"][key]}), flush=True)
    # the raw link: one pinned H2D of the capture, one pinned D2H of the flow table
    import torch
    d = torch.empty(len(blob), dtype=torch.uint8, device="cuda")
    f = torch.empty(cap * 32, dtype=torch.uint8, device="cuda")
    hin = torch.from_numpy(pin_in.array)
    hout = torch.from_numpy(pin_out.array.view(np.uint8))
    for label, fn, nb in (("h2d_pinned", lambda: d.copy_(hin, non_blocking=True), len(blob)),
                          ("d2h_pinned", lambda: hout.copy_(f, non_blocking=True), cap * 32)):
        fn(); torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / args.reps
        out["runs"][label] = {"s": round(t, 5), "GBps": round(nb / t / 1e9, 2)}
        print(json.dumps({"run": label, **out["runs"][label]}), flush=True)
    pin_in.close()
    pin_out.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
