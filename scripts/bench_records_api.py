"""Per-record entry points on the C2 capture (1M x 64-B records): device time of
npr_dev_convert_records and npr_dev_extract_flows (HIP events around K launches on one stream),
the host-memory npr_convert_records call (PCIe included), and the CPU oracle's convert_records
over the same record list.  Prints one JSON line.

Algorithmic bytes per record: 24 (the npr_record row) + 64 (the frame the decode reads) read;
written: convert 32 per Ok row (+ 32 for an IPv6 flow's side row), dense extract 32 per record
(+ 32 for an IPv6 flow's side row) + 1 B of status: 121 B per C2 record.  Usage: python scripts/bench_records_api.py [--records N] [--steps K] [--rounds R]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import _oracle  # noqa: E402
import net_parser_rs as npr  # noqa: E402
from net_parser_rs import _abi, device, synth  # noqa: E402


def timed_events(fn, steps, stream):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


# kernel_ms: the same capture and record list every launch (they stay in the 256 MiB Infinity
# Cache); kernel_ms_hbm: launches rotate over 4 copies (416 MB), so every launch reads HBM.


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=7, help="interleaved repetitions of the device timings (median + range)")
    args = ap.parse_args()
    n = args.records
    blob = synth.fixed64(n)
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert rc == 0 and len(recs) == n
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    buf = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(dev)
    drecs = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
    out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    out6 = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    f = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    f6 = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    ctx = npr.context(0)

    # correctness gate: the measured launch against the oracle
    want_f, want_v6 = _oracle.convert_records(blob, recs)
    _, _, n_out = device.dev_convert_records(buf, drecs, cap=n, out=out, out_v6=out6, ctx=ctx, stream=stream)
    torch.cuda.synchronize()
    assert int(n_out.item()) == len(want_f) and out.cpu().numpy().tobytes() == want_f.tobytes()

    # the same launches over 4 rotated copies of capture + records (416 MB, past the 256 MiB
    # Infinity Cache, as bench.py rotates its captures): every launch reads HBM.  The four timings
    # are interleaved `--rounds` times; each is reported as the median with its range (VERDICT r05:
    # the documents quote this file, not a best run)
    bufs = [buf] + [buf.clone() for _ in range(3)]
    drs = [drecs] + [drecs.clone() for _ in range(3)]
    it = iter(range(1 << 30))
    runs = {"cvt": [], "ext": [], "cvt_hbm": [], "ext_hbm": []}
    for _ in range(args.rounds):
        runs["cvt"].append(timed_events(lambda: device.dev_convert_records(buf, drecs, cap=n, out=out, out_v6=out6,
                                                                           ctx=ctx, stream=stream), args.steps, stream))
        runs["ext"].append(timed_events(lambda: device.dev_extract_flows(buf, drecs, f, f6, st, ctx=ctx, stream=stream),
                                        args.steps, stream))
        runs["cvt_hbm"].append(timed_events(
            lambda: (lambda i: device.dev_convert_records(bufs[i], drs[i], cap=n, out=out, out_v6=out6, ctx=ctx,
                                                          stream=stream))(next(it) % 4), args.steps, stream))
        runs["ext_hbm"].append(timed_events(
            lambda: (lambda i: device.dev_extract_flows(bufs[i], drs[i], f, f6, st, ctx=ctx, stream=stream))(next(it) % 4),
            args.steps, stream))
    med = {k: float(np.median(v)) for k, v in runs.items()}
    rng = {k: [round(min(v), 5), round(max(v), 5)] for k, v in runs.items()}
    cvt_ms, ext_ms, cvt_cold_ms, ext_cold_ms = med["cvt"], med["ext"], med["cvt_hbm"], med["ext_hbm"]
    del bufs[1:], drs[1:]
    # host-memory call (pageable buffers; PCIe in and out)
    a = np.frombuffer(blob, np.uint8)
    hf = np.zeros(n, _abi.FLOW_DTYPE)
    h6 = np.zeros(n, _abi.FLOW_V6_DTYPE)
    k = ctypes.c_size_t(0)
    call = lambda: ctx.check(ctx.lib.npr_convert_records(ctx.handle, a.ctypes.data, a.size, recs.ctypes.data, n,
                                                         hf.ctypes.data, h6.ctypes.data, n, ctypes.byref(k)))
    call()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        call()
    host_ms = (time.perf_counter() - t0) * 1e3 / reps
    assert k.value == len(want_f) and hf.tobytes() == want_f.tobytes()
    # FlowExtraction::extract_flow one record at a time (what the Rust crate's per-record trait
    # method does): one npr_extract_flows host call per record, its 80-B record as the input
    one = np.frombuffer(blob, np.uint8)[24:24 + 80].copy()
    r1 = np.zeros(1, _abi.RECORD_DTYPE)
    r1[0] = (0, 0, 0, 64, 64)
    f1 = np.zeros(1, _abi.FLOW_DTYPE)
    v1 = np.zeros(1, _abi.FLOW_V6_DTYPE)
    s1 = np.zeros(1, np.uint8)
    call1 = lambda: ctx.check(ctx.lib.npr_extract_flows(ctx.handle, one.ctypes.data, one.size, r1.ctypes.data, 1,
                                                        f1.ctypes.data, v1.ctypes.data, s1.ctypes.data))
    call1()
    reps1 = 200
    t0 = time.perf_counter()
    for _ in range(reps1):
        call1()
    per_call_us = (time.perf_counter() - t0) * 1e6 / reps1
    assert s1[0] == 0 and f1[0].tobytes()[:27] == want_f[-1].tobytes()[:27]  # record 0 (the last row), offset aside
    # the CPU oracle on the same list
    t0 = time.perf_counter()
    passes = 0
    while time.perf_counter() - t0 < 5.0:
        _oracle.convert_records(blob, recs)
        passes += 1
    cpu_ms = (time.perf_counter() - t0) * 1e3 / passes

    # row f4: the distinct-flow table over the convert_records table just made (C2: all distinct) and
    # over a Zipf mix of 5000 5-tuples
    agg_ms = timed_events(lambda: device.dev_flow_aggregate(out, out6, n=n, ctx=ctx, stream=stream), args.steps, stream)
    mix = synth.flow_mix(n, n_flows=5000)
    rcm, _, recm, _ = _oracle.capture_file_parse(mix)
    fm, f6m = _oracle.convert_records(mix, recm)
    fmt = torch.from_numpy(fm.view(np.uint8).copy()).to(dev)
    f6t = torch.from_numpy(f6m.view(np.uint8).copy()).to(dev)
    nm = len(fm)
    agg_mix_ms = timed_events(lambda: device.dev_flow_aggregate(fmt, f6t, n=nm, ctx=ctx, stream=stream), args.steps,
                              stream)
    n6 = int(((want_f["kind"] & _abi.KIND_IPV6) != 0).sum())
    cvt_bytes = n * (24 + 64) + len(want_f) * 32 + n6 * 32  # flow rows + side rows of IPv6 flows
    ext_bytes = n * (24 + 64 + 32 + 1) + n6 * 32  # side rows of IPv6 flows only (npr.h, since round 4)
    res = {
        "workload": f"C2 record list ({n} x 64-B frames), records + capture resident in HBM",
        "timing": f"HIP events over {args.steps} launches; kernel_ms = median of {args.rounds} interleaved rounds, "
                  "kernel_ms_range = [min, max]",
        "dev_convert_records": {"kernel_ms": round(cvt_ms, 5), "Mrecords_per_s": round(n / cvt_ms / 1e3, 1),
                                "alg_bytes": cvt_bytes, "GBps": round(cvt_bytes / cvt_ms / 1e6, 1),
                                "frac_of_8TBps": round(cvt_bytes / cvt_ms / 1e6 / 8000, 4),
                                "kernel_ms_hbm": round(cvt_cold_ms, 5),
                                "frac_of_8TBps_hbm": round(cvt_bytes / cvt_cold_ms / 1e6 / 8000, 4),
                                "kernel_ms_range": rng["cvt"], "kernel_ms_hbm_range": rng["cvt_hbm"]},
        "dev_extract_flows": {"kernel_ms": round(ext_ms, 5), "Mrecords_per_s": round(n / ext_ms / 1e3, 1),
                              "alg_bytes": ext_bytes, "GBps": round(ext_bytes / ext_ms / 1e6, 1),
                              "frac_of_8TBps": round(ext_bytes / ext_ms / 1e6 / 8000, 4),
                              "kernel_ms_hbm": round(ext_cold_ms, 5),
                              "frac_of_8TBps_hbm": round(ext_bytes / ext_cold_ms / 1e6 / 8000, 4),
                              "kernel_ms_range": rng["ext"], "kernel_ms_hbm_range": rng["ext_hbm"]},
        "dev_flow_aggregate": {"c2_all_distinct_ms": round(agg_ms, 5), "zipf_5000_flows_ms": round(agg_mix_ms, 5),
                               "rows": n, "zipf_rows": nm,
                               "Mrows_per_s": round(n / agg_ms / 1e3, 1)},
        "host_extract_flow_one_record": {"us_per_call": round(per_call_us, 1),
                                         "note": "one npr_extract_flows host call per record (the Rust "
                                                 "FlowExtraction::extract_flow default method): one launch over a page-locked "
                                                 "arena + sync; use extract_flows / convert_records for batches"},
        "host_convert_records": {"ms": round(host_ms, 3), "Mrecords_per_s": round(n / host_ms / 1e3, 1),
                                 "note": "pageable host buffers: capture + records H2D, flow rows D2H"},
        "cpu_oracle_convert_records": {"ms": round(cpu_ms, 3), "Mrecords_per_s": round(n / cpu_ms / 1e3, 2),
                                       "cores": 1, "passes": passes},
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
