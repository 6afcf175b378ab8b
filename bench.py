"""bench.py — device-resident record parse + extract_flow (+ convert_records) on MI355X.

One "step" = one launch of the resident single-pass HIP kernel (k_parse_resident) over one capture
already resident in HBM: CaptureFile::parse (record chain) + extract_flow for every record +
convert_records (Ok flows, reverse order), i.e. the reference's `extract` bench
(benches/benches.rs:40-74).

Workload (BASELINE.json configs[1], "C2"): 1,000,000 synthetic 64-B Ethernet/IPv4/TCP records per
GPU (80,000,024 B capture).  N > 1: one process per GPU, each parses its own 1M-record shard
(weak scaling, no collective in the timed region).  Steps rotate over 4 copies of the capture
(4 x 80 MB > the 256 MiB Infinity Cache together with the outputs) so every step reads HBM.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import net_parser_rs as npr  # noqa: E402
from net_parser_rs import device, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "Mpackets/s + GB/s, device-resident record parse+extract_flow, 1M×64B batch"


def cpu_baseline(blob, n_records, budget_s):
    """The CPU oracle (C restatement of the reference path, tests/_oracle.py) on 1 core."""
    import _oracle
    rec = np.zeros(n_records + 1, dtype=npr._abi.RECORD_DTYPE)
    fl = np.zeros(n_records + 1, dtype=npr._abi.FLOW_DTYPE)
    v6 = np.zeros(n_records + 1, dtype=npr._abi.FLOW_V6_DTYPE)
    _oracle.bench_extract(blob, rec, fl, v6)  # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        k, nr = _oracle.bench_extract(blob, rec, fl, v6)
        passes += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    assert nr == n_records
    rate = passes * n_records / el / 1e6
    return {"value": round(rate, 3), "unit": "Mpackets/s", "cores": 1, "kind": "port",
            "sample": f"C2 capture ({n_records} records, {len(blob)} B) x {passes} passes, "
                      f"CaptureFile::parse + convert_records, {el:.1f} s on 1 host core"}


def pmc_traffic(records):
    """HBM-side bytes per launch from the newest committed PMC summary of this workload (profiles/),
    or None.  Collected by scripts/pmc.sh: FETCH_SIZE x2 + WRITE_SIZE summed over both kernels."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_pmc_summary.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if records == 1_000_000 and d.get("workload", "").startswith("C2"):
            return d.get("traffic_bytes_per_launch"), os.path.basename(f)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["c2", "c3"], default="c2",
                    help="c2 (the headline: 1M x 64-B records) or c3 (8M records, frames U[64,1500], ~6.4 GB; "
                         "parsed as chained ~80 MB launches)")
    ap.add_argument("--records", type=int, default=None)
    ap.add_argument("--copies", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stats", action="store_true", help="print speculation / hand-off counters (stderr)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    c3 = args.config == "c3"
    n = args.records or (8_000_000 if c3 else 1_000_000)
    copies = args.copies or (1 if c3 else 4)
    # same capture on every rank: each GPU parses its own shard
    blob = synth.variable_mix(n) if c3 else synth.fixed64(n)
    host = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    bufs = [host.to(dev) for _ in range(copies)]
    hdr = npr.GlobalHeader.parse(blob[:24])[1]
    ws = device.Workspace(record_cap=n, flow_cap=n, device=local, records=False, offsets=False, status=False,
                          flows=True, flows_v6=True)
    stream = torch.cuda.Stream(dev)  # an explicit stream: events bracket exactly our launches
    torch.cuda.set_stream(stream)

    # correctness gate for the measured configuration
    ws.launch(bufs[0], start=24, endianness=hdr.endianness)
    sm = ws.check()
    # C2: every record is an Ok flow; C3: short TCP frames with a long data offset are not (Q9)
    assert sm.n_records == n and sm.consumed == len(blob) and (sm.n_flows == n or c3), (sm.n_records, sm.n_flows)
    n_flows = int(sm.n_flows)

    for i in range(args.warmup):
        ws.launch(bufs[i % copies], start=24, endianness=hdr.endianness)
    torch.cuda.synchronize()

    # ONE event pair brackets the K launches on their stream (per-step events would add marker
    # packets between launches: ~8 us of GPU time per step, scripts/launch_probe.py)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        ws.launch(bufs[i % copies], start=24, endianness=hdr.endianness)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    sm = ws.check()
    assert sm.n_records == n and sm.n_flows == n_flows
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # average launch (scan + emit) on the device
    if args.stats:
        import ctypes
        lib, h = ws.ctx.lib, ws.ctx.handle
        ws.ctx.check(lib.npr_ctx_set_stats(h, 2))
        for i in range(3):
            ws.launch(bufs[i % copies], start=24, endianness=hdr.endianness)
        ws.check()
        st = (ctypes.c_uint32 * 8)()
        ws.ctx.check(lib.npr_ctx_read_stats(h, st, 8, 1))
        ntl = ctypes.c_uint64(0)
        ws.ctx.check(lib.npr_ctx_read_stamps(h, None, 0, ctypes.byref(ntl)))  # tile count of the last launch
        nt = ntl.value
        stamps = np.zeros(nt * 16, dtype=np.uint64)
        ws.ctx.check(lib.npr_ctx_read_stamps(h, stamps.ctypes.data, stamps.size, ctypes.byref(ntl)))
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        np.save(os.path.join(REPO, "gpurun_out", f"stamps_rank{rank}.npy"), stamps.reshape(nt, 16))
        print(f"[rank {rank}] stats rewalk={st[0]} mism_wait={st[1]} none={st[5]} tiles={nt}", file=sys.stderr, flush=True)
        ws.ctx.check(lib.npr_ctx_set_stats(h, 0))

    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern_ms = float(t[0]), float(t[1])

    if rank == 0:
        ms_per_step = wall * 1e3 / args.steps
        total_records = n * world * args.steps
        value = total_records / wall / 1e6
        stream_bytes = len(blob) - 24                       # sum(16 + incl_len) per capture
        read_b = len(blob)                                  # every byte of the capture is read (C2:
        # = SURVEY 8d's 16 + min(incl, 64) per record; C3: the tiles stream whole payloads too)
        write_b = 32 * n_flows                              # one 32-B npr_flow per Ok record
        alg = read_b + write_b
        achieved = alg / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src = pmc_traffic(n) if not c3 else (None, None)
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpackets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (numpy PCG64 seed 0x4E50; C2 layout of SURVEY.md 8d)",
            "config": {"workload": ("C3: 8M records, frames U[64,1500] B, IPv4 TCP|UDP per GPU, device-resident"
                                    if c3 else "C2: 1M x 64-B Ethernet/IPv4/TCP records per GPU, device-resident"),
                       "records_per_gpu": n, "capture_bytes": len(blob), "parallelism": f"record-range x{world}",
                       "outputs": "convert_records flow table (32 B/flow incl. record offset)"},
            "stream_GBps": round(stream_bytes * world * args.steps / wall / 1e9, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "read_only_frac": round(read_b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "bytes_per_launch": alg, "kernel_ms": round(kern_ms, 5)},
        }
        if not args.no_cpu and not c3:
            out["cpu_baseline"] = cpu_baseline(blob, n, args.cpu_budget)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
