"""bench.py — device-resident record parse + extract_flow (+ convert_records) on MI355X.

One "step" = one pass of the hot path over one capture already resident in HBM: CaptureFile::parse
(record chain) + extract_flow for every record + convert_records (Ok flows, reverse order), i.e.
the reference's `extract` bench (benches/benches.rs:40-74).

Workloads (BASELINE.json configs; SURVEY.md §8 d):
  c2  (default at N=1, the headline) 1,000,000 synthetic 64-B Ethernet/IPv4/TCP records
      (80,000,024 B), one k_parse_resident launch per step; steps rotate over 4 copies of the
      capture (4 x 80 MB > the 256 MiB Infinity Cache with the outputs), so every step reads HBM.
  c3  8,000,000 records, frames U[64,1500] B, IPv4 TCP|UDP (6.4 GB): chained resident launches.
  c4  (default at N>1) the 64M x 64-B capture sharded by record range, 8M records per GPU (weak
      scaling: N=8 is exactly configs[3]).  Each rank holds ONLY its shard's file bytes; a step is
      its shard's parse (npr_dev_parse_extract_shard) + the one exchange (an RCCL all-gather of the
      device summaries, then the host replay of the serial chain).  The flow-table gather to rank 0
      over RCCL (point-to-point into the merged table) is timed separately: `gather_ms`,
      `end_to_end_Mpps`.

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
from net_parser_rs import device, parallel, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "Mpackets/s + GB/s, device-resident record parse+extract_flow, 1M×64B batch"
C4_PER_GPU = 8_000_000


def host_threads():
    """The host cores this process may use (the GPU box gives one GPU's job 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, env if env > 0 else n, 16))


def cpu_baseline(blob, n_records, budget_s, sample):
    """The CPU oracle (C restatement of the reference path, tests/_oracle.py), CaptureFile::parse +
    convert_records on the same capture: on all host threads and on one core (the reference itself
    is single-threaded, benches/benches.rs); the faster of the two is the reported baseline."""
    import _oracle
    rec = np.zeros(n_records + 1, dtype=npr._abi.RECORD_DTYPE)
    fl = np.zeros(n_records + 1, dtype=npr._abi.FLOW_DTYPE)
    v6 = np.zeros(n_records + 1, dtype=npr._abi.FLOW_V6_DTYPE)

    def timed(fn):
        fn()  # warm (first touch of the scratch)
        passes, t0 = 0, time.perf_counter()
        while True:
            k, nr = fn()
            passes += 1
            el = time.perf_counter() - t0
            if el >= budget_s:
                break
        assert nr == n_records
        return passes * n_records / el / 1e6, passes, el

    one, p1, e1 = timed(lambda: _oracle.bench_extract(blob, rec, fl, v6))
    del fl, v6
    T = host_threads()
    mt = _oracle.MtScratch(n_records + 1)
    many, pm, em = timed(lambda: _oracle.bench_extract_mt(blob, mt, T))
    # the reported value is the faster of the two (the threaded run is not always faster: the serial
    # chain walk plus a memory-bound extract), with `cores` the threads that run used
    best_mt = many >= one
    return {"value": round(many if best_mt else one, 3), "unit": "Mpackets/s", "cores": T if best_mt else 1,
            "kind": "port", "threaded_value": round(many, 3), "threads": T, "single_core_value": round(one, 3),
            "sample": f"{sample} ({n_records} records, {len(blob)} B): CaptureFile::parse + convert_records "
                      f"(oracle/npr_oracle.c), {pm} passes in {em:.1f} s on {T} host threads (serial chain walk, "
                      f"parallel extract_flow); {p1} passes in {e1:.1f} s on 1 core"}


# The PMC summaries bench.py quotes as roofline.traffic: fixed names, rewritten once per round by
# scripts/pmc.sh + scripts/pmc_summary.py (never "the newest file": an experiment's summary must not
# become the bench's traffic by sorting first).
PMC_SUMMARY = {"c2": "r06g_pmc_c2.json", "c3": "r06g_pmc_c3.json"}


def pmc_traffic(records, config="c2"):
    """HBM-side bytes per launch (C2) or per capture (C3: every kernel of one step) from this round's
    committed PMC summary of the workload (profiles/PMC_SUMMARY[config]), or None: FETCH_SIZE x2 +
    WRITE_SIZE (the gfx950 correction of MI355X_MICROARCH.md)."""
    name = PMC_SUMMARY.get(config)
    want = {"c2": 1_000_000, "c3": 8_000_000}.get(config)
    if not name or records != want:
        return None, None
    try:
        d = json.load(open(os.path.join(REPO, "profiles", name)))
    except (OSError, ValueError):
        return None, None
    return d.get("traffic_bytes_per_step"), name


def roofline(read_b, write_b, kern_ms, traffic=None, traffic_src=None, stream_b=None):
    alg = read_b + write_b
    achieved = alg / (kern_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
         "read_only_frac": round(read_b / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
         "bytes_per_launch": alg, "kernel_ms": round(kern_ms, 5)}
    if stream_b is not None:
        r["stream_GBps"] = round(stream_b / (kern_ms * 1e-3) / 1e9, 1)
    return r


def run_single(args, dev, local):
    """c2 / c3 (and c4 at N=1): one GPU, the whole capture in its HBM."""
    c3 = args.config == "c3"
    c4 = args.config == "c4"
    n = args.records or (8_000_000 if c3 else (C4_PER_GPU if c4 else 1_000_000))
    copies = args.copies or (4 if args.config == "c2" else 1)
    if c4:
        blob = synth.fixed64_range(0, n).tobytes()
    else:
        blob = synth.variable_mix(n) if c3 else synth.fixed64(n)
    host = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    bufs = [host.to(dev) for _ in range(copies)]
    del host
    hdr = npr.GlobalHeader.parse(blob[:24])[1]
    ws = device.Workspace(record_cap=n, flow_cap=n, device=local, records=False, offsets=False, status=False,
                          flows=True, flows_v6=True)
    stream = torch.cuda.Stream(dev)  # an explicit stream: events bracket exactly our launches
    torch.cuda.set_stream(stream)
    if args.sparse_span:
        ws.ctx.check(ws.ctx.lib.npr_ctx_set_option(ws.ctx.handle, npr._abi.OPT_SPARSE, args.sparse_span))

    # correctness gate for the measured configuration (tests/test_gpu_scale.py compares it bit for bit)
    ws.launch(bufs[0], start=24, endianness=hdr.endianness)
    pass_ran = {1: "two-pass", 2: "resident", 8: "sparse"}.get(ws.ctx.lib.npr_ctx_last_pass(ws.ctx.handle), "?")
    if args.no_gate:  # timing-only ablation builds (make ablate): their results are not checked
        torch.cuda.synchronize()
        n_flows = n
    else:
        sm = ws.check()
        # C2/C4: every record is an Ok flow; C3: short TCP frames with a long data offset are not (Q9)
        assert sm.n_records == n and sm.consumed == len(blob) and (sm.n_flows == n or c3), (sm.n_records, sm.n_flows)
        n_flows = int(sm.n_flows)
    for i in range(args.warmup):
        ws.launch(bufs[i % copies], start=24, endianness=hdr.endianness)
    torch.cuda.synchronize()

    # ONE event pair brackets the K steps on their stream (per-step events add marker packets)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        ws.launch(bufs[i % copies], start=24, endianness=hdr.endianness)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if not args.no_gate:
        sm = ws.check()
        assert sm.n_records == n and sm.n_flows == n_flows
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if args.stats:
        stats_dump(ws, bufs, hdr, copies, 0)
    # algorithmic bytes: 16 + min(incl, 64) read per record, 32 written per Ok flow.
    # C2 (80-B records): every byte of the capture.  C3 (frames >= 64 B): 80 B of each ~800-B record.
    read_b = len(blob) if args.config != "c3" else 80 * n
    write_b = 32 * n_flows
    traffic, src = pmc_traffic(n, args.config) if args.config in ("c2", "c3") else (None, None)
    out = base_line(args, 1, wall, n, len(blob))
    out["config"].update({"records_per_gpu": n, "capture_bytes": len(blob), "parallelism": "single GPU",
                          "pass": pass_ran})
    out["roofline"] = roofline(read_b, write_b, kern_ms, traffic, src, stream_b=len(blob) - 24)
    if c3:
        out["roofline"]["survey_8d_bytes_per_launch"] = read_b + write_b
        out["roofline"]["survey_8d_frac"] = out["roofline"]["frac"]
        out["roofline"]["note"] = ("C3: one step = the sparse record walk (k_sparse_walk: header hops, one 80-B window "
                                   "per record), k_sparse_scan and k_sparse_rows; achieved = SURVEY 8d bytes / step time "
                                   "(HIP events over the stream); stream_GBps = the capture's bytes / step time"
                                   if pass_ran == "sparse" else
                                   "C3 through the resident pass (every byte streams); achieved uses SURVEY 8d bytes")
    if not args.no_cpu:
        sample = {"c2": "the C2 capture", "c3": "the C3 capture", "c4": "one C4 shard"}[args.config]
        out["cpu_baseline"] = cpu_baseline(blob, n, args.cpu_budget, sample)
    return out


def stats_dump(ws, bufs, hdr, copies, rank):
    import ctypes
    lib, h = ws.ctx.lib, ws.ctx.handle
    ws.ctx.check(lib.npr_ctx_set_stats(h, 2))
    for i in range(3):
        ws.launch(bufs[i % copies], start=24, endianness=hdr.endianness)
    ws.check()
    st = (ctypes.c_uint32 * 8)()
    ws.ctx.check(lib.npr_ctx_read_stats(h, st, 8, 1))
    ntl = ctypes.c_uint64(0)
    nt = 0
    # per-wave stamps exist for the resident pass only (the sparse walk keeps counters, no stamps)
    if lib.npr_ctx_read_stamps(h, None, 0, ctypes.byref(ntl)) == 0:
        nt = ntl.value
        stamps = np.zeros(nt * 16, dtype=np.uint64)
        ws.ctx.check(lib.npr_ctx_read_stamps(h, stamps.ctypes.data, stamps.size, ctypes.byref(ntl)))
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        np.save(os.path.join(REPO, "gpurun_out", f"stamps_rank{rank}.npy"), stamps.reshape(nt, 16))
    print(f"[rank {rank}] stats rewalk={st[0]} mism_wait={st[1]} none={st[5]} lookback_rereads={st[6]} tiles={nt}",
          file=sys.stderr, flush=True)
    ws.ctx.check(lib.npr_ctx_set_stats(h, 0))


def base_line(args, world, wall, n_per_gpu, bytes_per_gpu):
    ms_per_step = wall * 1e3 / args.steps
    total = n_per_gpu * world * args.steps
    workload = {
        "c2": "C2: 1M x 64-B Ethernet/IPv4/TCP records per GPU, device-resident",
        "c3": "C3: 8M records, frames U[64,1500] B, IPv4 TCP|UDP per GPU, device-resident",
        "c4": "C4: 64M x 64-B records sharded by record range, 8M per GPU (N=8 = configs[3]), device-resident",
    }[args.config]
    return {
        "metric": METRIC,
        "value": round(total / wall / 1e6, 3),
        "unit": "Mpackets/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (numpy PCG64 seed 0x4E50; layouts of SURVEY.md 8d)",
        "config": {"workload": workload,
                   "outputs": "convert_records flow table (32 B/flow incl. record offset)"},
        "stream_GBps": round(bytes_per_gpu * world * args.steps / wall / 1e9, 2),
    }


def run_sharded(args, dev, local, rank, world):
    """c4 over N ranks: rank g holds records [g*R, (g+1)*R) of one capture (only those bytes)."""
    R = args.records or C4_PER_GPU
    n_total = R * world
    layout = parallel.record_range_shards(n_total, world)
    base, start, stop, spec = layout[rank]
    a = synth.fixed64_range(R * rank, R * (rank + 1))
    file_len = 24 + 80 * n_total
    buf = torch.from_numpy(a).to(dev)
    del a
    bounds = [(24 if g == 0 else layout[g][1], layout[g][2]) for g in range(world)]
    ws = device.Workspace(record_cap=1, flow_cap=R, device=local, records=False, offsets=False, status=False,
                          flows=True, flows_v6=False)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    # C4 frames are IPv4 by construction: no IPv6 side table to move (pass ws.flows_v6 rows otherwise)
    # the per-step 64-B summaries are exchanged on the host, off the GPU timeline: through node-local
    # shared memory (parallel.ShmExchange, ~40 us at 8 ranks), else gloo over loopback (~1.4 ms at 8
    # ranks), else an RCCL all-gather of the device summaries between two parses
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    try:
        meta = dist.new_group(backend="gloo")
    except RuntimeError as e:
        print(f"[rank {rank}] no gloo group ({e}); summaries over RCCL", file=sys.stderr, flush=True)
        meta = None
    xchg = None
    # eight steps in flight, the oldest four finished by ONE host exchange (so a slow exchange, gloo at
    # 8 ranks, is paid once per four parses)
    depth = 8
    if meta is not None:
        try:
            xchg = parallel.ShmExchange(meta, slot_bytes=depth * ws.summary.numel())
        except RuntimeError as e:
            print(f"[rank {rank}] no shared-memory exchange ({e}); summaries over gloo", file=sys.stderr, flush=True)
    step = parallel.DeviceShardedParse(ws, buf, base, bounds, file_len, usec_magic=True, ts_ref=1_600_000_000,
                                       meta_group=meta, depth=depth, exchange=xchg)
    metas, live, rounds = step.step()
    _, _, r_tot, f_tot = parallel.prefix_offsets(metas, live)
    assert rounds == 1 and r_tot == n_total and f_tot == n_total, (rounds, r_tot, f_tot)
    for _ in range(args.warmup):
        step.step()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # up to `depth` steps in flight: the host replay of exchanged summaries runs while later steps parse
    for _ in range(args.steps):
        step.launch_step()
        if len(step.pending) == depth:
            _, _, r = step.finish_steps(depth // 2)
            rounds = max(rounds, r)
    if step.pending:
        _, _, r = step.finish_steps(len(step.pending))
        rounds = max(rounds, r)
    torch.cuda.synchronize()
    dist.barrier()
    wall = time.perf_counter() - t0
    # the device time of this rank's launches alone (one event pair per launch series)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    kms = []
    for _ in range(3):
        ev0.record(stream)
        step._launch(step.start if rank == 0 else bounds[rank][0], rank > 0)
        ev1.record(stream)
        torch.cuda.synchronize()
        kms.append(ev0.elapsed_time(ev1))
    kern_ms = float(np.median(kms))
    step.step()
    # the flow-table gather to rank 0 (RCCL point-to-point into the merged table), timed apart
    gms = []
    for _ in range(max(1, min(3, args.steps))):
        dist.barrier()
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        fl, _ = step.rows()
        merged, _ = parallel.gather_flow_tables(fl, None, metas, live)
        torch.cuda.synchronize()
        dist.barrier()
        gms.append((time.perf_counter() - g0) * 1e3)
    bad = 0.0
    if rank == 0:
        # rows of the merged table run from the last record to the first: check both ends
        off = lambda r: int.from_bytes(bytes(r["record_offset"]), "little")
        if merged.numel() != 32 * n_total:
            bad = 1.0
        else:
            first = merged[:32].cpu().numpy().view(npr._abi.FLOW_DTYPE)[0]
            last = merged[-32:].cpu().numpy().view(npr._abi.FLOW_DTYPE)[0]
            bad = 0.0 if off(first) == file_len - 80 and off(last) == 24 else 1.0
    # the verdict rides on the same collective as the timings: every rank learns it, none waits
    # in a collective for a rank that stopped
    t = torch.tensor([wall, kern_ms, float(np.median(gms)), bad], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern_ms, gather_ms = float(t[0]), float(t[1]), float(t[2])
    if t[3] != 0:
        raise SystemExit(f"[rank {rank}] the merged flow table on rank 0 is not the capture's")
    out = base_line(args, world, wall, R, len(buf))
    out["config"].update({"records_per_gpu": R, "capture_bytes": file_len, "parallelism": f"record-range x{world}"})
    out["roofline"] = roofline(80 * R, 32 * R, kern_ms, stream_b=80 * R)
    step_ms = wall * 1e3 / args.steps
    how = ("node-local shared memory (npr_shm_all_gather)" if xchg is not None else "gloo over loopback")
    out["exchange"] = {"collective": (f"all-gather of the ranks' 64-B parse summaries on the host ({how}), one per "
                                      f"{depth // 2} steps ({depth} in flight), overlapped with the later steps' parses; RCCL "
                                      "carries the flow rows") if meta is not None
                       else "RCCL all_gather of the ranks' device summaries, one per step", "rounds": rounds}
    out["gather_ms"] = round(gather_ms, 3)
    out["gather"] = ("RCCL point-to-point of every rank's flow rows straight into rank 0's merged "
                     f"convert_records table ({32 * n_total / 1e9:.2f} GB)")
    out["end_to_end_Mpps"] = round(n_total / ((step_ms + gather_ms) * 1e-3) / 1e6, 3)
    return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["c2", "c3", "c4"], default=None,
                    help="c2 (N=1 default: 1M x 64-B records), c3 (8M records U[64,1500] B), "
                         "c4 (N>1 default: 8M x 64-B records per GPU, one capture sharded by record range)")
    ap.add_argument("--records", type=int, default=None)
    ap.add_argument("--copies", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=8.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gate", action="store_true", help=argparse.SUPPRESS)  # ablation builds only
    ap.add_argument("--stats", action="store_true", help="print speculation / hand-off counters (stderr)")
    ap.add_argument("--sparse-span", type=int, default=0,
                    help="c3: force the sparse record walk with lane ranges of N bytes (NPR_OPT_SPARSE N >= 64; 0 = auto)")
    ap.add_argument("--sharded", action="store_true",
                    help="c4 through the multi-GPU step (RCCL exchange + gather) even at N=1")
    # the launcher alone, on CPU: every rank joins a gloo group and rank 0 prints the world it saw
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank, world, port, argv):
    """One spawned rank: the torchrun environment, then the rank's run."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rank_main(parse_args(argv))


def spawn_ranks(args, argv):
    """`python bench.py --gpus N` with no launcher: start N rank processes (one per GPU) before this
    process touches any GPU, as torch.distributed.run would, and exit with the worst exit code.  A
    rank that fails ends the others (parallel.supervise_ranks), so none waits in a collective."""
    port = _free_port()
    codes = parallel.supervise_ranks(_rank_entry, [(r, args.gpus, port, argv) for r in range(args.gpus)])
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"bench.py: rank exit codes {codes}", file=sys.stderr, flush=True)
        sys.exit(bad[0] if bad[0] and bad[0] > 0 else 1)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:  # never measure another world than the one asked for
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    rank_main(args)


def rank_main(args):
    # the one JSON line goes to the original stdout; everything else written to fd 1 (e.g. the RCCL
    # version banner of communicator init) goes to stderr
    out_fd = os.dup(1)
    os.dup2(2, 1)
    json_out = os.fdopen(out_fd, "w")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        got = [None] * dist.get_world_size()
        dist.all_gather_object(got, rank)
        if rank == 0:
            print(json.dumps({"launch_check": {"world": dist.get_world_size(), "ranks": got}}), file=json_out,
                  flush=True)
        dist.destroy_process_group()
        return
    if args.config is None:
        args.config = "c2" if world == 1 else "c4"
    sharded = world > 1 or args.sharded
    if sharded:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the communicator has {dist.get_world_size()} ranks")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if sharded:
        if args.config != "c4":
            raise SystemExit("N > 1 runs the sharded C4 workload (--config c4)")
        out = run_sharded(args, dev, local, rank, dist.get_world_size())
    else:
        out = run_single(args, dev, local)
    if rank == 0:
        print(json.dumps(out), file=json_out, flush=True)
    if sharded:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
