"""The multi-rank path (net_parser_rs.parallel) on CPU: byte-range shards of one capture, the
one-exchange reconcile, the reverse-rank merge.  The oracle stands in for each rank's device
parse here (test infrastructure only); tests/test_gpu_parallel.py runs the same logic over the
device range API.  world_size 2 runs over torch.distributed `gloo` at 127.0.0.1."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import _oracle
from net_parser_rs import _abi, parallel, synth


def full_reference(blob, with_v6=False):
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert rc == 0
    flows, v6 = _oracle.convert_records(blob, recs)
    return (hdr, recs, cons, flows, v6) if with_v6 else (hdr, recs, cons, flows)


def oracle_local(blob, endianness, spec):
    """Rank-local parser over the oracle: records that start in [start, hi) of the chain from
    `start`; with speculative=True the start comes from `spec(lo, hi)` (right or wrong on purpose)."""
    def local(lo, hi, start, speculative):
        if speculative:
            start = spec(lo, hi)
            if start is None:
                return parallel.ShardResult(_abi.NO_ENTRY, hi, 0, 0, np.zeros(0, _abi.FLOW_DTYPE),
                                            np.zeros(0, _abi.FLOW_V6_DTYPE))
        recs, cons = _oracle.records_parse(blob[start:], endianness)
        recs = recs.copy()
        recs["offset"] += start
        keep = recs[recs["offset"] < hi]
        consumed = int(recs["offset"][len(keep)]) if len(keep) < len(recs) else start + cons
        flows, v6 = _oracle.convert_records(blob, keep)
        return parallel.ShardResult(start, consumed, len(keep), len(flows), flows, v6)
    return local


def spec_exact(recs):
    offs = np.asarray(recs["offset"], dtype=np.int64)

    def spec(lo, hi):  # the true first record start in [lo, hi)
        i = np.searchsorted(offs, lo)
        return int(offs[i]) if i < len(offs) and offs[i] < hi else lo
    return spec


def spec_off_by(recs, skip):
    exact = spec_exact(recs)
    offs = np.asarray(recs["offset"], dtype=np.int64)

    def spec(lo, hi):  # a WRONG guess: `skip` records late (a plausible but mis-aligned chain)
        e = exact(lo, hi)
        i = np.searchsorted(offs, e)
        return int(offs[min(i + skip, len(offs) - 1)])
    return spec


def v6_rows(flows, v6):
    """The IPv6 side rows that carry data (rows of IPv4 flows are unspecified)."""
    m = (flows["kind"] & _abi.KIND_IPV6) != 0
    return v6[m].tobytes()


def check_merge(blob, world, spec_maker):
    hdr, recs, cons, flows, v6 = full_reference(blob, with_v6=True)
    local = oracle_local(blob, hdr.endianness, spec_maker(recs))
    results, live, rounds = parallel.parse_sharded_inprocess(local, 24, len(blob), world)
    merged, merged6 = parallel.merge_flows(results, live)
    _, _, r_tot, f_tot = parallel.prefix_offsets(results, live)
    assert r_tot == len(recs) and f_tot == len(flows)
    assert merged.tobytes() == flows.tobytes()
    assert v6_rows(merged, merged6) == v6_rows(flows, v6)
    return rounds


@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_sharded_matches_serial_with_right_speculation(world):
    rounds = check_merge(synth.quirk_corpus(3_000, seed=31), world, spec_exact)
    assert rounds == 1  # one exchange, no rerun


@pytest.mark.parametrize("world", [2, 4])
def test_wrong_speculation_is_rerun(world):
    rounds = check_merge(synth.quirk_corpus(3_000, seed=32), world, lambda recs: spec_off_by(recs, 1))
    assert rounds > 1


def test_no_speculated_start():
    check_merge(synth.quirk_corpus(2_000, seed=33), 3, lambda recs: (lambda lo, hi: None))


def test_chain_end_inside_a_shard_stops_later_ranks():
    blob = synth.corrupt_midfile(synth.fixed64(4_000), at_record=700)   # END early: rank 0's range
    check_merge(blob, 4, spec_exact)


def test_jumbo_records_cross_shards():
    check_merge(synth.quirk_corpus(300, seed=34, jumbo_every=2), 6, spec_exact)


def test_replay_pure():
    bounds = [(24, 100), (100, 200), (200, 300)]
    ok = [parallel.ShardResult(24, 110, 3, 3), parallel.ShardResult(110, 205, 2, 1),
          parallel.ShardResult(205, 300, 2, 2)]
    assert parallel.replay(24, bounds, ok)[0] is None
    bad = list(ok)
    bad[2] = parallel.ShardResult(204, 300, 2, 2)
    r, e, _ = parallel.replay(24, bounds, bad)
    assert (r, e) == (2, 205)
    ended = [parallel.ShardResult(24, 90, 3, 3), parallel.ShardResult(110, 205, 2, 1),
             parallel.ShardResult(205, 300, 2, 2)]
    r, e, live = parallel.replay(24, bounds, ended)
    assert r is None and live == [True, False, False]


# ---- world_size 2 over gloo (one process per rank, 127.0.0.1) ----------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, blob, wrong, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hdr, recs, cons, flows, v6 = full_reference(blob, with_v6=True)
        spec = spec_off_by(recs, 1) if wrong else spec_exact(recs)
        local = oracle_local(blob, hdr.endianness, spec)
        mine, metas, live, rounds = parallel.parse_sharded(local, 24, len(blob))
        got = parallel.gather_flows(mine, metas, live)
        if rank == 0:
            merged, merged6 = got
            _, _, r_tot, f_tot = parallel.prefix_offsets(metas, live)
            n6 = int(((flows["kind"] & _abi.KIND_IPV6) != 0).sum())
            q.put((r_tot == len(recs), f_tot == len(flows), merged.tobytes() == flows.tobytes(),
                   n6 > 0 and v6_rows(merged, merged6) == v6_rows(flows, v6), rounds))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("wrong", [False, True], ids=["exact", "rerun"])
def test_gloo_world2(wrong):
    blob = synth.quirk_corpus(2_500, seed=35)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, blob, wrong, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    recs_ok, flows_ok, bytes_ok, v6_ok, rounds = q.get(timeout=10)
    assert recs_ok and flows_ok and bytes_ok and v6_ok
    assert (rounds > 1) == wrong


# ---- the device step's exchange protocol (DeviceShardedParse) over gloo ------------------------
class OracleShardWorkspace:
    """Stands in for device.Workspace on CPU: npr_dev_parse_extract_shard's contract (records that
    start in [start, stop), flow rows right-aligned, the summary as the device writes it), computed
    by the oracle from the rank's OWN shard bytes only (file offsets)."""

    def __init__(self, flow_cap, spec):
        import torch
        self.flow_cap, self.spec = flow_cap, spec
        self.summary = torch.zeros(64, dtype=torch.uint8)
        self.flows = torch.zeros(flow_cap * 32, dtype=torch.uint8)
        self.flows_v6 = torch.zeros(flow_cap * 32, dtype=torch.uint8)

    def launch_shard(self, buf, base, start, stop, endianness=0, speculative=False, usec_magic=True, ts_ref=None,
                     chunk_bytes=0, nbytes=None):
        import torch
        shard = buf.numpy().tobytes()
        if speculative:
            start = self.spec(start, stop)
        if start is None:
            sm = (0, 0, stop, _abi.NO_ENTRY)
            n_flows = 0
        else:
            recs, cons = _oracle.records_parse(shard[start - base:], endianness)
            recs = recs.copy()
            recs["offset"] += start - base
            keep = recs[recs["offset"] + base < stop]
            consumed = int(recs["offset"][len(keep)]) + base if len(keep) < len(recs) else start + cons
            flows, v6 = _oracle.convert_records(shard, keep)
            off = flows["record_offset"].astype(np.uint64)
            o = sum(off[:, i] << np.uint64(8 * i) for i in range(5)) + np.uint64(base)  # file offsets
            for i in range(5):
                flows["record_offset"][:, i] = ((o >> np.uint64(8 * i)) & np.uint64(0xff)).astype(np.uint8)
            n_flows = len(flows)
            self.flows[(self.flow_cap - n_flows) * 32:] = torch.from_numpy(flows.view(np.uint8).reshape(-1).copy())
            self.flows_v6[(self.flow_cap - n_flows) * 32:] = torch.from_numpy(v6.view(np.uint8).reshape(-1).copy())
            sm = (len(keep), n_flows, consumed, start)
        s = np.zeros(1, dtype=_abi.SUMMARY_DTYPE)
        s["n_records"], s["n_flows"], s["consumed"], s["entry"] = sm
        s["epoch"], s["flags"] = 1, 0
        self.summary[:40] = torch.from_numpy(s.view(np.uint8).copy())

    def flow_rows(self, n):
        lo = (self.flow_cap - n) * 32
        return self.flows[lo:], self.flows_v6[lo:]


def _step_rank_main(rank, world, port, blob, wrong, q, pipelined=False):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hdr, recs, cons, flows, v6 = full_reference(blob, with_v6=True)
        bounds = parallel.shard_bounds(24, len(blob), world)
        lo, hi = bounds[rank]
        base = 0 if rank == 0 else lo - lo % 16
        end = min(len(blob), hi + (1 << 20))
        shard = torch.from_numpy(np.frombuffer(blob[base:end], dtype=np.uint8).copy())
        spec = spec_off_by(recs, 1) if wrong else spec_exact(recs)
        ws = OracleShardWorkspace(len(recs) + 1, spec)
        meta = dist.new_group(backend="gloo") if str(pipelined).startswith("host_meta") else None
        xchg = parallel.ShmExchange() if str(pipelined).startswith("shm") else None
        deep = pipelined in ("host_meta_d4", "shm_d4")
        step = parallel.DeviceShardedParse(ws, shard, base, bounds, len(blob), meta_group=meta, depth=4 if deep else 2,
                                           exchange=xchg)
        if deep:  # the bench's N > 1 loop: four steps in flight, the oldest two finished by ONE exchange
            rounds = 0
            for _ in range(7):
                step.launch_step()
                if len(step.pending) == 4:
                    metas, live, r = step.finish_steps(2)
                    rounds = max(rounds, r)
            metas, live, r = step.finish_steps(len(step.pending))
            rounds = max(rounds, r)
        elif pipelined:  # two steps in flight, host replay of step k during step k+1
            rounds = 0
            for _ in range(3):
                step.launch_step()
                if len(step.pending) > 1:
                    metas, live, r = step.finish_step()
                    rounds = max(rounds, r)
            while step.pending:
                metas, live, r = step.finish_step()
                rounds = max(rounds, r)
        else:
            metas, live, rounds = step.step()
        fl, f6 = step.rows()
        merged, merged6 = parallel.gather_flow_tables(fl, f6, metas, live)
        if rank == 0:
            m = merged.numpy().view(_abi.FLOW_DTYPE)
            m6 = merged6.numpy().view(_abi.FLOW_V6_DTYPE)
            q.put((m.tobytes() == flows.tobytes(), v6_rows(m, m6) == v6_rows(flows, v6), rounds))
        else:
            assert merged is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, True, "host_meta", "host_meta_d4", "shm", "shm_d4"],
                         ids=["step", "launch_finish", "host_meta", "host_meta_depth4", "shm", "shm_depth4"])
@pytest.mark.parametrize("wrong", [False, True], ids=["exact", "rerun"])
def test_gloo_world2_device_step_protocol(wrong, pipelined):
    """DeviceShardedParse (the bench's multi-GPU step) + gather_flow_tables over gloo: each rank holds
    only its shard's bytes; summaries all-gathered, the chain replayed, a wrong speculated start
    re-parsed, flow rows sent point-to-point into the root's merged table."""
    blob = synth.quirk_corpus(2_500, seed=36)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step_rank_main, args=(r, 2, port, blob, wrong, q, pipelined)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    flows_ok, v6_ok, rounds = q.get(timeout=10)
    assert flows_ok and v6_ok
    assert (rounds > 1) == wrong


# ---- side rows when the root holds no flows; a record spanning a whole shard -------
def _v6_gather_main(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = synth.quirk_corpus(3_000, seed=38)
        _, _, recs, _ = _oracle.capture_file_parse(blob)
        flows, v6 = _oracle.convert_records(blob, recs)
        assert ((flows["kind"] & _abi.KIND_IPV6) != 0).any()
        full = parallel.ShardResult(24, len(blob), len(recs), len(flows), flows, v6)
        if mode == "missing":  # rank 0 holds flows but no side table, rank 1 holds one: both raise
            metas = [parallel.ShardResult(24, len(blob), len(recs), len(flows))] * 2
            mine = parallel.ShardResult(24, len(blob), len(recs), len(flows), flows, None) if rank == 0 else full
            try:
                parallel.gather_flows(mine, metas, [True, True])
            except ValueError:
                q.put((rank, "raised"))
            else:
                q.put((rank, "no error"))
            return
        # rank 0 (the root) holds no Ok flow (an empty side table, or None); rank 1 holds every flow
        metas = [parallel.ShardResult(24, 24, 0, 0), parallel.ShardResult(24, len(blob), len(recs), len(flows))]
        side = None if mode == "none" else np.zeros(0, _abi.FLOW_V6_DTYPE)
        empty = parallel.ShardResult(24, 24, 0, 0, np.zeros(0, _abi.FLOW_DTYPE), side)
        got = parallel.gather_flows(empty if rank == 0 else full, metas, [True, True])
        if rank == 0:
            m, m6 = got
            q.put((m.tobytes() == flows.tobytes(), m6 is not None and v6_rows(m, m6) == v6_rows(flows, v6)))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["empty", "none", "missing"])
def test_gloo_world2_v6_rows_root_without_flows(mode):
    """The root without flows holding an empty side table or none (None counts as empty
    on a rank without flows); a rank WITH flows but no side table while another has one: every rank
    raises instead of dropping IPv6 addresses."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_v6_gather_main, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    if mode == "missing":
        assert sorted(q.get(timeout=10) for _ in range(2)) == [(0, "raised"), (1, "raised")]
        return
    flows_ok, v6_ok = q.get(timeout=10)
    assert flows_ok and v6_ok


def spanning_capture():
    """64-B records, then ONE record whose payload spans the middle third of the capture, then more
    64-B records: with three equal byte ranges, no record starts in rank 1's range."""
    import struct
    a = synth.fixed64(150)
    b = synth.fixed64(150, seed=77, with_header=False)
    jumbo = struct.pack("<IIII", 1_600_000_000, 999_999, 30_000, 30_000) + bytes(30_000)
    return a + jumbo + b


def _span_rank_main(rank, world, port, blob, q, shm=False):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hdr, recs, cons, flows, v6 = full_reference(blob, with_v6=True)
        bounds = parallel.shard_bounds(24, len(blob), world)
        lo, hi = bounds[rank]
        base = 0 if rank == 0 else lo - lo % 16
        shard = torch.from_numpy(np.frombuffer(blob[base:], dtype=np.uint8).copy())
        # rank 1's speculation finds no record start (there is none): its first byte is the guess
        ws = OracleShardWorkspace(len(recs) + 1, spec_exact(recs))
        step = parallel.DeviceShardedParse(ws, shard, base, bounds, len(blob),
                                           exchange=parallel.ShmExchange() if shm else None)
        metas, live, rounds = step.step()
        fl, f6 = step.rows()
        merged, _ = parallel.gather_flow_tables(fl, None, metas, live)
        if rank == 0:
            q.put((merged.numpy().tobytes() == flows.tobytes(), metas[1].n_records, rounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shm", [False, True], ids=["gloo", "shm"])
def test_gloo_world3_record_spans_a_whole_shard(shm):
    blob = spanning_capture()
    bounds = parallel.shard_bounds(24, len(blob), 3)
    _, recs, _, _ = full_reference(blob)
    offs = recs["offset"]
    assert not ((offs >= bounds[1][0]) & (offs < bounds[1][1])).any()  # no record starts in rank 1's range
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_span_rank_main, args=(r, 3, port, blob, q, shm)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    flows_ok, n1, rounds = q.get(timeout=10)
    assert flows_ok and n1 == 0 and rounds == 2


# ---- a short halo: every rank raises HaloError together ------------------------------------------
def _halo_rank_main(rank, world, port, blob, q, shm=False):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, recs, _, _ = full_reference(blob)
        bounds = parallel.shard_bounds(24, len(blob), world)
        lo, hi = bounds[rank]
        base = 0 if rank == 0 else lo - lo % 16
        # rank 0's buffer ends 10 bytes before its stop: the record straddling that point is cut
        end = hi - 10 if rank == 0 else len(blob)
        shard = torch.from_numpy(np.frombuffer(blob[base:end], dtype=np.uint8).copy())
        ws = OracleShardWorkspace(len(recs) + 1, spec_exact(recs))
        step = parallel.DeviceShardedParse(ws, shard, base, bounds, len(blob),
                                           exchange=parallel.ShmExchange() if shm else None)
        try:
            step.step()
            q.put((rank, "no error"))
        except parallel.HaloError as e:
            q.put((rank, "halo" if "ranks [0]" in str(e) else str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shm", [False, True], ids=["gloo", "shm"])
def test_gloo_world2_short_halo_raises_on_every_rank(shm):
    """A rank whose buffer stops inside a record before its shard's stop: HaloError on BOTH ranks
    (decided from the shared summaries and buffer ends), so no rank goes on into a collective the
    raising rank never joins."""
    blob = synth.fixed64(4_000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_halo_rank_main, args=(r, 2, port, blob, q, shm)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=10) for _ in range(2))
    assert got == [(0, "halo"), (1, "halo")]


# ---- the summary exchange's latency at 8 ranks: node-local shared memory against gloo ------------
def _xchg_latency_main(rank, world, port, n, q):
    import time
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = torch.full((64,), rank, dtype=torch.uint8)
        res = {}
        for name, x in (("gloo", parallel.GlooExchange(None)), ("shm", parallel.ShmExchange())):
            for _ in range(20):
                x.all_gather(mine)
            dist.barrier()
            ts = []
            for i in range(n):
                mine[0] = i & 0xff
                t0 = time.perf_counter()
                out = x.all_gather(mine)
                ts.append(time.perf_counter() - t0)
                assert out.shape == (world, 64) and all(int(out[r, 1]) == r and int(out[r, 0]) == i & 0xff
                                                        for r in range(world))
            res[name] = float(np.median(ts)) * 1e6
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


def test_shm_exchange_latency_world8():
    """the per-step summary exchange at 8 ranks (one node).  Every step all-gathers a
    64-B summary per rank; over gloo (TCP loopback) that was 1.3 ms here, slower than one 0.23-ms
    shard parse.  Node-local shared memory (npr_shm_all_gather): 36-44 us median on this 8-CPU
    container, where pytest and the 8 ranks share the cores (the bound below leaves room for that
    noise)."""
    world, n = 8, 300

    def measure():
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_xchg_latency_main, args=(r, world, port, n, q)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(180)
            assert p.exitcode == 0
        return q.get(timeout=10)

    # the ranks spin on the host's cores, which other processes may hold (a parallel test run, the
    # previous test's stragglers: 144-308 us then, with gloo at 12 ms): up to three runs, the best
    # one judged, and the absolute bound only where gloo shows a quiet machine
    for _ in range(3):
        res = measure()
        print(f"median all-gather of 64 B at {world} ranks: shm {res['shm']:.1f} us, gloo {res['gloo']:.1f} us")
        assert res["shm"] < res["gloo"] / 5, res
        if res["shm"] < 80.0:
            break
    else:
        assert res["gloo"] > 5000.0, res  # a quiet machine that still misses 80 us


# ---- the bench's N = 8 loop on CPU, and a failing rank --------------------------
class _FailingWorkspace(OracleShardWorkspace):
    """An oracle workspace whose `fail_at`-th launch raises (a rank that dies mid-loop)."""

    def __init__(self, flow_cap, spec, fail_at):
        super().__init__(flow_cap, spec)
        self.fail_at, self.launches = fail_at, 0

    def launch_shard(self, *a, **k):
        self.launches += 1
        if self.launches == self.fail_at:
            raise RuntimeError("injected rank failure")
        return super().launch_shard(*a, **k)


def _step8_rank_main(rank, world, port, blob, fail_rank, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hdr, recs, cons, flows, v6 = full_reference(blob, with_v6=True)
        bounds = parallel.shard_bounds(24, len(blob), world)
        lo, hi = bounds[rank]
        base = 0 if rank == 0 else lo - lo % 16
        end = min(len(blob), hi + (1 << 20))
        shard = torch.from_numpy(np.frombuffer(blob[base:end], dtype=np.uint8).copy())
        spec = spec_exact(recs)
        ws = (_FailingWorkspace(len(recs) + 1, spec, fail_at=5) if rank == fail_rank
              else OracleShardWorkspace(len(recs) + 1, spec))
        depth = 8  # bench.run_sharded's loop: eight steps in flight, the oldest four per exchange
        xchg = parallel.ShmExchange(slot_bytes=depth * 64, timeout_s=300.0)
        step = parallel.DeviceShardedParse(ws, shard, base, bounds, len(blob), depth=depth, exchange=xchg)
        metas, live, rounds = step.step()
        for _ in range(20):
            step.launch_step()
            if len(step.pending) == depth:
                metas, live, r = step.finish_steps(depth // 2)
                rounds = max(rounds, r)
        metas, live, r = step.finish_steps(len(step.pending))
        fl, f6 = step.rows()
        merged, merged6 = parallel.gather_flow_tables(fl, f6, metas, live)
        if rank == 0:
            m = merged.numpy().view(_abi.FLOW_DTYPE)
            m6 = merged6.numpy().view(_abi.FLOW_V6_DTYPE)
            q.put((m.tobytes() == flows.tobytes(), v6_rows(m, m6) == v6_rows(flows, v6), max(rounds, r)))
    finally:
        dist.destroy_process_group()


def test_gloo_world8_depth8_shm_loop():
    """Eight ranks of the bench's N = 8 step loop (DeviceShardedParse at depth 8 over the node-local
    shared-memory exchange, oracle workspaces), merged table bit-exact on the root."""
    blob = synth.quirk_corpus(4_000, seed=37)
    q = mp.get_context("spawn").Queue()
    port = _free_port()
    codes = parallel.supervise_ranks(_step8_rank_main, [(r, 8, port, blob, -1, q) for r in range(8)])
    assert codes == [0] * 8, codes
    flows_ok, v6_ok, rounds = q.get(timeout=10)
    assert flows_ok and v6_ok and rounds == 1


def test_gloo_world8_failing_rank_ends_the_others():
    """Rank 5 dies at its fifth launch, with steps in flight on every rank: the others would wait
    in the exchange (here up to 300 s); supervise_ranks (bench.spawn_ranks) ends them at once."""
    import time
    blob = synth.quirk_corpus(4_000, seed=38)
    q = mp.get_context("spawn").Queue()
    port = _free_port()
    t0 = time.monotonic()
    codes = parallel.supervise_ranks(_step8_rank_main, [(r, 8, port, blob, 5, q) for r in range(8)])
    took = time.monotonic() - t0
    assert codes[5] == 1, codes  # the injected exception
    assert all(c != 0 for c in codes), codes  # nobody finished the loop without rank 5
    assert took < 120, took


# ---- row f4 across ranks: gather each rank's distinct flows, merge them weighted -----------------
def cpu_aggregate(flows, flows_v6, n, weights=None):
    """parallel.gather_distinct_flows' `aggregate` on host tensors: the row-f4 checker."""
    import torch
    import _flowtable_ref
    f = flows[: n * 32].numpy().view(_abi.FLOW_DTYPE)
    v = flows_v6[: n * 32].numpy().view(_abi.FLOW_V6_DTYPE) if flows_v6 is not None else np.zeros(n, _abi.FLOW_V6_DTYPE)
    rows, counts = _flowtable_ref.aggregate(f, v, None if weights is None else weights[:n].numpy())
    b = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy())
    return b(f[rows]), (b(v[rows]) if flows_v6 is not None else None), torch.from_numpy(counts.astype(np.int64)), len(rows)


def _distinct_main(rank, world, port, cuts, with_v6, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        blob = synth.flow_mix(6_000, n_flows=150, seed=44)
        _, _, recs, _ = _oracle.capture_file_parse(blob)
        flows, v6 = _oracle.convert_records(blob, recs)
        # the merged table's pieces in order belong to ranks world-1 ... 0 (reverse rank order)
        edges = [0] + list(cuts) + [len(flows)]
        j = world - 1 - rank
        lo, hi = edges[j], edges[j + 1]
        b = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy())
        got = parallel.gather_distinct_flows(b(flows[lo:hi]), b(v6[lo:hi]) if with_v6 else None, hi - lo,
                                             aggregate=cpu_aggregate)
        if rank == 0:
            want = cpu_aggregate(b(flows), b(v6) if with_v6 else None, len(flows))
            rows, rows6, cnt, k = got
            ok = k == want[3] and rows.numpy().tobytes() == want[0].numpy().tobytes() and \
                bool((cnt == want[2]).all()) and (not with_v6 or rows6.numpy().tobytes() == want[1].numpy().tobytes())
            q.put(bool(ok and 0 < k < len(flows)))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cuts,with_v6", [(2, (2500,), True), (3, (1000, 1000), True), (3, (700, 4100), False)])
def test_gloo_distinct_flow_gather_equals_one_aggregate(world, cuts, with_v6):
    """Each rank aggregates its piece of the convert_records table; the root merges the gathered
    distinct rows weighted by their counts: the same table as one aggregate of the whole (an empty
    piece included: cuts (1000, 1000) leave rank 1 with no rows)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_distinct_main, args=(r, world, port, cuts, with_v6, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) is True
