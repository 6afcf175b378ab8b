"""One capture sharded by byte range across ranks (SURVEY.md §8 row e).

The reference parses a capture serially (`PcapRecords::parse`, src/record.rs:21-54): record k+1
starts where record k ends, and the list stops at the first Incomplete record (Q3).  Sharded:

1. rank r owns the byte range [lo_r, hi_r) of the record stream: the records that START there;
2. every rank parses its range from a speculated first record start (rank 0: the exact start)
   with npr_dev_parse_extract_range, so all ranks run concurrently;
3. ONE exchange — an all-gather of {entry, consumed, n_records, n_flows} per rank — lets every
   rank replay the chain: rank r's exact entry is rank r-1's exact `consumed`.  The first rank
   whose speculated entry contradicts it re-parses from the exact entry; the exchange repeats
   (at most once per rank; with a plausible speculation it does not repeat at all);
4. a chain END (an Incomplete record) inside rank r's range ends the whole capture there:
   later ranks contribute nothing, exactly as the serial reference stops;
5. flows are gathered to the root in REVERSE rank order, which is convert_records' order
   (src/flow/mod.rs:101-123: reverse file order): point-to-point transfers of each rank's rows
   (and IPv6 side rows) straight into their place in the root's table — RCCL over xGMI for device
   tensors, gloo for host tensors.

The local parse is a callback (`LocalParse`), so the same reconcile logic drives the device paths
(`shard_local`: a rank holds only its shard, npr_dev_parse_extract_shard; `device_local`: the whole
capture in one HBM) and the CPU tests (tests/test_parallel.py, gloo, the oracle as the local parser).
"""
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np

from . import _abi

NO_ENTRY = _abi.NO_ENTRY


def shard_bounds(start: int, length: int, world: int):
    """Equal byte ranges [lo, hi) of the record stream [start, length)."""
    span = max(length - start, 0)
    return [(start + span * r // world, start + span * (r + 1) // world) for r in range(world)]


@dataclass
class ShardResult:
    entry: int        # first record start of this range's chain (NO_ENTRY: none found)
    consumed: int     # where the chain leaves the range (>= hi), or the END position (< hi)
    n_records: int
    n_flows: int
    flows: Optional[object] = None      # FLOW_DTYPE rows (numpy), or their bytes as a device tensor
    flows_v6: Optional[object] = None   # the IPv6 side rows, same form


# local(lo, hi, start, speculative) -> ShardResult for the records starting in [start, hi)
LocalParse = Callable[[int, int, int, bool], ShardResult]


def replay(start: int, bounds, results: List[ShardResult]):
    """The serial chain over the ranks' results.  Returns (first_bad_rank, exact_entry) for the
    first rank whose result does not continue the exact chain (None, None when all agree), and
    the per-rank `live` flags (False: after a chain END — the rank contributes nothing)."""
    e = start
    live = []
    for r, ((lo, hi), res) in enumerate(zip(bounds, results)):
        if e is None:                 # the chain ended in an earlier range (Q3)
            live.append(False)
            continue
        if e >= hi:                   # one record spans this whole range: nothing starts here
            if res.entry != e or res.n_records != 0 or res.consumed != e:
                return r, e, live
            live.append(True)
            continue
        if res.entry != e:
            return r, e, live
        live.append(True)
        e = res.consumed if res.consumed >= hi else None
    return None, None, live


def exact_result(local: LocalParse, lo: int, hi: int, e: int) -> ShardResult:
    if e >= hi:
        return ShardResult(entry=e, consumed=e, n_records=0, n_flows=0,
                           flows=np.zeros(0, _abi.FLOW_DTYPE), flows_v6=np.zeros(0, _abi.FLOW_V6_DTYPE))
    return local(lo, hi, e, False)


def parse_sharded_inprocess(local, start: int, length: int, world: int, bounds=None):
    """Every shard in this process (one GPU, or the CPU tests): same reconcile as the
    distributed form.  `local` is one LocalParse for all ranks, or a list of one per rank (each
    rank's shard in its own buffer).  Returns (results, live, rounds)."""
    bounds = bounds or shard_bounds(start, length, world)
    locals_ = local if isinstance(local, (list, tuple)) else [local] * world
    results = [locals_[r](lo, hi, lo, True) if r > 0 else locals_[r](lo, hi, start, False)
               for r, (lo, hi) in enumerate(bounds)]
    rounds = 1
    while True:
        bad, e, live = replay(start, bounds, results)
        if bad is None:
            return results, live, rounds
        results[bad] = exact_result(locals_[bad], *bounds[bad], e)
        rounds += 1


def _gather_meta(res: ShardResult, group, device):
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    mine = torch.tensor([res.entry if res.entry != NO_ENTRY else -1, res.consumed, res.n_records, res.n_flows],
                        dtype=torch.int64, device=device)
    out = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(out, mine, group=group)
    return [ShardResult(entry=(NO_ENTRY if int(t[0]) < 0 else int(t[0])), consumed=int(t[1]),
                        n_records=int(t[2]), n_flows=int(t[3])) for t in (x.cpu() for x in out)]


def parse_sharded(local: LocalParse, start: int, length: int, group=None, device="cpu", bounds=None):
    """Distributed form: this rank parses its range; one all-gather per round reconciles.
    Returns (my_result, metas, live, rounds); `metas` are every rank's final counts."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    bounds = bounds or shard_bounds(start, length, world)
    lo, hi = bounds[rank]
    mine = local(lo, hi, lo, True) if rank > 0 else local(lo, hi, start, False)
    rounds = 1
    while True:
        metas = _gather_meta(mine, group, device)
        bad, e, live = replay(start, bounds, metas)
        if bad is None:
            return mine, metas, live, rounds
        if bad == rank:
            mine = exact_result(local, lo, hi, e)
        rounds += 1


def prefix_offsets(metas: List[ShardResult], live):
    """Global record / flow index of each rank's first record / flow, and the totals."""
    rec_off, flow_off, r_tot, f_tot = [], [], 0, 0
    for m, ok in zip(metas, live):
        rec_off.append(r_tot)
        flow_off.append(f_tot)
        if ok:
            r_tot += m.n_records
            f_tot += m.n_flows
    return rec_off, flow_off, r_tot, f_tot


def merged_positions(metas: List[ShardResult], live):
    """Row of each live rank's first flow in the merged convert_records table (reverse file order:
    the LAST rank's flows come first, src/flow/mod.rs:101-123), and the total."""
    pos, p = {}, 0
    for r in reversed(range(len(metas))):
        if live[r] and metas[r].n_flows:
            pos[r] = p
            p += metas[r].n_flows
    return pos, p


def merge_flows(results: List[ShardResult], live):
    """convert_records order over the whole capture: the ranks' tables in reverse rank order.
    Returns (flows, flows_v6); flows_v6 is None unless every contributing rank has one."""
    parts = [res for res, ok in zip(results[::-1], live[::-1]) if ok and res.n_flows]
    flows = np.concatenate([r.flows for r in parts]) if parts else np.zeros(0, _abi.FLOW_DTYPE)
    if parts and all(r.flows_v6 is not None for r in parts):
        v6 = np.concatenate([r.flows_v6 for r in parts])
    else:
        v6 = None if parts else np.zeros(0, _abi.FLOW_V6_DTYPE)
    return flows, v6


def _as_bytes_tensor(x):
    import torch
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1).copy())
    return x.contiguous().view(-1)


def gather_flow_tables(flows, flows_v6, metas: List[ShardResult], live, group=None, dst=0):
    """Gather every rank's flow rows to `dst` by point-to-point transfers straight into their
    place in the merged table (no padding, no concatenation pass): rank r's rows land at
    merged_positions()[r].  `flows` / `flows_v6` are this rank's n_flows rows as uint8 tensors
    (n_flows * 32 bytes) on the backend's device: CUDA tensors over RCCL (xGMI), CPU tensors over
    gloo; flows_v6 may be None (then no side table is gathered; every rank must pass a side table,
    possibly empty, or every rank None: the transfers are matched pairwise).  Returns (merged, merged_v6)
    uint8 tensors on dst, (None, None) elsewhere."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    pos, total = merged_positions(metas, live)
    with_v6 = flows_v6 is not None
    if dist.get_backend(group) == "gloo":  # gloo moves host tensors only
        flows = flows.cpu() if flows is not None else None
        flows_v6 = flows_v6.cpu() if flows_v6 is not None else None
    gr = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    reqs = []
    if rank != dst:
        if rank in pos:
            n = metas[rank].n_flows
            reqs.append(dist.isend(flows[: n * 32].contiguous(), gr(dst), group=group))
            if with_v6:
                reqs.append(dist.isend(flows_v6[: n * 32].contiguous(), gr(dst), group=group))
        for q in reqs:
            q.wait()
        return None, None
    dev = flows.device if flows is not None else "cpu"
    out = torch.empty(max(total, 1) * 32, dtype=torch.uint8, device=dev)[: total * 32]
    out6 = torch.empty(max(total, 1) * 32, dtype=torch.uint8, device=dev)[: total * 32] if with_v6 else None
    for r, p in sorted(pos.items()):
        n = metas[r].n_flows
        sl = slice(p * 32, (p + n) * 32)
        if r == rank:
            out[sl].copy_(flows[: n * 32])
            if with_v6:
                out6[sl].copy_(flows_v6[: n * 32])
        else:
            reqs.append(dist.irecv(out[sl], gr(r), group=group))
            if with_v6:
                reqs.append(dist.irecv(out6[sl], gr(r), group=group))
    for q in reqs:
        q.wait()
    return out, out6


def gather_flows(mine: ShardResult, metas: List[ShardResult], live, group=None, dst=0):
    """gather_flow_tables over this rank's rows (numpy or tensors); on dst returns the merged
    (flows, flows_v6) as numpy record arrays (flows_v6 None when the ranks hold none)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    ok = live[rank] and mine.n_flows
    empty = torch.zeros(0, dtype=torch.uint8)
    fl = _as_bytes_tensor(mine.flows) if ok else empty
    # every rank must agree on whether a side table moves (a rank with no rows still takes part:
    # the root posts one receive per contributing rank's side rows).  One MAX all-reduce of
    # [holds a side table, has flows but no side table]: side rows move when any rank holds them; a
    # rank without flows counts as an empty side table; a rank with flows but none while another has
    # them would drop IPv6 addresses from the merged table, so every rank raises
    have = mine.flows_v6 is not None
    flag = torch.tensor([1 if have else 0, 1 if (ok and not have) else 0], dtype=torch.int64)
    dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    with_v6, missing = bool(flag[0].item()), bool(flag[1].item())
    if with_v6 and missing:
        raise ValueError("gather_flows: a rank with flows has no IPv6 side table while others have one")
    v6 = (_as_bytes_tensor(mine.flows_v6) if (ok and have) else empty) if with_v6 else None
    out, out6 = gather_flow_tables(fl, v6, metas, live, group=group, dst=dst)
    if out is None:
        return None
    f = out.cpu().numpy().view(_abi.FLOW_DTYPE)
    return f, (out6.cpu().numpy().view(_abi.FLOW_V6_DTYPE) if out6 is not None else None)


def device_aggregate(flows, flows_v6, n, weights=None):
    """Row f4 on this rank's GPU (npr_dev_flow_aggregate): -> (rows, rows_v6, counts, k), the first k
    rows / side rows (uint8, 32 B each) and their int64 counts."""
    import torch
    from . import device
    out, out6, cnt, n_out = device.dev_flow_aggregate(flows, flows_v6, n=n, weights=weights)
    k = int(n_out.item())  # synchronises the stream
    return out[: k * 32], (out6[: k * 32] if flows_v6 is not None else None), cnt[:k].to(torch.int64), k


def gather_distinct_flows(flows, flows_v6, n, weights=None, group=None, dst=0, aggregate=device_aggregate):
    """The distinct-flow table (row f4) of the merged convert_records table, moving only each rank's
    distinct rows (it shrinks the gather when flows repeat).  `flows` / `flows_v6`
    are this rank's n rows (uint8 tensors, n * 32 bytes; flows_v6 for every rank or for none) in the
    merged table's order, which puts the ranks in reverse (merged_positions); `weights` (int64) when
    the rows are already aggregates.  Every rank aggregates its rows; the k_r distinct rows, side
    rows and counts go to `dst` by point-to-point transfers, in reverse rank order; dst aggregates
    them again weighted by the counts.  That is exact: a key's first-seen row (lowest record offset)
    is in some rank's table, each rank's table keeps its first-seen rows in input order, and the
    counts add.  Returns (rows, rows_v6, counts, k) on dst, None elsewhere.  `aggregate` is the
    local table builder (device_aggregate; the CPU tests pass the checker)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    rows, rows6, cnt, k = aggregate(flows, flows_v6, n, weights)
    gloo = dist.get_backend(group) == "gloo"  # gloo moves host tensors only
    if gloo:
        rows, cnt = rows.cpu(), cnt.cpu()
        rows6 = rows6.cpu() if rows6 is not None else None
    dev = rows.device
    mine = torch.tensor([k, 1 if flows_v6 is not None else 0], dtype=torch.int64, device=dev)
    ks = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(ks, mine, group=group)
    ks = [(int(t[0]), int(t[1])) for t in (x.cpu() for x in ks)]
    if len({v for _, v in ks}) != 1:
        raise ValueError("gather_distinct_flows: every rank passes a side table, or none does")
    with_v6 = bool(ks[0][1])
    gr = (lambda r: dist.get_global_rank(group, r)) if group is not None else (lambda r: r)
    reqs = []
    if rank != dst:
        if k:
            reqs.append(dist.isend(rows.contiguous(), gr(dst), group=group))
            if with_v6:
                reqs.append(dist.isend(rows6.contiguous(), gr(dst), group=group))
            reqs.append(dist.isend(cnt.contiguous(), gr(dst), group=group))
        for q in reqs:
            q.wait()
        return None
    total = sum(kr for kr, _ in ks)
    all_rows = torch.empty(max(total, 1) * 32, dtype=torch.uint8, device=dev)[: total * 32]
    all_v6 = torch.empty(max(total, 1) * 32, dtype=torch.uint8, device=dev)[: total * 32] if with_v6 else None
    all_cnt = torch.empty(max(total, 1), dtype=torch.int64, device=dev)[:total]
    p = 0
    for r in reversed(range(world)):
        kr = ks[r][0]
        if not kr:
            continue
        sl, sc = slice(p * 32, (p + kr) * 32), slice(p, p + kr)
        if r == rank:
            all_rows[sl].copy_(rows)
            if with_v6:
                all_v6[sl].copy_(rows6)
            all_cnt[sc].copy_(cnt)
        else:
            reqs.append(dist.irecv(all_rows[sl], gr(r), group=group))
            if with_v6:
                reqs.append(dist.irecv(all_v6[sl], gr(r), group=group))
            reqs.append(dist.irecv(all_cnt[sc], gr(r), group=group))
        p += kr
    for q in reqs:
        q.wait()
    if gloo and flows.is_cuda:  # the merge runs where the local tables were built
        all_rows, all_cnt = all_rows.to(flows.device), all_cnt.to(flows.device)
        all_v6 = all_v6.to(flows.device) if all_v6 is not None else None
    return aggregate(all_rows, all_v6, total, all_cnt)


def device_local(ws, buf, length, endianness=_abi.LITTLE, ref_record=24) -> LocalParse:
    """The product's local parser: npr_dev_parse_extract_range on this rank's GPU (`ws` a
    device.Workspace, `buf` the whole capture in HBM).  Results are copied to the host."""
    def local(lo, hi, start, speculative):
        ws.launch_range(buf, start, hi, endianness=endianness, speculative=speculative,
                        ref_record=ref_record, nbytes=length)
        sm = ws.check()
        flows = ws.flows_np().copy() if ws.flows is not None else None
        v6 = ws.flows_v6_np().copy() if ws.flows_v6 is not None else None
        return ShardResult(entry=int(sm.entry), consumed=int(sm.consumed), n_records=int(sm.n_records),
                           n_flows=int(sm.n_flows), flows=flows, flows_v6=v6)
    return local


class HaloError(RuntimeError):
    """A shard's chain stopped at a record whose bytes run past the shard's buffer (not the end of
    the file): the buffer needs a longer halo."""


def shard_local(ws, buf, base, file_len, endianness=_abi.LITTLE, usec_magic=True, ts_ref=None,
                nbytes=None, chunk_bytes=0, to_host=False) -> LocalParse:
    """The product's local parser over a SHARD held by this device (npr_dev_parse_extract_shard):
    `buf` holds file bytes [base, base + nbytes).  Flow rows stay in HBM (device tensor views of
    the workspace, or host copies with to_host=True)."""
    n = buf.numel() if nbytes is None else int(nbytes)

    def local(lo, hi, start, speculative):
        ws.launch_shard(buf, base, start, hi, endianness=endianness, speculative=speculative,
                        usec_magic=usec_magic, ts_ref=ts_ref, chunk_bytes=chunk_bytes, nbytes=n)
        sm = ws.check()
        if sm.consumed < hi and base + n < file_len and sm.entry != NO_ENTRY:
            incl_end = sm.consumed  # the chain stopped inside the shard: is it the file's end?
            raise HaloError(f"shard [{base}, {base + n}) of a {file_len}-byte capture ends a chain at "
                            f"{incl_end} < stop {hi}: extend its buffer past the last record")
        if to_host:
            fl, v6 = ws.flows_np().copy(), (ws.flows_v6_np().copy() if ws.flows_v6 is not None else None)
        else:
            fl, v6 = ws.flow_rows(sm.n_flows)
        return ShardResult(entry=int(sm.entry), consumed=int(sm.consumed), n_records=int(sm.n_records),
                           n_flows=int(sm.n_flows), flows=fl, flows_v6=v6)
    return local


class GlooExchange:
    """The per-step summaries' all-gather over a gloo group (TCP over loopback on one node)."""

    def __init__(self, group):
        import torch.distributed as dist
        self.group, self.world = group, dist.get_world_size(group)

    def all_gather(self, mine):
        """mine: the same number of bytes on every rank (a CPU uint8 tensor) -> (world, n) uint8."""
        import torch
        import torch.distributed as dist
        out = torch.empty(self.world * mine.numel(), dtype=torch.uint8)
        dist.all_gather(list(out.view(self.world, -1).unbind(0)), mine.contiguous(), group=self.group)
        return out.view(self.world, -1)


class ShmExchange:
    """The per-step summaries' all-gather through node-local shared memory: every
    rank process of one node maps one segment; rank r publishes step k's bytes in its slot
    k mod depth (payload first, then the sequence number k in the slot's own cache line) and reads
    every rank's slot once its sequence number is k.  No socket, no kernel, no collective call:
    ~tens of microseconds where the gloo all-gather over loopback took 0.3 ms at 2 ranks and 1.3 ms
    at 8 (this container).  A slot is rewritten only depth >= 2 exchanges later, after every rank
    has read it (a rank writes step k + 1 only after reading all of step k).  x86 stores are seen
    in program order, so a reader that sees k sees k's payload.
    Built over a process group only to agree on the segment's name (all ranks on one host)."""

    HEADER = 64  # the sequence number's own cache line, then the payload

    def __init__(self, group=None, slot_bytes=1024, depth=4, directory="/dev/shm", timeout_s=120.0):
        import os
        import socket
        import uuid
        import torch.distributed as dist
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        hosts = [None] * self.world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise RuntimeError(f"ShmExchange: the ranks are on more than one host ({sorted(set(hosts))})")
        name = [f"npr_xchg_{os.getpid()}_{uuid.uuid4().hex}" if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(name, src=src, group=group)
        path = os.path.join(directory, name[0])
        self.slot_bytes, self.depth, self.timeout_s = int(slot_bytes), max(2, int(depth)), float(timeout_s)
        self.rec = (self.HEADER + self.slot_bytes + 63) // 64 * 64
        size = self.world * self.depth * self.rec
        ok = [True]
        if self.rank == 0:
            try:
                with open(path, "wb") as f:
                    f.truncate(size)
            except OSError:
                ok = [False]
        dist.broadcast_object_list(ok, src=src, group=group)
        if not ok[0]:
            raise RuntimeError(f"ShmExchange: cannot create {path}")
        try:
            self.mm = np.memmap(path, dtype=np.uint8, mode="r+", shape=(size,))
            mapped = True
        except (OSError, ValueError):
            mapped = False
        # every rank mapped (or failed): the name is no longer needed, and every rank agrees on the
        # outcome (one rank falling back alone would leave the others in an exchange it never joins)
        flags = [None] * self.world
        dist.all_gather_object(flags, mapped, group=group)
        if self.rank == 0:
            os.unlink(path)
        if not all(flags):
            raise RuntimeError(f"ShmExchange: {path} could not be mapped on every rank")
        grid = self.mm.reshape(self.world, self.depth, self.rec)
        self.seqs = grid.view(np.uint64)[:, :, 0]  # [rank, slot]: the slot's sequence number
        self.pay = grid[:, :, self.HEADER:]         # [rank, slot, byte]
        self.seq = 0
        try:  # the spin in C (npr_shm_all_gather: acquire / release atomics); numpy otherwise
            self.lib = _abi.load_library()
        except (ImportError, OSError):
            self.lib = None

    def all_gather(self, mine):
        """mine: the same number (<= slot_bytes) of bytes on every rank -> (world, n) uint8 tensor."""
        import time
        import torch
        a = (mine.numpy() if hasattr(mine, "numpy") else np.asarray(mine)).view(np.uint8).reshape(-1)
        n = a.size
        if n > self.slot_bytes:
            raise ValueError(f"ShmExchange: {n} bytes > slot of {self.slot_bytes}")
        self.seq += 1
        if self.lib is not None:
            a = np.ascontiguousarray(a)
            out = np.empty((self.world, n), dtype=np.uint8)
            st = self.lib.npr_shm_all_gather(self.mm.ctypes.data, self.world, self.rank, self.depth, self.rec, self.seq,
                                             a.ctypes.data, n, out.ctypes.data, int(self.timeout_s * 1000))
            if st != _abi.OK:
                raise RuntimeError(f"ShmExchange: exchange {self.seq} failed (status {st}: a rank did not publish)")
            return torch.from_numpy(out)
        d = self.seq % self.depth
        self.pay[self.rank, d, :n] = a
        self.seqs[self.rank, d] = self.seq  # published after the payload
        col = self.seqs[:, d]
        spins, t0 = 0, None
        while not (col == self.seq).all():
            spins += 1
            if spins > 64:
                time.sleep(0)  # yield: ranks may share host cores
                if t0 is None:
                    t0 = time.monotonic()
                elif time.monotonic() - t0 > self.timeout_s:
                    late = [int(r) for r in np.nonzero(col != self.seq)[0]]
                    raise RuntimeError(f"ShmExchange: ranks {late} did not publish step {self.seq}")
        return torch.from_numpy(np.ascontiguousarray(self.pay[:, d, :n]))


def record_range_shards(n_records, world, record_bytes=80, header=24):
    """C4 layout: a fixed-stride capture of n_records split by record range, rank g
    holding records [g*R, (g+1)*R): returns per rank (base, start, stop, speculative) in file
    offsets, rank 0's buffer starting at byte 0 (the global header)."""
    out = []
    for g in range(world):
        r0, r1 = n_records * g // world, n_records * (g + 1) // world
        lo, hi = header + record_bytes * r0, header + record_bytes * r1
        out.append((0 if g == 0 else lo, header if g == 0 else lo, hi, g > 0))
    return out


class DeviceShardedParse:
    """The device-resident multi-GPU step (C4 / C5, SURVEY.md 8 row e), one rank per GPU:

      launch this rank's shard (npr_dev_parse_extract_shard, chained resident launches) ->
      ONE RCCL all-gather of every rank's device summary {n_records, n_flows, consumed, entry}
      straight from HBM (stream-ordered behind the parse, no host round trip in between) ->
      replay the serial chain on the host; a rank whose speculated entry is contradicted re-parses
      from the exact one and the exchange repeats (never with a plausible speculation).

    The flow rows stay in this rank's HBM (`rows()`) until gather_flow_tables() moves them.
    `bounds` are every rank's (lo, hi) record-start ranges; this rank's buffer holds file bytes
    [base, base + nbytes)."""

    def __init__(self, ws, buf, base, bounds, file_len, endianness=_abi.LITTLE, usec_magic=True, ts_ref=None,
                 start=24, group=None, nbytes=None, chunk_bytes=0, meta_group=None, depth=2, exchange=None):
        import torch
        import torch.distributed as dist
        self.ws, self.buf, self.base, self.bounds = ws, buf, int(base), bounds
        self.file_len, self.e, self.usec, self.ts_ref = int(file_len), endianness, usec_magic, ts_ref
        self.start, self.group = int(start), group
        self.nbytes = buf.numel() if nbytes is None else int(nbytes)
        self.chunk = int(chunk_bytes)
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.gathered = torch.zeros(self.world * ws.summary.numel(), dtype=torch.uint8, device=ws.summary.device)
        # launch_step / finish_steps: up to `depth` steps in flight, each with its own exchange buffers
        # (device + page-locked host copies)
        pin = ws.summary.device.type == "cuda"
        self.depth = max(2, int(depth))
        self._g2 = [torch.zeros_like(self.gathered) for _ in range(self.depth)]
        self._h2 = [torch.zeros(self.gathered.numel(), dtype=torch.uint8, pin_memory=pin) for _ in range(self.depth)]
        self._ev2 = [torch.cuda.Event() if pin else None for _ in range(self.depth)]
        self._k = 0
        self.pending = []
        # exchange (ShmExchange: node-local shared memory) or meta_group (a gloo group over the same
        # ranks): the 64-B summaries move on the HOST (the parse stores its summary into page-locked
        # host memory, all-gathered in finish_steps), so no collective kernel or stream join sits
        # between two parses; the flow rows still go over RCCL
        self.meta_group = meta_group
        self.xchg = exchange if exchange is not None else (GlooExchange(meta_group) if meta_group is not None else None)
        # finish_steps(n) exchanges n summaries at once: a shared-memory slot must hold `depth` of them
        # (checked here, before any work is in flight)
        slot = getattr(self.xchg, "slot_bytes", None)
        if slot is not None and self.depth * ws.summary.numel() > slot:
            raise ValueError(f"DeviceShardedParse: depth {self.depth} x {ws.summary.numel()}-B summaries exceed the "
                             f"exchange's {slot}-B slot (ShmExchange(slot_bytes=...))")
        # every rank's buffer end, once: a chain that stops short of its shard's stop inside a buffer
        # that does not reach the file's end is a HaloError, and every rank must decide it alike
        # (the others would otherwise wait in their next collective for the rank that raised)
        if self.xchg is not None:
            mine = torch.tensor([self.base + self.nbytes], dtype=torch.int64)
            self.buf_ends = [int(x) for x in self.xchg.all_gather(mine.view(torch.uint8)).view(torch.int64).reshape(-1)]
        else:
            on_host = dist.get_backend(group) == "gloo"
            dev = torch.device("cpu") if on_host else ws.summary.device
            mine = torch.tensor([self.base + self.nbytes], dtype=torch.int64, device=dev)
            ends = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(self.world)]
            dist.all_gather(ends, mine, group=group)
            self.buf_ends = [int(e.item()) for e in ends]
        if self.xchg is not None:
            # the parse's last link stores its summary straight into page-locked host memory: the
            # host waits for an event behind the parse, no copy kernel needs a CU the next parse holds
            self._sum2 = [torch.zeros(ws.summary.numel(), dtype=torch.uint8, pin_memory=pin) for _ in range(self.depth)]
            self._gh = torch.zeros(self.gathered.numel(), dtype=torch.uint8)
            self._bind(self._sum2[0])

    def _check_halo(self, metas, live):
        """Raise HaloError on EVERY rank when any live rank's chain stopped short of its shard's stop
        inside a buffer that ends before the file does (it needs a longer halo)."""
        bad = [r for r in range(self.world)
               if live[r] and metas[r].consumed < self.bounds[r][1] and self.buf_ends[r] < self.file_len]
        if bad:
            raise HaloError(f"ranks {bad}: a chain stopped inside a short buffer at "
                            f"{[metas[r].consumed for r in bad]} < stop {[self.bounds[r][1] for r in bad]}")

    def _launch(self, start, speculative):
        lo, hi = self.bounds[self.rank]
        self.ws.summary.zero_()  # an unwritten summary (a launch that did not complete) reads epoch 0
        self.ws.launch_shard(self.buf, self.base, start, hi, endianness=self.e, speculative=speculative,
                             usec_magic=self.usec, ts_ref=self.ts_ref, chunk_bytes=self.chunk, nbytes=self.nbytes)

    def _empty_summary(self, e):
        """The summary of a shard no record starts in (the exact entry e is at or past its stop):
        {entry = consumed = e, no records, no flows}, what exact_result() builds on the host path.
        Written in place of a launch, so this rank keeps taking part in the exchange."""
        import torch
        s = np.zeros(1, dtype=_abi.SUMMARY_DTYPE)
        s["entry"], s["consumed"], s["n_records"], s["n_flows"] = e, e, 0, 0
        s["flags"], s["epoch"] = 0, 1  # epoch != 0: a completed parse (_metas)
        if torch.cuda.is_available() and self.ws.summary.is_cuda:
            torch.cuda.current_stream().synchronize()  # no launch of this step still writes the summary
        raw = torch.from_numpy(s.view(np.uint8).copy())
        self.ws.summary.zero_()
        self.ws.summary[: raw.numel()].copy_(raw.to(self.ws.summary.device))

    def _metas(self, host_bytes):
        g = host_bytes.numpy().reshape(self.world, -1)[:, :40].copy().view(_abi.SUMMARY_DTYPE).reshape(-1)
        if (g["epoch"] == 0).any() or (g["flags"] != 0).any():
            bad = [int(r) for r in range(self.world) if g["epoch"][r] == 0 or g["flags"][r] != 0]
            raise RuntimeError(f"shard parse did not complete or overflowed on ranks {bad}")
        return [ShardResult(entry=int(x["entry"]), consumed=int(x["consumed"]), n_records=int(x["n_records"]),
                            n_flows=int(x["n_flows"])) for x in g]

    def _bind(self, summary):
        if hasattr(self.ws, "use_summary"):
            self.ws.use_summary(summary)
        else:
            self.ws.summary = summary

    def _exchange(self):
        import torch
        import torch.distributed as dist
        if self.xchg is not None:  # the summary is in host memory: wait for the parse, gather on the host
            if torch.cuda.is_available():
                torch.cuda.current_stream().synchronize()
            return self._metas(self.xchg.all_gather(self.ws.summary).reshape(-1))
        dist.all_gather_into_tensor(self.gathered, self.ws.summary, group=self.group)
        return self._metas(self.gathered.cpu())

    def launch_step(self):
        """The step's device work without waiting for it: this rank's parse from its speculated (or
        known) start, the all-gather of the summaries and their copy to page-locked host memory,
        all stream-ordered.  finish_step() replays the chain on the host, so the host work of step k
        overlaps the parse of step k+1 (at most `depth` steps in flight: the exchange buffers rotate)."""
        import torch.distributed as dist
        if len(self.pending) >= self.depth:
            raise RuntimeError("finish_steps() the oldest steps first")
        import torch
        lo, hi = self.bounds[self.rank]
        i = self._k % self.depth
        self._k += 1
        if self.xchg is not None:
            self._bind(self._sum2[i])
            self._launch(self.start if self.rank == 0 else lo, self.rank > 0)
            if self._ev2[i] is not None:
                self._ev2[i].record()
        else:
            self._launch(self.start if self.rank == 0 else lo, self.rank > 0)
            dist.all_gather_into_tensor(self._g2[i], self.ws.summary, group=self.group)
            self._h2[i].copy_(self._g2[i], non_blocking=True)
            if self._ev2[i] is not None:
                self._ev2[i].record()
        self.pending.append(i)

    def finish_step(self):
        """-> (metas, live, rounds) of the oldest launch_step()."""
        return self.finish_steps(1)

    def finish_steps(self, n):
        """Finish the n oldest launch_step()s; -> (metas, live, rounds) of the last of them.  With a
        host metadata group their summaries move in ONE all-gather (n x 64 B per rank), so a host
        exchange slower than a parse is paid once per n steps.  Every rank must pass the same n
        (the bench's loop decides it from len(pending), which all ranks share).  A contradicted
        speculation (never on C4) drains the device and runs the whole step again synchronously
        (every rank decides the same from the same summaries, so the collectives stay matched)."""
        import torch
        import torch.distributed as dist
        n = min(int(n), len(self.pending))
        if n <= 0:
            raise RuntimeError("no step in flight")
        slots = [self.pending.pop(0) for _ in range(n)]
        for i in slots:
            if self._ev2[i] is not None:
                self._ev2[i].synchronize()
        if self.xchg is not None:  # the summaries' all-gather on the host, all n steps at once
            sn = self._sum2[0].numel()
            mine = torch.cat([self._sum2[i] for i in slots])
            per = self.xchg.all_gather(mine).view(self.world, n, sn)
            for j, i in enumerate(slots):
                self._h2[i].copy_(per[:, j, :].reshape(-1))
        res = None
        for i in slots:
            metas = self._metas(self._h2[i])
            bad, e, live = replay(self.start, self.bounds, metas)
            if bad is not None:
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
                while self.pending:  # later steps parsed from the same speculation: redone below
                    self.pending.pop(0)
                return self.step()
            self._check_halo(metas, live)
            self.metas, self.live = metas, live
            res = (metas, live, 1)
        return res

    def step(self):
        """-> (metas, live, rounds).  Raises HaloError (on every rank) when a chain stops short of a buffer end."""
        lo, hi = self.bounds[self.rank]
        self._launch(self.start if self.rank == 0 else lo, self.rank > 0)
        rounds = 1
        while True:
            metas = self._exchange()
            bad, e, live = replay(self.start, self.bounds, metas)
            if bad is None:
                break
            if bad == self.rank:
                if e >= hi:  # one record spans this whole shard: no record starts here (replay's rule)
                    self._empty_summary(e)
                else:
                    self._launch(e, False)
            else:  # keep the stream order: an empty launch is not needed, the others just re-gather
                pass
            rounds += 1
        self._check_halo(metas, live)
        self.metas, self.live = metas, live
        return metas, live, rounds

    def rows(self):
        m = self.metas[self.rank]
        return self.ws.flow_rows(m.n_flows if self.live[self.rank] else 0)


def supervise_ranks(target, rank_args, poll_s=0.2, grace_s=10.0):
    """Start one spawned process per rank (`target(*rank_args[r])`), wait for all of them, and end
    the others as soon as one exits with a non-zero code: a rank that failed must not leave the rest
    waiting in a collective (or in a shared-memory exchange) for it.  Returns the exit codes, a
    terminated rank's as the negative signal number."""
    import multiprocessing as mp
    import time
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of the parent's state is inherited
    procs = [ctx.Process(target=target, args=tuple(a)) for a in rank_args]
    for p in procs:
        p.start()
    try:
        while any(p.exitcode is None for p in procs):
            if any(p.exitcode not in (None, 0) for p in procs):
                for p in procs:
                    if p.exitcode is None:
                        p.terminate()
                t0 = time.monotonic()
                for p in procs:
                    p.join(max(0.1, grace_s - (time.monotonic() - t0)))
                for p in procs:
                    if p.exitcode is None:
                        p.kill()
                        p.join()
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.exitcode is None:
                p.kill()
                p.join()
    return [p.exitcode for p in procs]
