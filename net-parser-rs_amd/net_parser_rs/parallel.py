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
   (src/flow/mod.rs:101-123: reverse file order).

The local parse is a callback (`LocalParse`), so the same reconcile logic drives the device path
(`device_local`) and the CPU tests (tests/test_parallel.py, gloo, the oracle as the local parser).
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
    flows: Optional[np.ndarray] = None      # FLOW_DTYPE rows, convert_records order (reverse)
    flows_v6: Optional[np.ndarray] = None


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


def parse_sharded_inprocess(local: LocalParse, start: int, length: int, world: int):
    """Every shard in this process (one GPU, or the CPU tests): same reconcile as the
    distributed form.  Returns (results, live, rounds)."""
    bounds = shard_bounds(start, length, world)
    results = [local(lo, hi, lo, r > 0) if r > 0 else local(lo, hi, start, False)
               for r, (lo, hi) in enumerate(bounds)]
    rounds = 1
    while True:
        bad, e, live = replay(start, bounds, results)
        if bad is None:
            return results, live, rounds
        results[bad] = exact_result(local, *bounds[bad], e)
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


def parse_sharded(local: LocalParse, start: int, length: int, group=None, device="cpu"):
    """Distributed form: this rank parses its range; one all-gather per round reconciles.
    Returns (my_result, metas, live, rounds); `metas` are every rank's final counts."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    bounds = shard_bounds(start, length, world)
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


def merge_flows(results: List[ShardResult], live):
    """convert_records order over the whole capture: the ranks' tables in reverse rank order."""
    parts = [res.flows for res, ok in zip(results[::-1], live[::-1]) if ok and res.n_flows]
    return np.concatenate(parts) if parts else np.zeros(0, _abi.FLOW_DTYPE)


def gather_flows(mine: ShardResult, metas: List[ShardResult], live, group=None, dst=0):
    """Gather every rank's flow rows to `dst` (padded to the largest count) and merge there."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    width = max([m.n_flows for m in metas] + [1])
    buf = torch.zeros(width * 32, dtype=torch.uint8)
    if live[rank] and mine.n_flows:
        buf[: mine.n_flows * 32] = torch.from_numpy(mine.flows.view(np.uint8).copy())
    bufs = [torch.zeros_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    rows = [ShardResult(m.entry, m.consumed, m.n_records, m.n_flows,
                        flows=b[: m.n_flows * 32].numpy().view(_abi.FLOW_DTYPE)) for m, b in zip(metas, bufs)]
    return merge_flows(rows, live)


def device_local(ws, buf, length, endianness=_abi.LITTLE, ref_record=24) -> LocalParse:
    """The product's local parser: npr_dev_parse_extract_range on this rank's GPU (`ws` a
    device.Workspace, `buf` the capture — or this rank's range plus a halo — in HBM)."""
    def local(lo, hi, start, speculative):
        ws.launch_range(buf, start, hi, endianness=endianness, speculative=speculative,
                        ref_record=ref_record, nbytes=length)
        sm = ws.check()
        flows = ws.flows_np().copy() if ws.flows is not None else None
        v6 = ws.flows_v6_np().copy() if ws.flows_v6 is not None else None
        return ShardResult(entry=int(sm.entry), consumed=int(sm.consumed), n_records=int(sm.n_records),
                           n_flows=int(sm.n_flows), flows=flows, flows_v6=v6)
    return local
