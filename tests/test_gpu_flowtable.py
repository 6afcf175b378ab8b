"""Row f4: the distinct-flow table on the device (npr_dev_flow_aggregate) against the CPU checker
derived from the oracle's per-record flows (tests/_flowtable_ref.py).

Inputs are the device's own convert_records tables (right-aligned flow rows of a flows-only parse),
so the chain device parse -> device aggregate is what is checked, bit for bit: the first-seen rows,
their order, the counts, and the distinct count.  Merging (the multi-GPU use: one table per GPU,
then an aggregate of the aggregates weighted by their counts) must equal one aggregate of all rows.
"""
import numpy as np
import pytest
import torch

import _flowtable_ref
import _oracle
from net_parser_rs import _abi, device, synth

pytestmark = pytest.mark.gpu


def device_table(blob):
    n = len(blob) // 16 + 1
    ws = device.Workspace(n, n, records=False, status=False)
    buf = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
    ws.launch(buf, start=24)
    sm = ws.check()
    fl, f6 = ws.flow_rows()
    return fl.clone(), f6.clone(), int(sm.n_flows)


def check(fl, f6, n, weights=None, cap=None):
    flows = fl[: n * 32].cpu().numpy().view(_abi.FLOW_DTYPE)
    v6 = f6[: n * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE) if f6 is not None else np.zeros(n, _abi.FLOW_V6_DTYPE)
    w = None if weights is None else weights.cpu().numpy()
    rows, counts = _flowtable_ref.aggregate(flows, v6, w)
    out, out6, cnt, n_out = device.dev_flow_aggregate(fl, f6, n=n, weights=weights, cap=cap)
    torch.cuda.synchronize()
    k = int(n_out.item())
    assert k == len(rows)
    m = min(k, n if cap is None else cap)
    assert out[: m * 32].cpu().numpy().tobytes() == flows[rows[:m]].tobytes()
    if f6 is not None:
        assert out6[: m * 32].cpu().numpy().tobytes() == v6[rows[:m]].tobytes()
    assert np.array_equal(cnt[:m].cpu().numpy().astype(np.uint64), counts[:m])
    return out, out6, cnt, k


@pytest.mark.parametrize("n_flows", [1, 50, 5000])
def test_flow_mix_matches_checker(n_flows):
    blob = synth.flow_mix(40_000, n_flows=n_flows)
    fl, f6, n = device_table(blob)
    # the device table is the oracle's convert_records table
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    wf, _ = _oracle.convert_records(blob, recs)
    assert fl.cpu().numpy().tobytes() == wf.tobytes()
    check(fl, f6, n)


def test_capacity_ipv4_only_and_empty():
    blob = synth.flow_mix(10_000, n_flows=300, seed=3)
    fl, f6, n = device_table(blob)
    check(fl, f6, n, cap=17)
    out, out6, cnt, n_out = device.dev_flow_aggregate(fl[:0], None, n=0)
    torch.cuda.synchronize()
    assert int(n_out.item()) == 0
    c2 = synth.fixed64(20_000)  # IPv4 only, every 5-tuple distinct: no side table needed
    fl2, _, n2 = device_table(c2)
    _, _, cnt2, k2 = check(fl2, None, n2)
    assert k2 == n2 and bool((cnt2[:k2] == 1).all())


def test_merge_of_per_gpu_aggregates_equals_one_aggregate():
    blob = synth.flow_mix(60_000, n_flows=2000, seed=9)
    fl, f6, n = device_table(blob)
    h = n // 2  # two "GPUs": rows [0, h) and [h, n) of the table
    parts = [(fl[: h * 32], f6[: h * 32], h), (fl[h * 32: n * 32], f6[h * 32: n * 32], n - h)]
    aggs = []
    for a, a6, m in parts:
        out, out6, cnt, n_out = device.dev_flow_aggregate(a.contiguous(), a6.contiguous(), n=m)
        torch.cuda.synchronize()
        k = int(n_out.item())
        aggs.append((out[: k * 32], out6[: k * 32], cnt[:k], k))
    cat = torch.cat([a[0] for a in aggs]).contiguous()
    cat6 = torch.cat([a[1] for a in aggs]).contiguous()
    w = torch.cat([a[2] for a in aggs]).contiguous()
    mk = sum(a[3] for a in aggs)
    check(cat, cat6, mk, weights=w)  # the merge itself, against the checker with weights
    m_out, m_out6, m_cnt, m_n = device.dev_flow_aggregate(cat, cat6, n=mk, weights=w)
    f_out, f_out6, f_cnt, f_n = device.dev_flow_aggregate(fl, f6, n=n)
    torch.cuda.synchronize()
    assert int(m_n.item()) == int(f_n.item())

    def as_map(o, o6, c, k):
        rows = o[: k * 32].cpu().numpy().view(_abi.FLOW_DTYPE)
        r6 = o6[: k * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
        ks = _flowtable_ref.keys(rows, r6)
        return {key: (rows[i].tobytes(), int(c[i])) for i, key in enumerate(ks)}

    assert as_map(m_out, m_out6, m_cnt, int(m_n.item())) == as_map(f_out, f_out6, f_cnt, int(f_n.item()))


def test_c2_full_size_all_distinct():
    blob = synth.fixed64(1_000_000)
    fl, _, n = device_table(blob)
    out, out6, cnt, n_out = device.dev_flow_aggregate(fl, None, n=n)
    torch.cuda.synchronize()
    assert int(n_out.item()) == n == 1_000_000
    assert bool((cnt == 1).all())
    assert torch.equal(out[: n * 32], fl[: n * 32])  # every row is its own first-seen row, input order kept


def test_tied_first_seen_offsets_resolve_to_the_lowest_row():
    """Rows that share the first-seen offset (the same table twice, i.e. each record listed twice;
    tables of two captures merged, both starting at offset 24): one output row per flow, the
    lowest tied row, counts summed (every tied row was marked first)."""
    blob = synth.flow_mix(30_000, n_flows=700, seed=21)
    fl, f6, n = device_table(blob)
    twice = torch.cat([fl[: n * 32], fl[: n * 32]]).contiguous()
    twice6 = torch.cat([f6[: n * 32], f6[: n * 32]]).contiguous()
    _, _, cnt, k = check(twice, twice6, 2 * n)
    single = device.dev_flow_aggregate(fl, f6, n=n)
    torch.cuda.synchronize()
    assert k == int(single[3].item())
    assert bool((cnt[:k] % 2 == 0).all())
    # two different captures merged: their first records both sit at offset 24
    blob2 = synth.flow_mix(20_000, n_flows=300, seed=22)
    fl2, f62, n2 = device_table(blob2)
    cat = torch.cat([fl[: n * 32], fl2[: n2 * 32]]).contiguous()
    cat6 = torch.cat([f6[: n * 32], f62[: n2 * 32]]).contiguous()
    check(cat, cat6, n + n2)


def test_row_cap_is_rejected():
    fl = torch.zeros(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(Exception):
        device.dev_flow_aggregate(fl, None, n=(1 << 30) + 1, cap=0)


# ---- k_agg_insert's workgroup dedupe: rows of different keys whose 32-bit hashes collide ----------
def _mix64(x):
    x = x ^ (x >> np.uint64(30))
    x = x * np.uint64(0xBF58476D1CE4E5B9)
    x = x ^ (x >> np.uint64(27))
    x = x * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _key_h32(words):
    """npr_flowtable.hip key_hash over IPv4 keys {kind, ports, src ip, dst ip}: (hash >> 32) | 1."""
    h = np.full(len(words), 0x9E3779B97F4A7C15, np.uint64)
    for i in range(4):
        h = _mix64(h ^ (words[:, i].astype(np.uint64) * np.uint64(0xFF51AFD7ED558CCD) + np.uint64(i)))
    return (h >> np.uint64(32)) | np.uint64(1)


def test_hash32_collisions_inside_a_workgroup():
    rng = np.random.default_rng(21)
    m = 400_000  # ~19 expected pairs of equal 32-bit hashes among m random keys
    words = np.zeros((m, 4), np.uint32)
    words[:, 0] = rng.choice([0, _abi.KIND_UDP], m)
    words[:, 1:] = rng.integers(0, 2**32, (m, 3), dtype=np.uint32)
    h32 = _key_h32(words)
    order = np.argsort(h32, kind="stable")
    dup = np.nonzero(h32[order][1:] == h32[order][:-1])[0]
    pairs = [(order[d], order[d + 1]) for d in dup if (words[order[d]] != words[order[d + 1]]).any()]
    assert len(pairs) >= 4
    # each pair's two keys several times inside one 1024-row block (either may lead its LDS entry),
    # among distinct filler rows
    keys = []
    for a, b in pairs[:8]:
        blk = [a, b, a, a, b] if len(keys) % 2 == 0 else [b, a, b]
        keys += list(rng.permutation(blk)) + list(rng.integers(0, m, 40))
    keys = np.array(keys + list(rng.integers(0, m, 5000)))
    n = len(keys)
    rows = np.zeros(n, _abi.FLOW_DTYPE)
    raw = rows.view(np.uint32).reshape(n, 8)
    raw[:, 0], raw[:, 1], raw[:, 2] = words[keys, 2], words[keys, 3], words[keys, 1]
    raw[:, 3:6] = rng.integers(0, 2**32, (n, 3), dtype=np.uint32)  # vlan / MACs: not part of the key
    off = 24 + 64 * rng.permutation(n).astype(np.uint64)  # first-seen is not row order
    raw[:, 6] = (raw[:, 6] & 0xFFFF) | (words[keys, 0] << 16) | ((off & 0xFF).astype(np.uint32) << 24)
    raw[:, 7] = (off >> np.uint64(8)).astype(np.uint32)
    fl = torch.from_numpy(rows.view(np.uint8).copy()).cuda()
    check(fl, None, n)
    w = torch.from_numpy(rng.integers(1, 1000, n).astype(np.int64)).cuda()
    check(fl, None, n, weights=w)


@pytest.mark.parametrize("reps", [3, 16385])
def test_tiled_table_every_flow_tied(reps):
    """A 1024-row table repeated: every copy of a row carries the same record offset, so each flow's
    first-seen row is decided by the tie rule (lowest row: the first copy).  reps * 1024 > 2^24 runs
    the two-pass tie path (k_agg_tie); below that the packed {offset, row} minimum settles it."""
    blob = synth.flow_mix(1500, n_flows=300, seed=5)
    fl, f6, n = device_table(blob)
    t = 1024
    assert n >= t
    flows = fl[: t * 32].cpu().numpy().view(_abi.FLOW_DTYPE)
    v6 = f6[: t * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
    rows, counts = _flowtable_ref.aggregate(flows, v6, None)
    big, big6 = fl[: t * 32].repeat(reps), f6[: t * 32].repeat(reps)
    out, out6, cnt, n_out = device.dev_flow_aggregate(big, big6, n=t * reps)
    torch.cuda.synchronize()
    k = int(n_out.item())
    assert k == len(rows)
    assert out[: k * 32].cpu().numpy().tobytes() == flows[rows].tobytes()
    assert out6[: k * 32].cpu().numpy().tobytes() == v6[rows].tobytes()
    assert np.array_equal(cnt[:k].cpu().numpy().astype(np.uint64), counts.astype(np.uint64) * np.uint64(reps))
    del big, big6, out, out6, cnt
    torch.cuda.empty_cache()


def test_distinct_flow_gather_on_the_device_world1():
    """parallel.gather_distinct_flows with the device aggregate (world 1 over gloo: the local
    table, the all-gather of its size, then the weighted merge on the GPU)."""
    import socket
    import torch.distributed as dist
    from net_parser_rs import parallel
    blob = synth.flow_mix(30_000, n_flows=700, seed=12)
    fl, f6, n = device_table(blob)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        rows, rows6, cnt, k = parallel.gather_distinct_flows(fl[: n * 32], f6[: n * 32], n)
    finally:
        dist.destroy_process_group()
    flows = fl[: n * 32].cpu().numpy().view(_abi.FLOW_DTYPE)
    v6 = f6[: n * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
    want, counts = _flowtable_ref.aggregate(flows, v6, None)
    assert k == len(want) < n
    assert rows.cpu().numpy().tobytes() == flows[want].tobytes()
    assert rows6.cpu().numpy().tobytes() == v6[want].tobytes()
    assert np.array_equal(cnt.cpu().numpy().astype(np.uint64), counts)


@pytest.mark.parametrize("m", [1, 2, 100, 511, 512, 513, 1023, 1024, 1025])
def test_small_tables_read_without_device_sync(m):
    """Tables around the 512-row insert and 1024-row compaction block edges, the count read by
    .item() on the default stream with no torch.cuda.synchronize(): the device layer fences its
    side stream to the default stream (device._On), so the read waits for the aggregate."""
    blob = synth.flow_mix(3_000, n_flows=400, seed=77)
    fl, f6, n = device_table(blob)
    assert n >= m
    flows = fl[: m * 32].cpu().numpy().view(_abi.FLOW_DTYPE)
    v6 = f6[: m * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
    want, counts = _flowtable_ref.aggregate(flows, v6, None)
    out, out6, cnt, n_out = device.dev_flow_aggregate(fl[: m * 32].contiguous(), f6[: m * 32].contiguous(), n=m)
    k = int(n_out.item())
    assert k == len(want)
    assert out[: k * 32].cpu().numpy().tobytes() == flows[want].tobytes()
    assert np.array_equal(cnt[:k].cpu().numpy().astype(np.uint64), counts)
