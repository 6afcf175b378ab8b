"""Parity at the BASELINE.json configurations' full sizes, on one GPU (SURVEY.md §8 rows a–e):

- C2: the exact bench launch (1M x 64-B records, one resident launch, flows-only workspace) is
  byte-compared with the oracle;
- C3: the full 8M-record variable-length capture (6.4 GB, chained resident launches) is
  byte-compared with the oracle;
- C4: the 64M-record capture sharded by record range into 8 shards, each shard in its OWN HBM
  buffer holding only its file bytes (npr_dev_parse_extract_shard, exactly what each rank of the
  8-GPU run holds), reconciled by the one-exchange replay and merged in reverse rank order: bit-exact
  against the oracle at 16M records, and at the full 64M;
- C5 substitute (the 4SICS capture is absent, .MISSING_LARGE_BLOBS:1): a quirk-corpus tile
  repeated to 10 GB, sharded by BYTE range with halos (speculated starts inside adversarial
  payloads), every tile of the merged table compared with the single-tile oracle golden.

The oracle (tests/_oracle.py) is the checker only.  Heavy cases print progress so a long run is
never silent."""
import time

import numpy as np
import pytest
import torch

import _oracle
from net_parser_rs import _abi, device, parallel, synth

pytestmark = pytest.mark.gpu


def log(msg):
    print(f"[{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def to_dev(a):
    a = np.frombuffer(a, dtype=np.uint8) if isinstance(a, (bytes, bytearray)) else a
    t = torch.empty(a.size, dtype=torch.uint8, device="cuda")
    t.copy_(torch.from_numpy(a))
    return t


def oracle_flows(blob):
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert rc == 0
    flows, v6 = _oracle.convert_records(blob, recs)
    return hdr, recs, cons, flows, v6


def v6_rows(flows, v6):
    m = (flows["kind"] & _abi.KIND_IPV6) != 0
    return v6[m]


def test_c2_bench_launch_bit_exact():
    """The exact launch bench.py times: 1M records, one k_parse_resident dispatch."""
    blob = synth.fixed64(1_000_000)
    hdr, recs, cons, flows, _ = oracle_flows(blob)
    n = len(recs)
    ws = device.Workspace(record_cap=n, flow_cap=n, records=False, offsets=False, status=False,
                          flows=True, flows_v6=True)
    ws.launch(to_dev(blob), start=24, endianness=hdr.endianness)
    sm = ws.check()
    assert ws.ctx.lib.npr_ctx_last_pass(ws.ctx.handle) == _abi.PASS_RESIDENT
    assert (sm.n_records, sm.n_flows, sm.consumed) == (n, len(flows), cons)
    assert ws.flows_np().tobytes() == flows.tobytes()


def test_c3_full_8m_bit_exact():
    log("C3: generating 8M variable-length records")
    blob = synth.variable_mix(8_000_000)
    log(f"C3: {len(blob)} B; oracle")
    hdr, recs, cons, flows, _ = oracle_flows(blob)
    n = len(recs)
    assert n == 8_000_000
    ws = device.Workspace(record_cap=n, flow_cap=n, records=False, offsets=False, status=False,
                          flows=True, flows_v6=True)
    buf = to_dev(blob)
    lib, h = ws.ctx.lib, ws.ctx.handle
    # the default choice (the sparse record walk: ~800-B records), then the chained resident launches
    for mode, want_pass in ((0, _abi.PASS_SPARSE), (1, _abi.PASS_RESIDENT)):
        log(f"C3: device (NPR_OPT_SPARSE {mode})")
        ws.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, mode))
        try:
            ws.flows.zero_()
            ws.launch(buf, start=24, endianness=hdr.endianness)
            sm = ws.check()
            assert lib.npr_ctx_last_pass(h) == want_pass
        finally:
            ws.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, 0))
        assert (sm.n_records, sm.n_flows, sm.consumed) == (n, len(flows), cons)
        got = ws.flows_np()
        assert got.tobytes() == flows.tobytes()
    log("C3: ok")


@pytest.mark.parametrize("big", [False, True])
def test_adversarial_300mb_auto_sparse(big):
    """The auto choice on a large capture of the quirk corpus (every layer's quirks, IPv6, VLANs,
    ARP, fake header chains inside payloads, zero-length records, 20-70 KB jumbo records, a
    truncated tail; mean record > 384 B, > 256 MiB): the sparse walk, bit-exact against the oracle
    flows and IPv6 side rows, and against the resident pass forced."""
    log(f"adversarial 300 MB (big={big}): generating")
    blob = synth.quirk_corpus(360_000, seed=71 + big, big=big, jumbo_every=60, fake_every=7, zero_every=11,
                              tail="truncated_payload")
    assert len(blob) > (256 << 20)
    hdr, recs, cons, flows, v6 = oracle_flows(blob)
    n = len(recs)
    ws = device.Workspace(record_cap=n, flow_cap=n, records=False, offsets=False, status=False,
                          flows=True, flows_v6=True)
    buf = to_dev(blob)
    lib, h = ws.ctx.lib, ws.ctx.handle
    for mode, want_pass in ((0, _abi.PASS_SPARSE), (1, _abi.PASS_RESIDENT)):
        ws.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, mode))
        try:
            ws.flows.zero_()
            ws.launch(buf, start=24, endianness=hdr.endianness)
            sm = ws.check()
            assert lib.npr_ctx_last_pass(h) == want_pass
        finally:
            ws.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, 0))
        assert (sm.n_records, sm.n_flows, sm.consumed) == (n, len(flows), cons), mode
        got = ws.flows_np()
        assert got.tobytes() == flows.tobytes(), mode
        assert v6_rows(got, ws.flows_v6_np()).tobytes() == v6_rows(flows, v6).tobytes(), mode
    log("adversarial 300 MB: ok")


def c4_shards(n_records, world, host=None):
    """Each rank's buffer exactly as the 8-GPU run lays it out: its own file bytes only."""
    layout = parallel.record_range_shards(n_records, world)
    bufs = []
    for g, (base, start, stop, spec) in enumerate(layout):
        r0, r1 = n_records * g // world, n_records * (g + 1) // world
        a = synth.fixed64_range(r0, r1) if host is None else host[base:stop]
        assert a.size == stop - base
        bufs.append(to_dev(np.ascontiguousarray(a)))
    return layout, bufs


def run_c4(n_records, world=8):
    log(f"C4 {n_records}: generating")
    host = synth.fixed64_range(0, n_records)
    file_len = host.size
    layout, bufs = c4_shards(n_records, world, host)
    per = n_records // world + 1
    locals_ = []
    for (base, start, stop, spec), b in zip(layout, bufs):
        ws = device.Workspace(record_cap=1, flow_cap=per, records=False, offsets=False, status=False,
                              flows=True, flows_v6=True)
        locals_.append(parallel.shard_local(ws, b, base, file_len, usec_magic=True, ts_ref=1_600_000_000,
                                            to_host=True))
    bounds = [(start if g == 0 else base, stop) for g, (base, start, stop, spec) in enumerate(layout)]
    bounds[0] = (24, layout[0][2])
    log("C4: device shards")
    results, live, rounds = parallel.parse_sharded_inprocess(locals_, 24, file_len, world, bounds=bounds)
    assert rounds == 1 and all(live)
    for g, r in enumerate(results):  # every speculated start was the exact record boundary
        assert r.entry == bounds[g][0] and r.consumed == bounds[g][1]
    merged, merged6 = parallel.merge_flows(results, live)
    log("C4: oracle")
    hdr, recs, cons, flows, v6 = oracle_flows(host)
    assert len(recs) == n_records and cons == file_len
    _, _, r_tot, f_tot = parallel.prefix_offsets(results, live)
    assert (r_tot, f_tot) == (n_records, len(flows))
    assert merged.tobytes() == flows.tobytes()
    log("C4: ok")


def test_c4_16m_sharded_bit_exact():
    run_c4(16_000_000)


def test_c4_64m_sharded_bit_exact():
    run_c4(64_000_000)


def test_c5_tiled_quirk_capture():
    """SURVEY.md §8 d C5 (10 GB) with the quirk corpus standing in for the absent 4SICS file: one
    tile of complete records repeated to 10 GB; byte-range shards with halos; each tile's slice of
    the merged table equals the single-tile golden with its record offsets moved by the tile's place."""
    tile_blob = synth.quirk_corpus(30_000, seed=77, fake_every=25, jumbo_every=5_000)
    hdr, recs, cons, gold, gold6 = oracle_flows(tile_blob)
    assert cons == len(tile_blob)       # a tile of complete records: the chain runs on into the next
    body = np.frombuffer(tile_blob, dtype=np.uint8)[24:]
    T, K = body.size, 10_000_000_000 // body.size
    log(f"C5: tile {T} B x {K}")
    host = np.empty(24 + T * K, dtype=np.uint8)
    host[:24] = np.frombuffer(tile_blob[:24], dtype=np.uint8)
    host[24:] = np.tile(body, K)
    file_len = host.size
    world, halo = 8, 1 << 20             # jumbo records are <= 70 KB: a 1 MiB halo holds any record
    bounds = parallel.shard_bounds(24, file_len, world)
    locals_ = []
    for g, (lo, hi) in enumerate(bounds):
        base = 0 if g == 0 else lo - lo % 16
        end = min(file_len, hi + halo)
        ws = device.Workspace(record_cap=1, flow_cap=len(gold) * (K // world + 2), records=False, offsets=False,
                              status=False, flows=True, flows_v6=True)
        locals_.append(parallel.shard_local(ws, to_dev(np.ascontiguousarray(host[base:end])), base, file_len,
                                            usec_magic=True, ts_ref=1_600_000_000, to_host=True))
    log("C5: device shards")
    results, live, rounds = parallel.parse_sharded_inprocess(locals_, 24, file_len, world, bounds=bounds)
    merged, merged6 = parallel.merge_flows(results, live)
    n = len(gold)
    assert all(live) and len(merged) == n * K
    # tile k occupies rows [(K-1-k) * n, (K-k) * n) of the reverse-order table
    got = merged.reshape(K, n)[::-1]
    off = got["record_offset"].astype(np.uint64)
    goff = gold["record_offset"].astype(np.uint64)
    offs = sum(off[..., i] << np.uint64(8 * i) for i in range(5))
    goffs = sum(goff[..., i] << np.uint64(8 * i) for i in range(5))
    want = goffs[None, :] + np.arange(K, dtype=np.uint64)[:, None] * np.uint64(T)
    assert np.array_equal(offs, want)
    strip = lambda a: a.view(np.uint8).reshape(a.shape + (32,))[..., :27]  # every field but the offset
    assert np.array_equal(strip(got), np.broadcast_to(strip(gold), got.shape + (27,)))
    g6 = merged6.reshape(K, n)[::-1]
    m = (gold["kind"] & _abi.KIND_IPV6) != 0
    assert m.any() and np.array_equal(g6[:, m], np.broadcast_to(gold6[m], (K, int(m.sum()))))
    log(f"C5: ok ({rounds} exchange rounds)")


@pytest.mark.parametrize("records", [3_100, 50_000, 250_000])
def test_fresh_context_slot_sizing(records):
    """Resident launches of 61, ~1000 and ~4900 tiles on FRESH contexts (the workgroup
    aggregates once overran the slot allocation at these sizes; the host now refuses such a launch)."""
    import net_parser_rs as npr
    blob = synth.fixed64(records)
    hdr, recs, cons, flows, _ = oracle_flows(blob)
    ws = device.Workspace(record_cap=1, flow_cap=len(recs), records=False, flows=True, flows_v6=False,
                          ctx=npr.Context(0))
    ws.launch(to_dev(blob), start=24, endianness=hdr.endianness)
    sm = ws.check()
    assert (sm.n_records, sm.consumed) == (len(recs), cons)
    assert ws.flows_np().tobytes() == flows.tobytes()


def test_summary_in_page_locked_host_memory():
    """Workspace.use_summary(page-locked host tensor): the parse's last link stores the summary
    straight over PCIe (the multi-GPU step reads it after an event, no copy kernel); it equals the
    device summary of the same parse, over a chained (multi-link) capture too."""
    stream = torch.cuda.Stream()  # launches and the event on one explicit stream (NULL = the context's own)
    torch.cuda.set_stream(stream)
    for blob in (synth.fixed64(300_000), synth.variable_mix(200_000)):
        buf = to_dev(blob)
        ws = device.Workspace(record_cap=1, flow_cap=len(blob) // 80 + 1, records=False, flows=True, flows_v6=False)
        ws.launch_chunked(buf, chunk_bytes=4 << 20)
        want = ws.check()
        host = torch.zeros(64, dtype=torch.uint8, pin_memory=True)
        ws.use_summary(host)
        ev = torch.cuda.Event()
        ws.launch_chunked(buf, chunk_bytes=4 << 20)
        ev.record()
        ev.synchronize()
        got = host[:40].numpy().copy().view(_abi.SUMMARY_DTYPE)[0]
        assert (int(got["n_records"]), int(got["n_flows"]), int(got["consumed"])) == \
            (want.n_records, want.n_flows, want.consumed)
        assert int(got["epoch"]) != 0 and int(got["flags"]) == 0
    torch.cuda.set_stream(torch.cuda.default_stream())


def test_device_step_two_in_flight_world1():
    """DeviceShardedParse's launch_step / finish_step with the summaries in host memory and a gloo
    metadata group (the bench's multi-GPU loop), at world size 1 on the GPU: three steps in flight,
    then the rows byte-compared with the oracle."""
    import os
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    torch.cuda.set_stream(torch.cuda.Stream())  # as bench.py: an explicit stream (NULL = the context's own)
    try:
        blob = synth.fixed64(400_000)
        buf = to_dev(blob)
        n = 400_000
        ws = device.Workspace(record_cap=1, flow_cap=n, records=False, flows=True, flows_v6=False)
        step = parallel.DeviceShardedParse(ws, buf, 0, [(24, len(blob))], len(blob), usec_magic=True,
                                           meta_group=dist.group.WORLD)
        for _ in range(3):
            step.launch_step()
            if len(step.pending) > 1:
                step.finish_step()
        while step.pending:
            metas, live, rounds = step.finish_step()
        assert rounds == 1 and metas[0].n_records == n and metas[0].n_flows == n
        fl, _ = step.rows()
        want = oracle_flows(blob)[3]
        assert fl.cpu().numpy().tobytes() == want.tobytes()
    finally:
        torch.cuda.set_stream(torch.cuda.default_stream())
        dist.destroy_process_group()
