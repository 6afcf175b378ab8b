"""The byte-range device API (npr_dev_parse_extract_range) and the sharded reconcile of
net_parser_rs.parallel over it, on one GPU: every shard is launched in turn, with the device's
own speculation for ranges that start mid-stream; the merged result must equal the serial
reference (oracle) bit for bit."""
import numpy as np
import pytest
import torch

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, device, parallel, synth

pytestmark = pytest.mark.gpu


def to_dev(blob):
    t = torch.empty(len(blob), dtype=torch.uint8, device="cuda")
    t.copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    return t


def reference(blob):
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert rc == 0
    flows, v6 = _oracle.convert_records(blob, recs)
    return hdr, recs, cons, flows, v6


def test_range_stops_at_stop():
    blob = synth.quirk_corpus(4_000, seed=41)
    hdr, recs, cons, flows, _ = reference(blob)
    stop = len(blob) // 2
    keep = recs[recs["offset"] < stop]
    buf = to_dev(blob)
    ws = device.Workspace(len(recs) + 1, len(recs) + 1, status=True)
    ws.launch_range(buf, 24, stop, endianness=hdr.endianness)
    sm = ws.check()
    assert sm.n_records == len(keep) and sm.entry == 24
    assert ws.records_np().tobytes() == keep.tobytes()
    want_f, _ = _oracle.convert_records(blob, keep)
    assert ws.flows_np().tobytes() == want_f.tobytes()
    assert sm.consumed == (recs["offset"][len(keep)] if len(keep) < len(recs) else cons)


def test_speculative_range_finds_the_next_record():
    blob = synth.fixed64(20_000)
    hdr, recs, cons, flows, _ = reference(blob)
    lo = 24 + 80 * 5000 + 37          # the middle of record 5000
    ws = device.Workspace(len(recs) + 1, len(recs) + 1)
    ws.launch_range(to_dev(blob), lo, len(blob), endianness=hdr.endianness, speculative=True)
    sm = ws.check()
    assert sm.entry == 24 + 80 * 5001
    assert sm.n_records == len(recs) - 5001 and sm.consumed == len(blob)


@pytest.mark.parametrize("world", [2, 3, 7])
@pytest.mark.parametrize("corpus", ["c2", "quirk", "adversarial", "jumbo"])
def test_sharded_device_matches_serial(world, corpus):
    blob = {"c2": lambda: synth.fixed64(30_000),
            "quirk": lambda: synth.quirk_corpus(6_000, seed=42),
            "adversarial": lambda: synth.quirk_corpus(3_000, seed=43, fake_every=3, zero_every=7, jumbo_every=150),
            "jumbo": lambda: synth.quirk_corpus(400, seed=44, jumbo_every=2)}[corpus]()
    hdr, recs, cons, flows, v6 = reference(blob)
    buf = to_dev(blob)
    ws = device.Workspace(len(recs) + 1, len(recs) + 1, records=False)
    local = parallel.device_local(ws, buf, len(blob), endianness=hdr.endianness)
    results, live, rounds = parallel.parse_sharded_inprocess(local, 24, len(blob), world)
    _, _, r_tot, f_tot = parallel.prefix_offsets(results, live)
    assert r_tot == len(recs) and f_tot == len(flows)
    merged, merged6 = parallel.merge_flows(results, live)
    assert merged.tobytes() == flows.tobytes()
    m = (flows["kind"] & _abi.KIND_IPV6) != 0
    assert merged6[m].tobytes() == v6[m].tobytes()
    last = [r for r in range(world) if live[r]][-1]
    assert results[last].consumed == cons or results[last].consumed >= len(blob)


def test_sharded_device_chain_end():
    blob = synth.corrupt_midfile(synth.fixed64(20_000), at_record=9_000)
    hdr, recs, cons, flows, _ = reference(blob)
    ws = device.Workspace(20_001, 20_001, records=False)
    local = parallel.device_local(ws, to_dev(blob), len(blob), endianness=hdr.endianness)
    results, live, rounds = parallel.parse_sharded_inprocess(local, 24, len(blob), 4)
    _, _, r_tot, f_tot = parallel.prefix_offsets(results, live)
    assert r_tot == 9_000 and f_tot == len(flows)
    assert parallel.merge_flows(results, live)[0].tobytes() == flows.tobytes()


@pytest.mark.parametrize("lanes", [2, 256])
@pytest.mark.parametrize("corpus", ["quirk", "c3", "adversarial"])
def test_shard_buffers_sparse_forced(corpus, lanes):
    """npr_dev_parse_extract_shard (each shard its own buffer of file bytes [base, end), base > 0,
    a speculated first record, the speculation context from the host) through the sparse record
    walk forced on (NPR_OPT_SPARSE 2: lanes sized from the density; 256: 256-B lanes, most of them
    speculating inside payloads), merged and compared with the serial oracle."""
    blob = {"quirk": lambda: synth.quirk_corpus(5_000, seed=45),
            "c3": lambda: synth.variable_mix(6_000),
            "adversarial": lambda: synth.quirk_corpus(3_000, seed=46, fake_every=3, zero_every=7,
                                                      jumbo_every=150)}[corpus]()
    hdr, recs, cons, flows, v6 = reference(blob)
    host = np.frombuffer(blob, dtype=np.uint8)
    world, halo = 3, 1 << 17
    bounds = parallel.shard_bounds(24, len(blob), world)
    locals_ = []
    for g, (lo, hi) in enumerate(bounds):
        base = 0 if g == 0 else lo - lo % 16
        end = min(len(blob), hi + halo)
        ws = device.Workspace(record_cap=1, flow_cap=len(recs) + 1, records=False, offsets=False, status=False,
                              flows=True, flows_v6=True)
        locals_.append(parallel.shard_local(ws, to_dev(np.ascontiguousarray(host[base:end]).tobytes()), base,
                                            len(blob), endianness=hdr.endianness, usec_magic=True,
                                            ts_ref=1_600_000_000, to_host=True))
    ctx = npr.context(0)  # every Workspace of this thread shares it
    mode = 2 if lanes == 2 else lanes
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_SPARSE, mode))
    try:
        results, live, rounds = parallel.parse_sharded_inprocess(locals_, 24, len(blob), world, bounds=bounds)
        assert ctx.lib.npr_ctx_last_pass(ctx.handle) == _abi.PASS_SPARSE
    finally:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_SPARSE, 0))
    _, _, r_tot, f_tot = parallel.prefix_offsets(results, live)
    assert r_tot == len(recs) and f_tot == len(flows)
    merged, merged6 = parallel.merge_flows(results, live)
    assert merged.tobytes() == flows.tobytes()
    m = (flows["kind"] & _abi.KIND_IPV6) != 0
    assert merged6[m].tobytes() == v6[m].tobytes()
