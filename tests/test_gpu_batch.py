"""npr_dev_parse_extract_batch (k_parse_batch): several independent captures in ONE resident
launch, each capture's results bit-exact against the oracle (and so equal to its own
npr_dev_parse_extract).  Cases: full-size C2 batches (the bench's batched line), mixed corpora and
endiannesses, the same capture bytes in several items, items a batch does not take (a record table
requested, an empty capture, one larger than a launch holds) between batchable ones, more items than
one launch takes (kMaxBatch = 8), and the capped-wave variant whose deferred tiles re-read through a
ring holding the next capture's staged tiles."""
import numpy as np
import pytest
import torch

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, device, synth

pytestmark = pytest.mark.gpu


def dev(blob):
    return torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()


def expected(blob, start=24, endianness=None):
    if start == 24:
        rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
        e = hdr.endianness
    else:
        recs, c = _oracle.records_parse(blob[start:], endianness)
        recs = recs.copy()
        recs["offset"] += start
        cons, e = start + c, endianness
    flows, v6 = _oracle.convert_records(blob, recs)
    return len(recs), cons, flows, v6, e


def run_batch(blobs, starts=None, endians=None, status=None):
    starts = starts or [24] * len(blobs)
    wants = [expected(b, s, None if endians is None else endians[i]) for i, (b, s) in enumerate(zip(blobs, starts))]
    items = []
    for i, (b, s, w) in enumerate(zip(blobs, starts, wants)):
        cap = max((len(b) - s) // 16 + 1, 1)
        ws = device.Workspace(cap, cap, records=False, status=bool(status and status[i]))
        items.append((ws, dev(b), s, w[4]))
    device.launch_batch(items)
    for i, ((ws, *_), (nr, cons, flows, v6, _)) in enumerate(zip(items, wants)):
        sm = ws.check()
        assert (sm.n_records, sm.consumed, sm.n_flows) == (nr, cons, len(flows)), i
        got = ws.flows_np()
        assert got.tobytes() == flows.tobytes(), f"item {i}"
        m = (flows["kind"] & _abi.KIND_IPV6) != 0
        if m.any():
            assert ws.flows_v6_np()[m].tobytes() == v6[m].tobytes(), f"item {i} v6"
    return items


@pytest.mark.parametrize("k", [2, 4, 8])
def test_full_size_c2_batches(k):
    blobs = [synth.fixed64(1_000_000, seed=100 + i) for i in range(k)]
    run_batch(blobs)


def test_mixed_corpora_and_endianness():
    blobs = [synth.quirk_corpus(6_000, seed=41), synth.variable_mix(20_000),
             synth.quirk_corpus(4_000, seed=42, big=True, fake_every=5, jumbo_every=300),
             synth.fixed64(50_000, seed=43), synth.vxlan_corpus(3_000), synth.flow_mix(9_000),
             synth.quirk_corpus(2_000, seed=44, tail="truncated_payload")]
    run_batch(blobs)


def test_same_bytes_in_several_items():
    b = synth.quirk_corpus(5_000, seed=45)
    run_batch([b, b, b])


def test_items_a_batch_does_not_take():
    blobs = [synth.fixed64(20_000, seed=46), synth.global_header(), synth.quirk_corpus(3_000, seed=47),
             synth.fixed64(10_000, seed=48), synth.variable_mix(5_000)]
    run_batch(blobs, status=[False, False, False, True, False])  # item 3 asks for per-record status


def test_more_items_than_one_launch():
    blobs = [synth.fixed64(30_000 + 1000 * i, seed=50 + i) for i in range(11)]
    run_batch(blobs)


def test_bare_records_items():
    body = synth.quirk_corpus(3_000, seed=49, with_header=False)
    run_batch([body, synth.fixed64(5_000, seed=51)], starts=[0, 24], endians=[npr.Endianness.Little, None])


@pytest.mark.parametrize("waves", [7, 100])
def test_capped_waves_deferred_tiles(waves):
    ctx = npr.context(0)
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, waves))
    try:
        run_batch([synth.fixed64(60_000, seed=52), synth.quirk_corpus(8_000, seed=53, jumbo_every=400),
                   synth.variable_mix(15_000)])
    finally:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 1))
