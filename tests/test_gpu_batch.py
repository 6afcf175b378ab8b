"""npr_dev_parse_extract_batch: several independent captures in one call (each item the ordinary
npr_dev_parse_extract launch, in order on the stream), each item's results bit-exact against the
oracle.  Cases: mixed corpora and endiannesses, the same capture bytes in several items, an item
asking for per-record status and an empty capture between flows-only ones, more than 8 items, and
bare records (start 0).  (Round 3's one-launch k_parse_batch is gone: DESIGN.md §3.2.)"""
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
