"""npr_parse_extract (host capture in, host flow table out) with the overlapped chunked copy
(NPR_OPT_STREAM_CHUNK) against the CPU oracle, bit-exact.

The streamed call copies the capture in chunks on a second stream and chains one resident launch
per chunk; its results must be those of the unchunked call for every corpus, including records
longer than a chunk (the call falls back to one launch over the staged capture) and the chain
ends of the reference's tail quirks (Q3).
"""
import numpy as np
import pytest

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, device, synth

pytestmark = pytest.mark.gpu


def check_host(blob, chunk_kib):
    ctx = npr.context(0)
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, chunk_kib))
    try:
        flows, v6, n_flows, consumed, hdr = device.host_parse_extract(blob, ctx=ctx)
    finally:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, 0))
    rc, ohdr, want_recs, want_cons = _oracle.capture_file_parse(blob)
    assert rc == 0 and hdr.endianness == ohdr.endianness
    want_flows, want_v6 = _oracle.convert_records(blob, want_recs)
    assert (n_flows, consumed) == (len(want_flows), want_cons)
    assert flows.tobytes() == want_flows.tobytes()
    m = (want_flows["kind"] & _abi.KIND_IPV6) != 0
    if m.any():
        assert v6[m].tobytes() == want_v6[m].tobytes()
    return n_flows, consumed


CORPORA = {
    "c2": lambda: synth.fixed64(40_000),
    "c3": lambda: synth.variable_mix(6_000),
    "quirk": lambda: synth.quirk_corpus(6_000, seed=61),
    "quirk_big_endian": lambda: synth.quirk_corpus(4_000, seed=62, big=True),
    "adversarial": lambda: synth.quirk_corpus(3_000, seed=63, fake_every=3, zero_every=7, jumbo_every=150),
    "jumbo_longer_than_a_chunk": lambda: synth.quirk_corpus(300, seed=64, jumbo_every=2),
}


@pytest.mark.parametrize("chunk_kib", [0, 64, 100, 1024])
@pytest.mark.parametrize("corpus", sorted(CORPORA))
def test_streamed_host_parse_matches_oracle(corpus, chunk_kib):
    check_host(CORPORA[corpus](), chunk_kib)


@pytest.mark.parametrize("tail", ["truncated_header", "truncated_payload", "huge_incl"])
def test_streamed_chain_ends(tail):
    check_host(synth.quirk_corpus(5_000, seed=65, tail=tail), 64)


def test_streamed_corrupt_incl_mid_file():
    n_flows, consumed = check_host(synth.corrupt_midfile(synth.fixed64(30_000), at_record=12_345), 64)
    assert consumed == 24 + 12_345 * 80


def test_stream_chunk_option_rejects_tiny_chunks():
    ctx = npr.context(0)
    assert ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, 16) == _abi.ERR_ARG
    assert ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, -1) == _abi.ERR_ARG
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, 0))


def test_streamed_large_capture_properties():
    """~320 MB C2 capture through the default 32 MiB chunks: counts, consumed and every flow's
    record offset follow from the fixed 80-B layout (no oracle at this size); convert_records
    emits the flows last record first."""
    n = 4_000_000
    blob = synth.fixed64(n)
    ctx = npr.context(0)
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, 32 << 10))
    try:
        flows, _, n_flows, consumed, _ = device.host_parse_extract(blob, with_v6=False, ctx=ctx)
    finally:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_STREAM_CHUNK, 0))
    assert (n_flows, consumed) == (n, len(blob))
    ro = flows["record_offset"]
    got = ro[:, 0].astype(np.uint64) | (ro[:, 1].astype(np.uint64) << 8) | (ro[:, 2].astype(np.uint64) << 16) | \
        (ro[:, 3].astype(np.uint64) << 24) | (ro[:, 4].astype(np.uint64) << 32)
    assert np.array_equal(got, 24 + 80 * np.arange(n - 1, -1, -1, dtype=np.int64).astype(np.uint64))


def check_pipelined(blob, chunk_bytes, pinned):
    """npr_parse_extract_pipelined: pinned chunked H2D, chained launches, per-link D2H of the rows;
    flows right-aligned in the caller's table."""
    rc, ohdr, want_recs, want_cons = _oracle.capture_file_parse(blob)
    want_flows, want_v6 = _oracle.convert_records(blob, want_recs)
    cap = len(want_recs) + 7  # spare rows: the flows must end at out[cap - 1]
    if pinned:
        src = device.PinnedArray(len(blob))
        src.array[:] = np.frombuffer(blob, dtype=np.uint8)
        fo = device.PinnedArray(cap * 32, _abi.FLOW_DTYPE)
        f6 = device.PinnedArray(cap * 32, _abi.FLOW_V6_DTYPE)
        a, out, out6 = src.array, fo.array, f6.array
    else:
        a = np.frombuffer(blob, dtype=np.uint8).copy()
        out, out6 = np.zeros(cap, _abi.FLOW_DTYPE), np.zeros(cap, _abi.FLOW_V6_DTYPE)
    try:
        flows, v6, n_flows, consumed = device.host_parse_extract_pipelined(a, out, out6, cap, chunk_bytes)
        assert (n_flows, consumed) == (len(want_flows), want_cons)
        assert flows.tobytes() == want_flows.tobytes()
        m = (want_flows["kind"] & _abi.KIND_IPV6) != 0
        assert v6[m].tobytes() == want_v6[m].tobytes()
    finally:
        if pinned:
            for p in (src, fo, f6):
                p.close()


@pytest.mark.parametrize("chunk_bytes", [65536, 100_000, 1 << 20, 0])
@pytest.mark.parametrize("corpus", sorted(CORPORA))
def test_pipelined_host_parse_matches_oracle(corpus, chunk_bytes):
    check_pipelined(CORPORA[corpus](), chunk_bytes, pinned=False)


@pytest.mark.parametrize("corpus", ["c2", "adversarial", "jumbo_longer_than_a_chunk"])
def test_pipelined_host_parse_pinned_buffers(corpus):
    check_pipelined(CORPORA[corpus](), 65536, pinned=True)


def test_tiny_pipelined_calls_then_pageable_copies():
    """Round 6: many pipelined calls on tiny captures (their capture and row arrays
    are small heap objects sharing pages), then host-path parses that copy rows into fresh pageable
    arrays; every result against the oracle."""
    base = synth.quirk_corpus(40, seed=81)
    rc, hdr, recs, cons = _oracle.capture_file_parse(base)
    for k in range(64):
        cut = int(recs["offset"][k % len(recs)]) + 16 + (k % 7)
        check_pipelined(base[:max(cut, 25)], 65536, pinned=False)
    for seed in (82, 83):
        check_host(synth.quirk_corpus(20_000, seed=seed), 0)


def test_pipelined_c2_x4_320mb():
    """The measured configuration: 4M C2 records, 32 MiB chunks, bit-exact."""
    check_pipelined(synth.fixed64(4_000_000), 0, pinned=True)


# ---- the bounded device window (NPR_OPT_DEVICE_WINDOW): captures larger than device memory ----
WINDOW_CORPORA = {  # each larger than 3 windowed chunks of 512 KiB
    "c2": lambda: synth.fixed64(100_000),
    "c3": lambda: synth.variable_mix(6_000),
    "quirk_big_endian": lambda: synth.quirk_corpus(40_000, seed=62, big=True),
    "adversarial": lambda: synth.quirk_corpus(6_000, seed=63, fake_every=3, zero_every=7, jumbo_every=150),
    "truncated_payload": lambda: synth.quirk_corpus(30_000, seed=65, tail="truncated_payload"),
    "huge_incl": lambda: synth.quirk_corpus(30_000, seed=66, tail="huge_incl"),
    "corrupt_incl_mid_file": lambda: synth.corrupt_midfile(synth.fixed64(60_000), at_record=41_234),
}


def check_windowed(blob, chunk_bytes, window, pinned=False):
    """npr_parse_extract_pipelined through a ring of `window` chunk slots (plus the halo mirror)
    and three flow-row slots, against the oracle; flows right-aligned in the caller's table."""
    rc, ohdr, want_recs, want_cons = _oracle.capture_file_parse(blob)
    want_flows, want_v6 = _oracle.convert_records(blob, want_recs)
    cap = len(want_recs) + 5
    if pinned:
        src = device.PinnedArray(len(blob))
        src.array[:] = np.frombuffer(blob, dtype=np.uint8)
        a = src.array
    else:
        a = np.frombuffer(blob, dtype=np.uint8).copy()
    out, out6 = np.zeros(cap, _abi.FLOW_DTYPE), np.zeros(cap, _abi.FLOW_V6_DTYPE)
    try:
        flows, v6, n_flows, consumed = device.host_parse_extract_pipelined(a, out, out6, cap, chunk_bytes,
                                                                           window=window)
    finally:
        if pinned:
            src.close()
    assert (n_flows, consumed) == (len(want_flows), want_cons)
    assert flows.tobytes() == want_flows.tobytes()
    assert not out[:cap - n_flows].view(np.uint8).any()  # nothing written left of the flows
    m = (want_flows["kind"] & _abi.KIND_IPV6) != 0
    assert v6[m].tobytes() == want_v6[m].tobytes()
    return n_flows, consumed


@pytest.mark.parametrize("window", [3, 5])
@pytest.mark.parametrize("corpus", sorted(WINDOW_CORPORA))
def test_windowed_pipelined_matches_oracle(corpus, window):
    check_windowed(WINDOW_CORPORA[corpus](), 1 << 19, window)


def test_windowed_chunks_not_a_multiple_of_the_tile():
    """A requested chunk is rounded up to 4 KiB and to the 512 KiB minimum."""
    check_windowed(synth.variable_mix(3_000), 600_001, 3, pinned=True)


def test_windowed_c2_x4_320mb():
    """4M C2 records (320 MB) through 8 slots of 32 MiB: the default chunk, bit-exact."""
    check_windowed(synth.fixed64(4_000_000), 0, 8, pinned=True)


def _with_long_record(incl, at_byte):
    """C2 records, then one record of `incl` payload bytes starting near `at_byte`, then more."""
    head = np.frombuffer(synth.fixed64((at_byte - 24) // 80), dtype=np.uint8)
    tail = np.frombuffer(synth.fixed64(20_000), dtype=np.uint8)[24:]
    rec = np.zeros(16 + incl, dtype=np.uint8)
    rec[:16] = np.frombuffer(head[24:40].tobytes(), dtype=np.uint8)  # the first record's timestamps
    rec[8:12] = np.frombuffer(np.uint32(incl).tobytes(), dtype=np.uint8)
    rec[12:16] = rec[8:12]
    rec[16:] = np.frombuffer(head[40:104].tobytes() * (incl // 64 + 1), dtype=np.uint8)[:incl]
    return np.concatenate([head, rec, tail]).tobytes()


def test_windowed_record_longer_than_the_halo():
    """A 300 KB record across a chunk end does not fit the window's 260 KiB halo: the windowed call
    says so (NPR_ERR_CAPACITY) instead of stopping the chain there; the staged call parses it."""
    blob = _with_long_record(300_000, (1 << 19) - 8_000)
    with pytest.raises(npr.DeviceError, match="halo"):
        device.host_parse_extract_pipelined(np.frombuffer(blob, dtype=np.uint8).copy(), chunk_bytes=1 << 19, window=3)
    check_pipelined(blob, 1 << 19, pinned=False)


def test_windowed_record_within_the_halo():
    """A 250 KB record across a chunk end is read from the next slot's mirror / halo."""
    check_windowed(_with_long_record(250_000, 3 * (1 << 19) - 8_000), 1 << 19, 3)


def test_device_window_option_values():
    ctx = npr.context(0)
    for bad in (-1, 1, 2):
        assert ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_DEVICE_WINDOW, bad) == _abi.ERR_ARG
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_DEVICE_WINDOW, 3))
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_DEVICE_WINDOW, 0))
