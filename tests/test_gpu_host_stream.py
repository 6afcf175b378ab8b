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


def test_pipelined_c2_x4_320mb():
    """The measured configuration: 4M C2 records, 32 MiB chunks, bit-exact."""
    check_pipelined(synth.fixed64(4_000_000), 0, pinned=True)
