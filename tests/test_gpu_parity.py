"""Parity of the HIP path (through the C-ABI) against the CPU oracle, bit-exact.

Every case runs the fused device kernel (npr_dev_parse_extract) and compares: the record table
(offset, ts, lengths), per-record flow status, the convert_records flow table (bytes, incl. IPv6
side table), n_records / n_flows and `consumed` (the Rust remainder).  Inputs are seeded
synthetic captures (net_parser_rs.synth) sized so the oracle finishes in seconds, plus the
reference's own KAT frames.  Full-size configs (C2 1M, C3 8M, C4 16M/64M, the C5 tiled corpus) are
checked bit-exact or per shard in test_gpu_scale.py.
"""
import ctypes
import json
import os
import struct

import numpy as np
import pytest
import torch

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, device, synth

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KATS = {k["name"]: k for k in json.load(open(os.path.join(REPO, "tests", "golden", "kat.json")))["kats"]}


def to_dev(blob):
    t = torch.empty(max(len(blob), 1), dtype=torch.uint8, device="cuda")
    if blob:
        t[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    return t[: len(blob)] if blob else t[:0]


def expect(blob, start=24, endianness=None):
    """The oracle's (records, consumed, flows, flows_v6, status, endianness) of a capture."""
    if start == 24:
        rc, hdr, want_recs, want_cons = _oracle.capture_file_parse(blob)
        assert rc == 0
        e = hdr.endianness if endianness is None else endianness
    else:
        e = endianness
        want_recs, cons = _oracle.records_parse(blob[start:], e)
        want_recs = want_recs.copy()
        want_recs["offset"] += start
        want_cons = start + cons
    want_flows, want_v6 = _oracle.convert_records(blob, want_recs)
    _, _, want_status = _oracle.extract_flows(blob, want_recs)
    return want_recs, want_cons, want_flows, want_v6, want_status, e


def check_flows(w, want):
    """A flows-only workspace's results against expect()'s."""
    want_recs, want_cons, want_flows, want_v6, _, _ = want
    sm = w.check()
    assert sm.n_records == len(want_recs), (sm.n_records, len(want_recs))
    assert sm.consumed == want_cons, (sm.consumed, want_cons)
    assert sm.n_flows == len(want_flows)
    got_flows = w.flows_np()
    assert got_flows.tobytes() == want_flows.tobytes(), first_diff(got_flows, want_flows)
    v6mask = (want_flows["kind"] & _abi.KIND_IPV6) != 0
    if v6mask.any():
        assert w.flows_v6_np()[v6mask].tobytes() == want_v6[v6mask].tobytes()
    return sm


def check_parity(blob, start=24, endianness=None, ws=None, light=False):
    """Run the device path on `blob` and compare everything with the oracle.

    light requests flows only (no record table / status), so the flow table, counts and
    `consumed` are compared.  light=True runs the resident single pass (k_parse_resident, the
    default for flows-only launches); light=N (an int > 1) the same with at most N waves, so
    each wave owns a long tile range (kept-round overflow -> deferred tiles, many ranges per
    64-wave group, speculation at range starts deep inside the capture); light="decode" the
    two-pass kernels (NPR_OPT_RESIDENT off); light="sparse" the sparse record walk
    forced (NPR_OPT_SPARSE 2), "sparse_sN" with lane ranges of N bytes, "..._cK" with K Ok-flow
    slots per lane (lanes past their slots walk the rest again when rows are written)."""
    if isinstance(light, str) and light.startswith("sparse"):
        return check_sparse(blob, start, endianness, ws, light)
    if light == "decode" or (light is not True and isinstance(light, int) and light > 1):
        ctx = npr.context(0)
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 0 if light == "decode" else light))
        try:
            sm = check_parity(blob, start, endianness, ws, light=True)
        finally:
            ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 1))
        want = _abi.PASS_TWO_PASS if light == "decode" else _abi.PASS_RESIDENT  # the pass that ran
        assert ctx.lib.npr_ctx_last_pass(ctx.handle) == want, (ctx.lib.npr_ctx_last_pass(ctx.handle), want)
        return sm
    want = expect(blob, start, endianness)
    want_recs, want_cons, want_flows, want_v6, want_status, e = want
    buf = to_dev(blob)
    n = len(blob)
    cap = max((n - start) // 16 + 1, 1)
    w = ws or (device.Workspace(cap, cap, records=False, status=False) if light else device.Workspace(cap, cap, status=True))
    w.launch(buf, start=start, endianness=e, nbytes=n)
    if light:
        return check_flows(w, want)
    sm = w.check()
    assert sm.n_records == len(want_recs), (sm.n_records, len(want_recs))
    assert sm.consumed == want_cons, (sm.consumed, want_cons)
    assert sm.n_flows == len(want_flows)
    got_recs = w.records_np()
    assert got_recs.tobytes() == want_recs.tobytes(), first_diff(got_recs, want_recs)
    got_status = w.status_np()
    assert np.array_equal(got_status, want_status), first_diff(got_status, want_status)
    got_flows = w.flows_np()
    assert got_flows.tobytes() == want_flows.tobytes(), first_diff(got_flows, want_flows)
    v6mask = (want_flows["kind"] & _abi.KIND_IPV6) != 0
    if v6mask.any():
        assert w.flows_v6_np()[v6mask].tobytes() == want_v6[v6mask].tobytes()
    return sm


def sparse_opts(light):
    """NPR_OPT_SPARSE / NPR_OPT_SPARSE_CAP values of a "sparse[_sN][_cK]" variant."""
    mode, cap = 2, 0
    for part in light.split("_")[1:]:
        if part[0] == "s":
            mode = int(part[1:])
        elif part[0] == "c":
            cap = int(part[1:])
    return mode, cap


class sparse_forced:
    """Every flows-only launch of the context runs the sparse record walk inside the block."""
    def __init__(self, light="sparse"):
        self.mode, self.cap = sparse_opts(light)
        self.ctx = npr.context(0)

    def __enter__(self):
        lib, h = self.ctx.lib, self.ctx.handle
        self.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, self.mode))
        self.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE_CAP, self.cap))
        return self

    def __exit__(self, *exc):
        lib, h = self.ctx.lib, self.ctx.handle
        self.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE, 0))
        self.ctx.check(lib.npr_ctx_set_option(h, _abi.OPT_SPARSE_CAP, 0))


def check_sparse(blob, start, endianness, ws, light):
    with sparse_forced(light) as f:
        sm = check_parity(blob, start, endianness, ws, light=True)
        assert f.ctx.lib.npr_ctx_last_pass(f.ctx.handle) == _abi.PASS_SPARSE
    return sm


def first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i].tobytes() != b[i].tobytes():
            return f"first diff at {i}: got {a[i]} want {b[i]} (len {len(a)} vs {len(b)})"
    return f"lengths {len(a)} vs {len(b)}"


# ---- the reference's own vectors through the device ------------------------------------------
def test_kat_file_bytes_parse_big_endian():
    blob = bytes.fromhex(KATS["file_bytes_parse"]["input"])
    sm = check_parity(blob)
    assert sm.n_records == 1 and sm.consumed == len(blob) and sm.n_flows == 1
    rem, f = npr.CaptureFile.parse(blob)  # the mirror API (host memory in, host memory out)
    assert len(rem) == 0 and f.global_header.endianness == npr.Endianness.Big and f.records.len() == 1
    rec = f.records.into_inner()[0]
    fl = rec.extract_flow()
    assert (fl.source.port, fl.destination.port) == (50871, 80)
    pairs = npr.flow.convert_records(f.records.into_inner())
    assert len(pairs) == 1 and pairs[0][1] == fl


@pytest.mark.parametrize("name", ["convert_ethernet_tcp", "encapsulated", "not_encapsulated",
                                  "parse_ethernet_payload"])
def test_kat_frames_as_records(name):
    frame = bytes.fromhex(KATS[name]["input"])
    blob = synth.global_header() + struct.pack("<IIII", 1, 2, len(frame), len(frame)) + frame
    check_parity(blob)


# ---- synthetic corpora ---------------------------------------------------------------------
# resident_w16 / _w48: whole 16-wave workgroups (one and three), long ranges with deferred tiles
# sparse: the sparse record walk forced; _s256: 256-B lane ranges (records span many lanes, most
# lanes speculate inside payloads); _s4096_c2: two Ok-flow slots per lane (the overflow walk);
# _s16384: 16-KiB lanes of short records (up to ~200 per lane: slots past 64 in the second mask word,
# and the overflow walk past the default 96 slots)
LIGHT = pytest.mark.parametrize("light", [False, True, 7, 100, 16, 48, "decode",
                                          "sparse", "sparse_s256", "sparse_s4096_c2", "sparse_s16384"],
                                ids=["full", "resident", "resident_w7", "resident_w100", "resident_w16",
                                     "resident_w48", "two_pass",
                                     "sparse", "sparse_s256", "sparse_s4096_c2", "sparse_s16384"])


@LIGHT
def test_c2_small(light):
    check_parity(synth.fixed64(50_000), light=light)


@LIGHT
def test_c3_small(light):
    check_parity(synth.variable_mix(20_000), light=light)


@LIGHT
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_quirk_corpus(seed, light):
    check_parity(synth.quirk_corpus(8_000, seed=seed), light=light)


@LIGHT
def test_quirk_corpus_big_endian(light):
    check_parity(synth.quirk_corpus(6_000, seed=11, big=True), light=light)


@LIGHT
def test_adversarial_speculation(light):
    """Fake record-header chains inside payloads, zero-filled payloads and jumbo (> tile) records
    defeat the per-tile start speculation; the exact prefix must still reproduce the serial chain."""
    check_parity(synth.quirk_corpus(4_000, seed=5, fake_every=3, zero_every=7, jumbo_every=200), light=light)


@LIGHT
def test_jumbo_records_span_many_tiles(light):
    check_parity(synth.quirk_corpus(600, seed=6, jumbo_every=2), light=light)


@pytest.mark.parametrize("span", [1 << 20, 4 << 20])
@pytest.mark.parametrize("corpus", ["jumbo", "c3"])
def test_sparse_lane_ranges_past_the_slot_offset_limit(corpus, span):
    """A sparse slot keeps its record offset as 18 bits relative to the lane start, so lane ranges
    are capped at 256 KiB (npr_internal.hpp kSparseSpanMax): larger forced ranges run at the cap,
    with the same results (jumbo records of 20-70 KB, and C3-like records)."""
    blob = {"jumbo": lambda: synth.quirk_corpus(900, seed=66, jumbo_every=2),
            "c3": lambda: synth.variable_mix(60_000)}[corpus]()
    check_parity(blob, light=f"sparse_s{span}")


@pytest.mark.parametrize("span", [128, 256])
def test_sparse_resolve_queue_overflow(span):
    """Fake record-header chains in every other payload under short lane ranges: most lanes
    mis-speculate, so a resolve pass queues more re-walks than the 2048-task shared queue holds (the
    rest wait for the next pass; stats counter [4] counts such passes).  Results stay the serial
    chain's."""
    blob = synth.quirk_corpus(40_000, seed=67, fake_every=2)
    ctx = npr.context(0)
    lib, h = ctx.lib, ctx.handle
    st = (ctypes.c_uint32 * 8)()
    ctx.check(lib.npr_ctx_set_stats(h, 1))
    ctx.check(lib.npr_ctx_read_stats(h, st, 8, 1))  # (zero the counters)
    try:
        check_parity(blob, light=f"sparse_s{span}")
        ctx.check(lib.npr_ctx_read_stats(h, st, 8, 1))
    finally:
        ctx.check(lib.npr_ctx_set_stats(h, 0))
    assert st[0] > 2048 and st[4] > 0, list(st)


@LIGHT
@pytest.mark.parametrize("tail", ["truncated_header", "truncated_payload", "huge_incl"])
def test_truncated_tails(tail, light):
    sm = check_parity(synth.quirk_corpus(3_000, seed=9, tail=tail), light=light)
    assert sm.consumed < len(synth.quirk_corpus(3_000, seed=9, tail=tail))


@LIGHT
def test_corrupt_incl_mid_file_stops_chain(light):
    blob = synth.corrupt_midfile(synth.fixed64(30_000), at_record=12_345)
    sm = check_parity(blob, light=light)
    assert sm.n_records == 12_345


def lattice_breaker(kind, n=40_000):
    """C2-shaped 80-B records with a few records that keep every later record on the 80-B lattice
    but move its flow index, so that the resident pass's lattice rows (kFlagLattice) of every later
    range land on wrong rows and must be rewritten exactly: `notok` an unknown EtherType (a non-Ok
    flow), `double` one 160-B Ok record (a record less), `pair` a 40-B non-Ok + a 120-B Ok record in
    place of two; `early` breaks the first wave's range, `many` all three kinds at several places."""
    b = bytearray(synth.fixed64(n))
    rec = lambda k: 24 + 80 * k

    def notok(k):
        b[rec(k) + 16 + 12: rec(k) + 16 + 14] = b"\x99\x99"

    def double(k):
        struct.pack_into("<II", b, rec(k) + 8, 144, 144)
        b[rec(k + 1): rec(k + 2)] = bytes(80)  # the trailer of the 144-B frame (IPv4 total_length 50)

    def pair(k):
        frame = bytes(b[rec(k) + 16: rec(k) + 80])
        struct.pack_into("<II", b, rec(k) + 8, 24, 24)  # 24-B frame: IPv4 incomplete
        q = rec(k) + 40
        ts = bytes(b[rec(k): rec(k) + 8])
        b[q: q + 8] = ts
        struct.pack_into("<II", b, q + 8, 104, 104)
        b[q + 16: q + 120] = frame + bytes(40)

    if kind == "notok":
        notok(n // 2)
    elif kind == "double":
        double(n // 3)
    elif kind == "pair":
        pair(n // 2 + 7)
    elif kind == "early":
        notok(3)
    elif kind == "many":
        for k in (5, 1_000, 9_001):
            notok(k)
        double(15_000)
        pair(22_222)
        double(n - 100)
    return bytes(b)


@LIGHT
@pytest.mark.parametrize("kind", ["notok", "double", "pair", "early", "many"])
def test_lattice_breakers(kind, light):
    check_parity(lattice_breaker(kind), light=light)


@LIGHT
def test_empty_and_header_only(light):
    check_parity(synth.global_header(), light=light)                           # 0 records, rem empty
    check_parity(synth.global_header() + bytes(10), light=light)               # 0 records, 10-byte rem
    check_parity(synth.global_header() + struct.pack("<IIII", 0, 0, 0, 0), light=light)  # one zero-length record


@LIGHT
def test_records_without_file_header(light):
    """PcapRecords::parse(input, endianness) over bare records (start = 0)."""
    body = synth.quirk_corpus(3_000, seed=4, with_header=False)
    check_parity(body, start=0, endianness=npr.Endianness.Little, light=light)
    body = synth.quirk_corpus(3_000, seed=4, with_header=False, big=True)
    check_parity(body, start=0, endianness=npr.Endianness.Big, light=light)


def test_workspace_reuse_many_launches():
    blob = synth.quirk_corpus(5_000, seed=21, fake_every=9)
    cap = len(blob) // 16 + 1
    ws = device.Workspace(cap, cap, status=True)
    wl = device.Workspace(cap, cap, records=False, status=False)
    for _ in range(5):
        check_parity(blob, ws=ws)
        check_parity(blob, ws=wl, light=True)  # alternate modes on one context
    check_parity(synth.fixed64(10_000), ws=ws)
    check_parity(synth.fixed64(10_000), ws=wl, light=True)


@pytest.mark.parametrize("records", [True, False], ids=["full", "flows_only"])
def test_flow_capacity_overflow_reports_exact_counts(records):
    blob = synth.fixed64(5_000)
    buf = to_dev(blob)
    ws = device.Workspace(10_000, 100, records=records)
    ws.launch(buf)
    with pytest.raises(npr.DeviceError):
        ws.check()
    assert ws.last.n_flows == 5_000 and ws.last.n_records == 5_000 and ws.last.flags == 2


def test_misaligned_input_rejected():
    blob = synth.fixed64(100)
    buf = to_dev(b"\0" + blob)
    ws = device.Workspace(200, 200)
    with pytest.raises(npr.DeviceError):
        ws.launch(buf[1:])


# ---- the dense extract / convert_records entry points over arbitrary record lists -----------
def test_extract_flows_over_arbitrary_records():
    blob = synth.quirk_corpus(4_000, seed=13)
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    recs = recs.copy()
    rng = np.random.default_rng(0)
    shrink = rng.random(len(recs)) < 0.2   # records whose payload is a prefix of the frame
    recs["actual_length"][shrink] = (recs["actual_length"][shrink] * rng.random(shrink.sum())).astype(np.uint32)
    perm = rng.permutation(len(recs))
    recs = recs[perm]
    want_f, want_v6, want_st = _oracle.extract_flows(blob, recs)
    ctx = npr.context()
    a = np.frombuffer(blob, dtype=np.uint8)
    n = len(recs)
    f = np.zeros(n, _abi.FLOW_DTYPE)
    v6 = np.zeros(n, _abi.FLOW_V6_DTYPE)
    st = np.zeros(n, np.uint8)
    ctx.check(ctx.lib.npr_extract_flows(ctx.handle, a.ctypes.data, a.size, recs.ctypes.data, n, f.ctypes.data,
                                        v6.ctypes.data, st.ctypes.data))
    assert np.array_equal(st, want_st)
    assert f.tobytes() == want_f.tobytes()
    assert v6.tobytes() == want_v6.tobytes()
    # convert_records over the same (permuted) list: reverse LIST order
    wf, wv6 = _oracle.convert_records(blob, recs)
    out = np.zeros(n, _abi.FLOW_DTYPE)
    out6 = np.zeros(n, _abi.FLOW_V6_DTYPE)
    import ctypes
    k = ctypes.c_size_t(0)
    ctx.check(ctx.lib.npr_convert_records(ctx.handle, a.ctypes.data, a.size, recs.ctypes.data, n, out.ctypes.data,
                                          out6.ctypes.data, n, ctypes.byref(k)))
    assert k.value == len(wf)
    assert out[: k.value].tobytes() == wf.tobytes()
    m = (wf["kind"] & _abi.KIND_IPV6) != 0
    assert out6[: k.value][m].tobytes() == wv6[m].tobytes()


def test_mirror_api_matches_oracle():
    blob = synth.quirk_corpus(2_000, seed=17)
    rem, f = npr.parse(blob)
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert len(rem) == len(blob) - cons and f.records.len() == len(recs)
    pairs = npr.flow.convert_records(f.records.into_inner())
    wf, _ = _oracle.convert_records(blob, recs)
    assert [p[0].offset for p in pairs] == [int.from_bytes(bytes(x), "little") for x in wf["record_offset"]]
    rem2, recs2 = npr.PcapRecords.parse(blob[24:], npr.Endianness.Little)
    assert recs2.len() == len(recs)
    recs_list = npr.CaptureParser.parse_file(blob)
    assert len(recs_list) == len(recs)


def test_mirror_convert_records_keeps_repeated_records():
    """convert_records(Vec<PcapRecord>) pops every element (src/flow/mod.rs:101-123): a record listed
    twice yields two (record, flow) pairs, each paired with its own list element."""
    blob = synth.quirk_corpus(500, seed=18)
    _, f = npr.parse(blob)
    rs = f.records.into_inner()
    lst = rs[:40] + rs[10:20] + rs[5:6] + rs[300:]
    pairs = npr.flow.convert_records(lst)
    want = []
    for r in reversed(lst):
        try:
            want.append((r, r.extract_flow()))
        except npr.flow.FlowError:
            pass
    assert len(pairs) == len(want)
    for (r, fl), (wr, wfl) in zip(pairs, want):
        assert r is wr and fl == wfl


# ---- chained launches (npr_dev_parse_extract_chunked): the capture parsed chunk after chunk --------
def check_chunked(blob, chunk, start=24, endianness=None):
    if start == 24:
        rc, hdr, want_recs, want_cons = _oracle.capture_file_parse(blob)
        e = hdr.endianness if endianness is None else endianness
    else:
        e = endianness
        want_recs, cons = _oracle.records_parse(blob[start:], e)
        want_recs = want_recs.copy()
        want_recs["offset"] += start
        want_cons = start + cons
    want_flows, want_v6 = _oracle.convert_records(blob, want_recs)
    cap = max((len(blob) - start) // 16 + 1, 1)
    w = device.Workspace(cap, cap, records=False, status=False)
    w.launch_chunked(to_dev(blob), start=start, endianness=e, chunk_bytes=chunk, nbytes=len(blob))
    sm = w.check()
    assert (sm.n_records, sm.n_flows, sm.consumed) == (len(want_recs), len(want_flows), want_cons)
    assert sm.entry == start  # the chain's first record, carried through every link
    got = w.flows_np()
    assert got.tobytes() == want_flows.tobytes(), first_diff(got, want_flows)
    v6mask = (want_flows["kind"] & _abi.KIND_IPV6) != 0
    if v6mask.any():
        assert w.flows_v6_np()[v6mask].tobytes() == want_v6[v6mask].tobytes()
    return sm


CHUNKS = pytest.mark.parametrize("chunk", [1000, 4096, 40_000, 333_333])


@CHUNKS
@pytest.mark.parametrize("corpus", ["c2", "c3", "quirk", "adversarial", "jumbo", "v6", "lattice"])
def test_chunked_matches_serial(corpus, chunk):
    blob = {"c2": lambda: synth.fixed64(30_000),
            "lattice": lambda: lattice_breaker("many"),
            "c3": lambda: synth.variable_mix(8_000),
            "quirk": lambda: synth.quirk_corpus(6_000, seed=52),
            "adversarial": lambda: synth.quirk_corpus(3_000, seed=53, fake_every=3, zero_every=7, jumbo_every=150),
            "jumbo": lambda: synth.quirk_corpus(400, seed=54, jumbo_every=2),
            "v6": lambda: synth.quirk_corpus(5_000, seed=55, big=True)}[corpus]()
    check_chunked(blob, chunk)


@CHUNKS
def test_chunked_chain_end_and_tails(chunk):
    sm = check_chunked(synth.corrupt_midfile(synth.fixed64(20_000), at_record=7_777), chunk)
    assert sm.n_records == 7_777
    for tail in ("truncated_header", "truncated_payload", "huge_incl"):
        check_chunked(synth.quirk_corpus(2_000, seed=56, tail=tail), chunk)


@pytest.mark.parametrize("chunk", [333_333, 0])
@pytest.mark.parametrize("corpus", ["c3", "quirk", "adversarial", "jumbo", "v6"])
def test_chunked_packing_pass(corpus, chunk):
    """At most 7 waves: links longer than one kept round per tile run the PACK instantiation
    (sparse tiles share kept rounds, unused lanes read the first used lane's record, the IPv4-only
    decode variant when it applies, deferred tiles once the kept rounds are full); chunk 0 = the
    density-sized links (the capture is >= 8 x one dense link)."""
    blob = {"c3": lambda: synth.variable_mix(8_000),
            "quirk": lambda: synth.quirk_corpus(40_000, seed=58),
            "adversarial": lambda: synth.quirk_corpus(20_000, seed=59, fake_every=3, zero_every=7, jumbo_every=150),
            "jumbo": lambda: synth.quirk_corpus(1_500, seed=60, jumbo_every=2),
            "v6": lambda: synth.quirk_corpus(30_000, seed=61, big=True)}[corpus]()
    ctx = npr.context(0)
    ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 7))
    try:
        check_chunked(blob, chunk)
    finally:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 1))


@pytest.mark.parametrize("chunk", [40_000, 333_333])
@pytest.mark.parametrize("corpus", ["c3", "quirk", "adversarial", "jumbo", "v6", "tails"])
def test_chunked_sparse_links(corpus, chunk):
    """Sparse walks as chained links (each continues the previous link's device summary): lane 0
    starts at the previous link's exit, the scan checks it against that summary."""
    blob = {"c3": lambda: synth.variable_mix(8_000),
            "quirk": lambda: synth.quirk_corpus(6_000, seed=62),
            "adversarial": lambda: synth.quirk_corpus(3_000, seed=63, fake_every=3, zero_every=7, jumbo_every=150),
            "jumbo": lambda: synth.quirk_corpus(400, seed=64, jumbo_every=2),
            "v6": lambda: synth.quirk_corpus(5_000, seed=65, big=True),
            "tails": lambda: synth.corrupt_midfile(synth.fixed64(20_000), at_record=7_777)}[corpus]()
    with sparse_forced("sparse_s512_c4") as f:
        check_chunked(blob, chunk)
        assert f.ctx.lib.npr_ctx_last_pass(f.ctx.handle) == _abi.PASS_SPARSE


def test_sparse_range_speculative_start():
    """A byte range whose start is not a record boundary (the shard form): the sparse walk
    speculates the first record like the resident pass and reports it in summary->entry."""
    blob = synth.variable_mix(6_000)
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    offs = recs["offset"].astype(np.int64)
    lo = int(offs[1234]) - 5                       # inside record 1233
    stop = int(offs[4000]) + 3
    want = recs[(offs >= int(offs[1234])) & (offs < stop)]
    wf, _ = _oracle.convert_records(blob, want)
    buf = to_dev(blob)
    cap = len(blob) // 16 + 1
    with sparse_forced("sparse_s1024"):
        w = device.Workspace(cap, cap, records=False, status=False)
        w.launch_range(buf, lo, stop, endianness=hdr.endianness, speculative=True)
        sm = w.check()
    assert sm.entry == int(offs[1234]) and sm.n_records == len(want) and sm.n_flows == len(wf)
    assert w.flows_np().tobytes() == wf.tobytes()


def test_chunked_bare_records_and_tiny_inputs():
    body = synth.quirk_corpus(3_000, seed=57, with_header=False)
    check_chunked(body, 5_000, start=0, endianness=npr.Endianness.Little)
    check_chunked(synth.global_header(), 4096)
    check_chunked(synth.global_header() + bytes(10), 7)


def test_capture_past_2GiB():
    """C3-shaped capture of ~2.2 GB: record offsets past 2^31 (a sign-extension regression), both
    kernel families, against the oracle."""
    n = 2_800_000
    blob = synth.variable_mix(n)
    rc, hdr, want_recs, want_cons = _oracle.capture_file_parse(blob)
    want_flows, _ = _oracle.convert_records(blob, want_recs)
    buf = to_dev(blob)
    del blob
    ctx = npr.context(0)
    try:
        for resident in (1, 0):
            ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, resident))
            w = device.Workspace(n + 1, n + 1, records=False, status=False)
            w.launch(buf, start=24, endianness=hdr.endianness)
            sm = w.check()
            assert (sm.n_records, sm.n_flows, sm.consumed) == (len(want_recs), len(want_flows), want_cons)
            got = w.flows_np()
            assert got.tobytes() == want_flows.tobytes(), first_diff(got, want_flows)
            del w
    finally:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_RESIDENT, 1))
