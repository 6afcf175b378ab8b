"""Per-record entry points over device-resident records, bit-exact against the oracle.

npr_dev_extract_flows (FlowExtraction::extract_flow per record, src/flow/mod.rs:20-48) and
npr_dev_convert_records (flow::convert_records, src/flow/mod.rs:101-123: Ok flows in REVERSE
record order) take an arbitrary npr_record list, so the cases go past what a parse produces:
permuted lists, payloads shortened to a prefix of the frame, records that do not lie inside the
buffer, payloads ending at the buffer's last byte (the staged 96-B window falls back to global
bytes), output capacity below the Ok count, and list lengths around the 256-record block.
"""
import numpy as np
import pytest
import torch

from net_parser_rs import _abi, device, synth

import _oracle

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()


def records_of(blob, shrink=0.0, permute=False, seed=0):
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert rc == 0
    recs = recs.copy()
    rng = np.random.default_rng(seed)
    if shrink:
        m = rng.random(len(recs)) < shrink
        recs["actual_length"][m] = (recs["actual_length"][m] * rng.random(m.sum())).astype(np.uint32)
    if permute:
        recs = recs[rng.permutation(len(recs))]
    return recs


def check_dense(blob, recs):
    want_f, want_v6, want_st = _oracle.extract_flows(blob, recs)
    n = len(recs)
    f, f6, st = device.dev_extract_flows(dev(np.frombuffer(blob, np.uint8)), dev(recs))
    torch.cuda.synchronize()
    assert np.array_equal(st[:n].cpu().numpy(), want_st)
    assert f[: n * 32].cpu().numpy().tobytes() == want_f.tobytes()
    m = (want_f["kind"] & _abi.KIND_IPV6) != 0  # side rows of IPv6 flows only (npr.h)
    got6 = f6[: n * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
    assert got6[m].tobytes() == want_v6[m].tobytes()


def check_convert(blob, recs, cap=None, with_v6=True):
    want_f, want_v6 = _oracle.convert_records(blob, recs)
    k = len(want_f)
    n = len(recs)
    cap = n if cap is None else cap
    out, out6, n_out = device.dev_convert_records(dev(np.frombuffer(blob, np.uint8)), dev(recs), cap=cap,
                                                  with_v6=with_v6)
    torch.cuda.synchronize()
    assert int(n_out.item()) == k
    w = min(k, cap)
    assert out[: w * 32].cpu().numpy().tobytes() == want_f[:w].tobytes()
    if with_v6:  # side rows of IPv6 flows (IPv4 rows' side rows are not written)
        m = (want_f["kind"][:w] & _abi.KIND_IPV6) != 0
        got6 = out6[: w * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)
        assert got6[m].tobytes() == want_v6[:w][m].tobytes()
    return k


CORPORA = {
    "quirk": lambda: synth.quirk_corpus(8_000, seed=3),
    "quirk_be": lambda: synth.quirk_corpus(5_000, seed=11, big=True),
    "c2": lambda: synth.fixed64(50_000),
    "c3": lambda: synth.variable_mix(20_000),
    "adversarial": lambda: synth.quirk_corpus(4_000, seed=5, fake_every=3, zero_every=7, jumbo_every=200),
}


@pytest.mark.parametrize("name", sorted(CORPORA))
@pytest.mark.parametrize("variant", ["parsed", "shrunk_permuted"])
def test_dev_per_record_matches_oracle(name, variant):
    blob = CORPORA[name]()
    recs = records_of(blob, shrink=0.2, permute=True, seed=7) if variant != "parsed" else records_of(blob)
    check_dense(blob, recs)
    assert check_convert(blob, recs) > 0 or name == "adversarial"


# block shapes on 256 CUs (launch_convert_records): one record per lane up to 256 x 1024, then 2, 3
# and 4 per lane with ragged last rounds, then several generations of 4096-record blocks
@pytest.mark.parametrize("n", [0, 1, 255, 1023, 1024, 1025, 64 * 256 + 3, 256 * 1024, 256 * 1024 + 1, 600_000,
                               256 * 4096, 256 * 4096 + 1])
def test_dev_convert_block_edges(n):
    blob = synth.fixed64(max(n, 1))
    recs = records_of(blob)[:n]
    if n:
        check_dense(blob, recs)
    assert check_convert(blob, recs) == n  # every fixed64 frame is an Ok flow


def test_dev_convert_capacity_below_count():
    blob = synth.variable_mix(30_000)
    recs = records_of(blob)
    k = check_convert(blob, recs, cap=1000)
    assert k > 1000
    check_convert(blob, recs, cap=0)
    check_convert(blob, recs, with_v6=False)


def test_records_outside_the_buffer_and_at_its_end():
    """Records past the buffer (status 0xff, never a flow), and the buffer cut right after a
    frame so the last payloads end at its final byte (window past the end -> global bytes)."""
    blob = synth.quirk_corpus(3_000, seed=21)
    recs = records_of(blob)
    last = recs[-1]
    cut = blob[: int(last["offset"]) + 16 + int(last["actual_length"])]
    check_dense(cut, recs)
    check_convert(cut, recs)
    bad = recs[:300].copy()
    bad["offset"][::3] += len(blob)                       # header past the end
    bad["actual_length"][1::3] = len(blob)                # payload past the end
    check_dense(blob, bad)
    check_convert(blob, bad)


def test_dev_convert_c2_full_size():
    """The C2 bench capture (1M 64-B frames): every record, one launch, bit-exact."""
    blob = synth.fixed64(1_000_000)
    recs = records_of(blob)
    assert check_convert(blob, recs) == 1_000_000
    check_dense(blob, recs)


def test_dev_convert_far_groups():
    """4.3M frames: 1,052 blocks of 4096 records, so the upper blocks take the groups more than
    three below their own through the group sums, and a ragged last block."""
    n = 64 * 64 * 1024 + 111_111
    blob = synth.fixed64(n)
    recs = records_of(blob)
    assert check_convert(blob, recs) == n


def test_dev_convert_beyond_64_group_sums():
    """17.8M frames (1.4 GB): 4,356 blocks, so the top blocks fold more than 64 group sums (two
    windows of sums) below their near groups."""
    n = 68 * 64 * 4096 + 12_345
    blob = synth.fixed64(n)
    recs = records_of(blob)
    assert check_convert(blob, recs) == n


def dev_details(blob, recs):
    import ctypes
    import net_parser_rs as npr
    ctx = npr.context(0)
    n = len(recs)
    buf, r = dev(np.frombuffer(blob, np.uint8)), dev(recs)
    st = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
    det = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    ctx.check(ctx.lib.npr_dev_flow_details(ctx.handle, buf.data_ptr(), buf.numel(), r.data_ptr(), n, st.data_ptr(),
                                           det.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
    torch.cuda.synchronize()
    return st[:n].cpu().numpy(), det[:n].cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("name", sorted(CORPORA) + ["vxlan", "flow_mix"])
def test_flow_error_details_match_oracle(name):
    """The payload each record's error variant carries (include/npr.h npr_flow_details: Needed sizes,
    remainders, failure offsets, versions, EtherTypes, protocol ids), device vs oracle, on parsed and
    shrunk+permuted record lists (shrinking produces every Incomplete step)."""
    blob = {"vxlan": lambda: synth.vxlan_corpus(3_000), "flow_mix": lambda: synth.flow_mix(5_000)}.get(
        name, CORPORA.get(name))()
    for recs in (records_of(blob), records_of(blob, shrink=0.5, permute=True, seed=9)):
        want_st, want_det = _oracle.flow_details(blob, recs)
        st, det = dev_details(blob, recs)
        assert np.array_equal(st, want_st)
        assert np.array_equal(det, want_det)


def test_flow_error_details_host_call_and_mirror():
    """npr_flow_details (host memory) and the mirror's FlowError.size / .detail."""
    import net_parser_rs as npr
    from net_parser_rs import flow
    blob = synth.quirk_corpus(2_000, seed=13)
    rem, f = npr.CaptureFile.parse(blob)
    recs = f.records.into_inner()
    want_st, want_det = _oracle.flow_details(blob, records_of(blob))
    st, det = flow._details(recs[0]._buf, recs)
    assert np.array_equal(st, want_st) and np.array_equal(det, want_det)
    seen = 0
    for i in np.nonzero(want_st != 0)[0][:40]:
        with pytest.raises(flow.FlowError) as e:
            recs[i].extract_flow()
        assert e.value.code == want_st[i] and e.value.detail == int(want_det[i])
        seen += e.value.size is not None
    assert seen > 0


@pytest.mark.parametrize("n_rec", [1, 7, 1_500, 12_000], ids=["one", "seven", "small_arena", "staged"])
def test_host_extract_and_details_both_paths(n_rec):
    """npr_extract_flows / npr_flow_details with host buffers: calls whose input + records fit the
    256-KiB page-locked arena run one launch over it (the kernel reads and writes host memory);
    larger ones stage through device buffers.  Both against the oracle, IPv6 side rows included."""
    import net_parser_rs as npr
    blob = synth.quirk_corpus(n_rec, seed=21)
    recs = records_of(blob, shrink=0.2, permute=True, seed=3)
    assert (len(blob) + 24 * len(recs) <= (256 << 10)) == (n_rec < 5_000)  # which path each case takes
    want_f, want_v6, want_st = _oracle.extract_flows(blob, recs)
    ctx = npr.context()
    a = np.frombuffer(blob, dtype=np.uint8)
    n = len(recs)
    f = np.zeros(n, _abi.FLOW_DTYPE)
    v6 = np.zeros(n, _abi.FLOW_V6_DTYPE)
    st = np.zeros(n, np.uint8)
    for _ in range(2):  # the second call reuses the arena
        ctx.check(ctx.lib.npr_extract_flows(ctx.handle, a.ctypes.data, a.size, recs.ctypes.data, n, f.ctypes.data,
                                            v6.ctypes.data, st.ctypes.data))
        assert np.array_equal(st, want_st)
        assert f.tobytes() == want_f.tobytes()
        assert v6.tobytes() == want_v6.tobytes()
    want_ds, want_det = _oracle.flow_details(blob, recs)
    ds = np.zeros(n, np.uint8)
    det = np.zeros(n, np.uint64)
    ctx.check(ctx.lib.npr_flow_details(ctx.handle, a.ctypes.data, a.size, recs.ctypes.data, n, ds.ctypes.data,
                                       det.ctypes.data))
    assert np.array_equal(ds, want_ds) and np.array_equal(det, want_det)
    # convert_records over the same list (reverse LIST order), both with room for every row and capped
    import ctypes
    wf, wv6 = _oracle.convert_records(blob, recs)
    for cap in (n, max(len(wf) // 2, 1)):
        out = np.zeros(n, _abi.FLOW_DTYPE)
        out6 = np.zeros(n, _abi.FLOW_V6_DTYPE)
        k = ctypes.c_size_t(0)
        rc = ctx.lib.npr_convert_records(ctx.handle, a.ctypes.data, a.size, recs.ctypes.data, n, out.ctypes.data,
                                         out6.ctypes.data, cap, ctypes.byref(k))
        assert k.value == len(wf)
        assert rc == (0 if cap >= len(wf) else _abi.ERR_CAPACITY)
        m = min(cap, len(wf))
        assert out[:m].tobytes() == wf[:m].tobytes()
        is6 = (wf[:m]["kind"] & _abi.KIND_IPV6) != 0
        assert out6[:m][is6].tobytes() == wv6[:m][is6].tobytes()
