"""The flows-only parse chooses its pass by the record density of the capture's first 256 KiB and
remembers it per (device address, range, byte order) (npr_capi.hip probe_density).  New bytes at the
same address must not keep the old choice: the host entry points forget their staging buffer's
density when they stage new bytes, npr_ctx_forget_density forgets it on request, and npr_dev_check
corrects a remembered density that the parse's own summary contradicts.  Results are
exact whichever pass runs; these tests pin which one runs."""
import numpy as np
import pytest
import torch

import net_parser_rs as npr
from net_parser_rs import _abi, device, synth

pytestmark = pytest.mark.gpu

MIN_SPARSE = 256 << 20  # npr_capi.hip kSparseMinBytes


@pytest.fixture(scope="module")
def captures():
    """A long-record capture (C3-like, mean ~800 B) past the sparse walk's 256 MiB floor, and a
    C2-like capture of 80-B records cut to the same length (its tail record is incomplete)."""
    n = MIN_SPARSE // 780 + 2000
    long_ = synth.variable_mix(n)
    assert len(long_) > MIN_SPARSE
    k = (len(long_) - 24) // 80 + 1
    short = synth.fixed64(k)[: len(long_)]
    return long_, n, short, (len(long_) - 24) // 80


def last_pass(ws):
    return ws.ctx.lib.npr_ctx_last_pass(ws.ctx.handle)


def test_device_buffer_rewritten(captures):
    long_, n_long, short, n_short = captures
    L = len(long_)
    buf = torch.empty(L, dtype=torch.uint8, device="cuda")
    ws = device.Workspace(1, (L - 24) // 16 + 1, records=False, status=False, flows_v6=False)
    buf.copy_(torch.frombuffer(bytearray(long_), dtype=torch.uint8))
    ws.launch(buf)
    sm = ws.check()
    assert last_pass(ws) == _abi.PASS_SPARSE and sm.n_records == n_long
    # the same address now holds 80-B records
    buf.copy_(torch.frombuffer(bytearray(short), dtype=torch.uint8))
    ws.launch(buf)  # chooses by the remembered density (exact results either way)
    sm = ws.check()  # ... and this check corrects it from the summary
    assert sm.n_records == n_short and sm.consumed == 24 + 80 * n_short
    ws.launch(buf)
    sm = ws.check()
    assert last_pass(ws) == _abi.PASS_RESIDENT and sm.n_records == n_short
    # back to long records, forgotten explicitly: the very next parse probes again
    buf.copy_(torch.frombuffer(bytearray(long_), dtype=torch.uint8))
    ws.forget_density(buf)
    ws.launch(buf)
    sm = ws.check()
    assert last_pass(ws) == _abi.PASS_SPARSE and sm.n_records == n_long


def test_host_entry_point_restages(captures):
    long_, n_long, short, n_short = captures
    ctx = npr.context(0)
    a = np.frombuffer(long_, dtype=np.uint8)
    _, _, nf, cons, _ = device.host_parse_extract(a, with_v6=False, ctx=ctx)
    assert ctx.lib.npr_ctx_last_pass(ctx.handle) == _abi.PASS_SPARSE and cons == len(long_)
    b = np.frombuffer(short, dtype=np.uint8)
    _, _, nf, cons, _ = device.host_parse_extract(b, with_v6=False, ctx=ctx)
    assert ctx.lib.npr_ctx_last_pass(ctx.handle) == _abi.PASS_RESIDENT
    assert nf == n_short and cons == 24 + 80 * n_short


def test_one_workspace_alternating_buffers(captures):
    """One Workspace (one summary buffer) alternating between a long-record capture and an 80-B one
    at two addresses: checking one capture's parse must not rewrite the other's remembered density
    (every entry that had held the summary pointer took the last parse's density)."""
    long_, n_long, short, n_short = captures
    L = len(long_)
    a = torch.frombuffer(bytearray(long_), dtype=torch.uint8).cuda()
    b = torch.frombuffer(bytearray(short), dtype=torch.uint8).cuda()
    ws = device.Workspace(1, (L - 24) // 16 + 1, records=False, status=False, flows_v6=False)
    for _ in range(3):
        ws.launch(a)
        sm = ws.check()
        assert last_pass(ws) == _abi.PASS_SPARSE and sm.n_records == n_long
        ws.launch(b)
        sm = ws.check()
        assert last_pass(ws) == _abi.PASS_RESIDENT and sm.n_records == n_short
    # a caller's own range launch on the same summary corrects no entry either
    ws.launch_range(b, 24, L)
    sm = ws.check()
    assert sm.n_records == n_short
    ws.launch(a)
    sm = ws.check()
    assert last_pass(ws) == _abi.PASS_SPARSE and sm.n_records == n_long
