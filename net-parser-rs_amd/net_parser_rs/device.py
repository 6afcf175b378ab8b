"""Device-resident entry points over torch tensors (torch = HBM allocation + streams only).

    ws = Workspace(record_cap, flow_cap, device=0)      # outputs allocated once, reused
    ws.launch(buf, start=24, endianness=Endianness.Little)   # async, on the current torch stream
    summary = ws.check()                                 # sync + totals / capacity errors

`buf` is a contiguous uint8 CUDA tensor (16-byte aligned, as torch allocations are).  Outputs
follow npr_dev_outputs (include/npr.h): dense record table / status in file order, flows in
convert_records order RIGHT-aligned in [flow_cap - n_flows, flow_cap).
"""
import ctypes

import numpy as np
import torch

from . import _abi, context

_side_streams = {}


class _On:
    """The stream a call launches on.  The caller's stream when it has a handle; torch's default
    stream is the null stream, which the C-ABI cannot name (NULL selects the context's own
    non-blocking stream, unordered with the null stream), so then a side stream fenced to it on
    both sides: it waits for the default stream's earlier work, and the default stream waits for
    the call (exit)."""

    def __init__(self, dev, stream):
        dev = torch.device(dev)
        self.user = stream if stream is not None else torch.cuda.current_stream(dev)
        self.s = self.user
        if self.user.cuda_stream == 0:
            key = dev.index or 0
            if key not in _side_streams:
                _side_streams[key] = torch.cuda.Stream(device=dev)
            self.s = _side_streams[key]
            self.s.wait_stream(self.user)

    def __enter__(self):
        return self.s

    def __exit__(self, *exc):
        if self.s is not self.user:
            self.user.wait_stream(self.s)
        return False



class Workspace:
    def __init__(self, record_cap, flow_cap, device=0, records=True, offsets=False, status=False,
                 flows=True, flows_v6=True, ctx=None):
        self.device = torch.device("cuda", device)
        self.ctx = ctx if ctx is not None else context(device)  # a Context is per thread (npr_ctx)
        self.record_cap, self.flow_cap = int(record_cap), int(flow_cap)
        mk = lambda nbytes: torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.device)
        self.records = mk(self.record_cap * 24) if records else None
        self.offsets = mk(self.record_cap * 8) if offsets else None
        self.status = mk(self.record_cap) if status else None
        self.flows = mk(self.flow_cap * 32) if flows else None
        self.flows_v6 = mk(self.flow_cap * 32) if flows_v6 else None
        self.summary = torch.zeros(64, dtype=torch.uint8, device=self.device)
        p = lambda t: t.data_ptr() if t is not None else None
        self.outs = _abi.DevOutputsC(p(self.offsets), p(self.records), p(self.status), self.record_cap,
                                     p(self.flows), p(self.flows_v6), self.flow_cap, p(self.summary))
        self.last = None

    def launch(self, buf, start=24, endianness=_abi.LITTLE, nbytes=None, stream=None):
        assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
        n = buf.numel() if nbytes is None else int(nbytes)
        with _On(self.device, stream) as s:
            st = self.ctx.lib.npr_dev_parse_extract(self.ctx.handle, buf.data_ptr(), n, start, endianness,
                                                    ctypes.byref(self.outs), ctypes.c_void_p(s.cuda_stream))
        self.ctx.check(st)
        self._stream = s

    def forget_density(self, buf=None):
        """New bytes replace the capture at `buf`'s address (None: any capture): the next parse probes
        its record density afresh (npr_ctx_forget_density; the pass choice never changes a result)."""
        self.ctx.check(self.ctx.lib.npr_ctx_forget_density(self.ctx.handle, buf.data_ptr() if buf is not None else None))

    def launch_range(self, buf, start, stop, endianness=_abi.LITTLE, speculative=False, ref_record=24,
                     nbytes=None, stream=None):
        """Records that START in [start, stop) of `buf` (payloads may run past stop): one shard of a
        capture (npr_dev_parse_extract_range).  speculative=True: `start` is a byte position, the
        first record at/after it is speculated and reported as summary.entry."""
        assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
        n = buf.numel() if nbytes is None else int(nbytes)
        ref = _abi.NO_ENTRY if ref_record is None else int(ref_record)
        with _On(self.device, stream) as s:
            st = self.ctx.lib.npr_dev_parse_extract_range(self.ctx.handle, buf.data_ptr(), n, int(start), int(stop),
                                                          endianness, 1 if speculative else 0, ref,
                                                          ctypes.byref(self.outs), ctypes.c_void_p(s.cuda_stream))
        self.ctx.check(st)
        self._stream = s

    def launch_chunked(self, buf, start=24, endianness=_abi.LITTLE, chunk_bytes=0, nbytes=None, stream=None):
        """The capture in chunks of ~chunk_bytes chained on the device (npr_dev_parse_extract_chunked):
        one launch per chunk, no host synchronisation, same outputs as launch()."""
        assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
        n = buf.numel() if nbytes is None else int(nbytes)
        with _On(self.device, stream) as s:
            st = self.ctx.lib.npr_dev_parse_extract_chunked(self.ctx.handle, buf.data_ptr(), n, int(start), endianness,
                                                            ctypes.byref(self.outs), int(chunk_bytes),
                                                            ctypes.c_void_p(s.cuda_stream))
        self.ctx.check(st)
        self._stream = s

    def launch_shard(self, buf, base, start, stop, endianness=_abi.LITTLE, speculative=False, usec_magic=True,
                     ts_ref=None, chunk_bytes=0, nbytes=None, stream=None):
        """One shard held by this device (npr_dev_parse_extract_shard): `buf` holds FILE bytes
        [base, base + nbytes); records that START in [start, stop) are produced, with file offsets.
        usec_magic / ts_ref: the capture's speculation context (its buffer lacks the header)."""
        assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
        n = buf.numel() if nbytes is None else int(nbytes)
        sh = _abi.ShardC(int(base), int(start), int(stop), 1 if speculative else 0, 1 if usec_magic else 0,
                         _abi.NO_ENTRY if ts_ref is None else int(ts_ref), int(chunk_bytes))
        with _On(self.device, stream) as s:
            st = self.ctx.lib.npr_dev_parse_extract_shard(self.ctx.handle, buf.data_ptr(), n, endianness, ctypes.byref(sh),
                                                          ctypes.byref(self.outs), ctypes.c_void_p(s.cuda_stream))
        self.ctx.check(st)
        self._stream = s

    def use_summary(self, summary):
        """Launches from now on write their npr_summary into `summary`: 64 uint8 on this device, or in
        page-locked host memory (the last launch of a parse then stores it straight over PCIe, so the
        host reads it after an event, with no copy kernel behind the parse)."""
        assert (summary.is_cuda or summary.is_pinned()) and summary.dtype == torch.uint8 and summary.numel() >= 64
        self.summary = summary
        self.outs.summary = summary.data_ptr()

    def flow_rows(self, n_flows=None):
        """The right-aligned flow rows as device tensors (views, no copy): (flows, flows_v6)."""
        k = min(self.last.n_flows if n_flows is None else int(n_flows), self.flow_cap)
        lo, hi = (self.flow_cap - k) * 32, self.flow_cap * 32
        return (self.flows[lo:hi] if self.flows is not None else None,
                self.flows_v6[lo:hi] if self.flows_v6 is not None else None)

    def check(self):
        sm = _abi.SummaryC()
        st = self.ctx.lib.npr_dev_check(self.ctx.handle, ctypes.byref(self.outs),
                                        ctypes.c_void_p(self._stream.cuda_stream), ctypes.byref(sm))
        self.last = sm
        if st not in (_abi.OK,):
            self.ctx.check(st)
        return sm

    # ---- host views of the results (for tests) ----
    def records_np(self):
        n = min(self.last.n_records, self.record_cap)
        return self.records[: n * 24].cpu().numpy().view(_abi.RECORD_DTYPE)

    def offsets_np(self):
        n = min(self.last.n_records, self.record_cap)
        return self.offsets[: n * 8].cpu().numpy().view("<u8")

    def status_np(self):
        n = min(self.last.n_records, self.record_cap)
        return self.status[:n].cpu().numpy()

    def flows_np(self):
        k = min(self.last.n_flows, self.flow_cap)
        return self.flows[(self.flow_cap - k) * 32: self.flow_cap * 32].cpu().numpy().view(_abi.FLOW_DTYPE)

    def flows_v6_np(self):
        k = min(self.last.n_flows, self.flow_cap)
        return self.flows_v6[(self.flow_cap - k) * 32: self.flow_cap * 32].cpu().numpy().view(_abi.FLOW_V6_DTYPE)


def launch_batch(items, ctx=None, stream=None):
    """npr_dev_parse_extract_batch: several captures in one call (one ordinary launch each, in
    order).  items: (ws, buf, start, endianness) per capture, each parsed as ws.launch(buf, start,
    endianness) would (its outputs in that Workspace; check each with ws.check()).  Asynchronous on `stream` (default: the current
    stream of the first buffer's device)."""
    items = list(items)
    if not items:
        return
    ctx = ctx if ctx is not None else items[0][0].ctx
    arr = (_abi.BatchItemC * len(items))()
    for i, (ws, buf, start, e) in enumerate(items):
        assert buf.is_cuda and buf.dtype == torch.uint8 and buf.is_contiguous()
        arr[i] = _abi.BatchItemC(buf.data_ptr(), buf.numel(), int(start), int(e), 0, ws.outs)
    with _On(items[0][1].device, stream) as s:
        ctx.check(ctx.lib.npr_dev_parse_extract_batch(ctx.handle, ctypes.cast(arr, ctypes.c_void_p), len(items),
                                                       ctypes.c_void_p(s.cuda_stream)))
    for ws, *_ in items:
        ws._stream = s


class Result:
    def __init__(self, ws, sm):
        self.ws = ws
        self.n_records, self.n_flows, self.consumed, self.flags = sm.n_records, sm.n_flows, sm.consumed, sm.flags

    def records_np(self):
        return self.ws.records_np()

    def status_np(self):
        return self.ws.status_np()

    def flows_np(self):
        return self.ws.flows_np()

    def flows_v6_np(self):
        return self.ws.flows_v6_np()


def parse_extract(buf, start=24, endianness=_abi.LITTLE, record_cap=None, flow_cap=None, status=True):
    """One-shot device parse + extract + convert over a CUDA uint8 tensor (sync)."""
    n = buf.numel()
    cap = max((n - start) // 16 + 1, 1) if n > start else 1
    ws = Workspace(record_cap if record_cap is not None else cap, flow_cap if flow_cap is not None else cap,
                   device=buf.device.index or 0, status=status)
    ws.launch(buf, start=start, endianness=endianness)
    sm = ws.check()
    return Result(ws, sm)


def _dev_records(recs):
    """A device npr_record table: a CUDA uint8 tensor of n * 24 bytes (or int64 of n * 3)."""
    assert recs.is_cuda and recs.is_contiguous()
    nbytes = recs.numel() * recs.element_size()
    assert nbytes % 24 == 0 and recs.data_ptr() % 8 == 0
    return nbytes // 24


def dev_extract_flows(buf, recs, flows=None, flows_v6=None, status=None, ctx=None, stream=None):
    """FlowExtraction::extract_flow per record over device-resident records (npr_dev_extract_flows),
    async on `stream`: dense (flows, flows_v6, status) tensors, row i for record i (zero rows where
    the status is not Ok)."""
    n = _dev_records(recs)
    dev = buf.device
    mk = lambda nbytes: torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    flows = mk(n * 32) if flows is None else flows
    flows_v6 = mk(n * 32) if flows_v6 is None else flows_v6
    status = mk(n) if status is None else status
    ctx = ctx if ctx is not None else context(dev.index or 0)
    with _On(dev, stream) as s:
        ctx.check(ctx.lib.npr_dev_extract_flows(ctx.handle, buf.data_ptr(), buf.numel(), recs.data_ptr(), n,
                                                flows.data_ptr(), flows_v6.data_ptr(), status.data_ptr(),
                                                ctypes.c_void_p(s.cuda_stream)))
    return flows, flows_v6, status


def dev_flow_aggregate(flows, flows_v6=None, n=None, weights=None, cap=None, ctx=None, stream=None):
    """Row f4: the distinct-flow table of a device flow table (npr_dev_flow_aggregate), async on
    `stream`.  flows / flows_v6: CUDA uint8 tensors of 32-B rows (e.g. Workspace.flow_rows());
    weights: CUDA int64 counts per row (merging aggregated tables) or None.  Returns (out, out_v6,
    counts, n_out) with n_out a one-element CUDA int64 tensor: rows [0, min(n_out, cap)) valid."""
    assert flows.is_cuda and flows.dtype == torch.uint8 and flows.is_contiguous()
    n = flows.numel() // 32 if n is None else int(n)
    dev = flows.device
    cap = n if cap is None else int(cap)
    mk = lambda nbytes: torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    out, out_v6 = mk(cap * 32), mk(cap * 32)
    counts = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
    n_out = torch.zeros(1, dtype=torch.int64, device=dev)
    if weights is not None:
        assert weights.is_cuda and weights.dtype == torch.int64 and weights.numel() >= n
    ctx = ctx if ctx is not None else context(dev.index or 0)
    p = lambda t: t.data_ptr() if t is not None else None
    with _On(dev, stream) as s:
        ctx.check(ctx.lib.npr_dev_flow_aggregate(ctx.handle, flows.data_ptr(), p(flows_v6), p(weights), n,
                                                 out.data_ptr(), out_v6.data_ptr(), counts.data_ptr(), cap,
                                                 n_out.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
    return out, out_v6, counts, n_out


def dev_vxlan_flows(buf, recs, dst_port=0, big=True, ctx=None, stream=None):
    """Row f3: the VXLAN inner flow of every device-resident record (npr_dev_vxlan_flows), async on
    `stream`: dense (flows, flows_v6, status, vni) tensors, row i for record i."""
    n = _dev_records(recs)
    dev = buf.device
    mk = lambda nbytes: torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    flows, flows_v6, status, vni = mk(n * 32), mk(n * 32), mk(n), mk(n * 4)
    ctx = ctx if ctx is not None else context(dev.index or 0)
    with _On(dev, stream) as s:
        ctx.check(ctx.lib.npr_dev_vxlan_flows(ctx.handle, buf.data_ptr(), buf.numel(), recs.data_ptr(), n,
                                              int(dst_port), _abi.BIG if big else _abi.LITTLE, flows.data_ptr(),
                                              flows_v6.data_ptr(), status.data_ptr(), vni.data_ptr(),
                                              ctypes.c_void_p(s.cuda_stream)))
    return flows, flows_v6, status, vni


def dev_convert_records(buf, recs, cap=None, out=None, out_v6=None, with_v6=True, ctx=None, stream=None):
    """flow::convert_records over device-resident records (npr_dev_convert_records), async on
    `stream`: (out, out_v6 or None, n_out) where rows [0, min(n_out, cap)) are the Ok flows in
    reverse record order and n_out is a one-element CUDA int64 tensor (-1 = UINT64_MAX: timed out)."""
    n = _dev_records(recs)
    dev = buf.device
    cap = n if cap is None else int(cap)
    mk = lambda nbytes: torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)
    out = mk(cap * 32) if out is None else out
    out_v6 = (mk(cap * 32) if out_v6 is None else out_v6) if with_v6 else None
    n_out = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx = ctx if ctx is not None else context(dev.index or 0)
    with _On(dev, stream) as s:
        ctx.check(ctx.lib.npr_dev_convert_records(ctx.handle, buf.data_ptr(), buf.numel(), recs.data_ptr(), n,
                                                  out.data_ptr(), out_v6.data_ptr() if out_v6 is not None else None,
                                                  cap, n_out.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
    return out, out_v6, n_out


def host_parse_extract(data, flow_cap=None, with_v6=True, ctx=None):
    """npr_parse_extract without a record table: a host capture (bytes / uint8 array) in, the
    convert_records flow table out on the host.  Captures of more than two NPR_OPT_STREAM_CHUNK
    chunks are copied in chunks overlapped with the chained parse.  Returns (flows, flows_v6 or
    None, n_flows, consumed, header)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    ctx = ctx or context(0)
    cap = max((a.size - 24) // 16 + 1, 1) if flow_cap is None else flow_cap
    flows = np.zeros(cap, dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(cap, dtype=_abi.FLOW_V6_DTYPE) if with_v6 else None
    hdr = _abi.GlobalHeaderC()
    n_flows, consumed = ctypes.c_size_t(0), ctypes.c_size_t(0)
    st = ctx.lib.npr_parse_extract(ctx.handle, a.ctypes.data if a.size else None, a.size, ctypes.byref(hdr), None, 0,
                                   None, flows.ctypes.data, v6.ctypes.data if v6 is not None else None, cap,
                                   ctypes.byref(n_flows), ctypes.byref(consumed))
    ctx.check(st)
    k = min(n_flows.value, cap)
    return flows[:k], (v6[:k] if v6 is not None else None), n_flows.value, consumed.value, hdr


class PinnedArray:
    """A page-locked host buffer from npr_host_alloc, viewed as a numpy array (freed on close)."""

    def __init__(self, nbytes, dtype=np.uint8, ctx=None):
        self.ctx = ctx or context(0)
        p = ctypes.c_void_p()
        self.ctx.check(self.ctx.lib.npr_host_alloc(self.ctx.handle, max(int(nbytes), 1), ctypes.byref(p)))
        self.ptr = p
        raw = (ctypes.c_uint8 * max(int(nbytes), 1)).from_address(p.value)
        self.array = np.frombuffer(raw, dtype=np.uint8)[: int(nbytes)].view(dtype)

    def close(self):
        if self.ptr is not None:
            self.array = None
            self.ctx.lib.npr_host_free(self.ctx.handle, self.ptr)
            self.ptr = None


def host_parse_extract_pipelined(data, out=None, out_v6=None, flow_cap=None, chunk_bytes=0, ctx=None, window=None):
    """npr_parse_extract_pipelined: a host capture (numpy uint8, ideally a PinnedArray's) in, the
    convert_records flow table out on the host, transfers overlapped.  Returns (flows, flows_v6 or
    None, n_flows, consumed): views of the right-aligned rows of `out` / `out_v6`.  `window` (chunks,
    >= 3) streams the capture through a bounded device window for this call (NPR_OPT_DEVICE_WINDOW)."""
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    ctx = ctx or context(0)
    if window is not None:
        ctx.check(ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_DEVICE_WINDOW, int(window)))
        try:
            return host_parse_extract_pipelined(a, out, out_v6, flow_cap, chunk_bytes, ctx)
        finally:
            ctx.lib.npr_ctx_set_option(ctx.handle, _abi.OPT_DEVICE_WINDOW, 0)
    cap = max((a.size - 24) // 16 + 1, 1) if flow_cap is None else flow_cap
    if out is None:
        out = np.zeros(cap, dtype=_abi.FLOW_DTYPE)
    hdr = _abi.GlobalHeaderC()
    n_flows, consumed = ctypes.c_size_t(0), ctypes.c_size_t(0)
    st = ctx.lib.npr_parse_extract_pipelined(ctx.handle, a.ctypes.data if a.size else None, a.size, ctypes.byref(hdr),
                                             out.ctypes.data, out_v6.ctypes.data if out_v6 is not None else None, cap,
                                             ctypes.byref(n_flows), ctypes.byref(consumed), int(chunk_bytes))
    ctx.check(st)
    k = min(n_flows.value, cap)
    return out[cap - k:cap], (out_v6[cap - k:cap] if out_v6 is not None else None), n_flows.value, consumed.value
