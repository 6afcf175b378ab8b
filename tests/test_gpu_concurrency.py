"""Concurrent use of the C-ABI: the reference's functions are pure and reentrant, and its errors are
Send + Sync (src/errors.rs:13-14; SURVEY.md §8 b "Threading"), so callers may parse from several
threads at once.  Each thread has its own context (npr_ctx is per thread) and stream; libnpr orders
the look-back launches of all contexts on a device (npr_capi.hip ordered_launch), which is what keeps
two resident launches from interleaving on the CUs (round 2: two contexts on two streams deadlocked
until the 1-s bounded waits aborted them with NPR_ERR_TIMEOUT).

Every output is compared byte for byte with the oracle."""
import threading

import numpy as np
import pytest
import torch

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, device, synth

pytestmark = pytest.mark.gpu


def expected(blob):
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    flows, _ = _oracle.convert_records(blob, recs)
    return len(recs), cons, flows.tobytes(), recs


def test_two_contexts_two_streams_interleaved():
    """scripts/microbench/inflight.py at depth 2: one host thread, C2 launches dealt round-robin to
    two contexts on two streams, never synchronised in between."""
    n = 1_000_000
    blob = synth.fixed64(n)
    nr, cons, want, _ = expected(blob)
    dev = torch.device("cuda", 0)
    host = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    bufs = [host.to(dev) for _ in range(2)]
    wss = [device.Workspace(n, n, records=False, status=False, ctx=npr.Context(0)) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for i in range(40):
        wss[i % 2].launch(bufs[i % 2], start=24, stream=streams[i % 2])
    torch.cuda.synchronize()
    for ws in wss:
        sm = ws.check()  # raises DeviceError on NPR_ERR_TIMEOUT
        assert (sm.n_records, sm.n_flows, sm.consumed) == (nr, nr, cons)
        assert ws.flows_np().tobytes() == want


def _worker(blob, want, reps, errors, barrier, convert):
    try:
        nr, cons, flows, recs = want
        ctx = npr.Context(0)  # this thread's own context
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        s = torch.cuda.Stream(dev)
        buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
        cap = len(blob) // 16 + 1
        ws = device.Workspace(cap, cap, records=False, status=False, ctx=ctx)
        drecs = torch.from_numpy(recs.view(np.uint8).reshape(-1).copy()).to(dev)
        torch.cuda.synchronize()
        barrier.wait()
        for r in range(reps):
            for _ in range(5):  # several launches in flight on this stream, the other thread's between them
                ws.launch(buf, start=24, stream=s)
            if convert:
                with torch.cuda.stream(s):
                    out, _, n_out = device.dev_convert_records(buf, drecs, ctx=ctx, stream=s, with_v6=False)
            sm = ws.check()
            assert (sm.n_records, sm.n_flows, sm.consumed) == (nr, len(flows) // 32, cons), r
            assert ws.flows_np().tobytes() == flows, r
            if convert:
                s.synchronize()
                k = int(n_out.item())
                assert k == len(flows) // 32 and out[: k * 32].cpu().numpy().tobytes() == flows, r
    except Exception as e:  # noqa: BLE001 — reported by the main thread
        errors.append(repr(e))


def test_two_threads_own_contexts():
    """Two host threads, each with its own context and stream, parse (and convert) different
    captures at the same time: no timeout, every result bit-exact."""
    blobs = [synth.fixed64(400_000, seed=5), synth.quirk_corpus(60_000, seed=6, jumbo_every=500, fake_every=50)]
    wants = [expected(b) for b in blobs]
    errors, barrier = [], threading.Barrier(2)
    ts = [threading.Thread(target=_worker, args=(blobs[i], wants[i], 8, errors, barrier, i == 0)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(240)
        assert not t.is_alive(), "a thread did not finish"
    assert not errors, errors


def test_stream_release_before_destroy():
    """A caller-created HIP stream used for a launch, handed over with npr_stream_release, then
    destroyed; another context's next launch (whose order wait would have recorded the pending event
    on the freed stream) runs and is exact."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n = 200_000
    blob = synth.fixed64(n, seed=9)
    nr, cons, want, _ = expected(blob)
    dev = torch.device("cuda", 0)
    buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    a, b = (device.Workspace(n, n, records=False, status=False, ctx=npr.Context(0)) for _ in range(2))
    torch.cuda.synchronize()
    raw = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
    a.launch(buf, start=24, stream=torch.cuda.ExternalStream(raw.value, device=dev))
    sm = a.check()  # (on the launch's stream: before it is destroyed)
    assert (sm.n_records, sm.n_flows, sm.consumed) == (nr, nr, cons) and a.flows_np().tobytes() == want
    a.ctx.release_stream(raw.value)
    assert hip.hipStreamDestroy(raw) == 0
    s = torch.cuda.Stream(dev)
    b.launch(buf, start=24, stream=s)
    sm = b.check()
    assert (sm.n_records, sm.n_flows, sm.consumed) == (nr, nr, cons) and b.flows_np().tobytes() == want
