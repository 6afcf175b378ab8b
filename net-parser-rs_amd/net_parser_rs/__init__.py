"""net_parser_rs — host-side mirror of protectwise/net-parser-rs 0.3.0's API over libnpr.so.

Same names, argument meaning and error behaviour as the Rust crate, so code (and tests) written
against the reference read the same here:

    rem, f = net_parser_rs.parse(data)                    # src/lib.rs:44-46
    rem, f = CaptureFile.parse(data)                      # src/file.rs:14-35
    rem, recs = PcapRecords.parse(data, Endianness.Big)   # src/record.rs:21-54
    rem, rec = PcapRecord.parse(data, Endianness.Big)     # src/record.rs:102-121
    flow = rec.extract_flow()                             # src/flow/mod.rs:23-41
    pairs = flow.convert_records(recs.into_inner())       # src/flow/mod.rs:101-123
    CaptureParser.parse_file / parse_records / parse_record   (README.md:17-28 facade)

Every multi-record parse runs on the MI355X (HIP kernels in libnpr.so); there is no CPU
fallback — importing works without a GPU, the first device call raises if none is present.
Returned values borrow the input like the Rust API: a record's payload is a memoryview slice.
"""
import ctypes
import threading

import numpy as np

from . import _abi
from ._abi import LITTLE, BIG

__all__ = ["Endianness", "Error", "GlobalHeader", "PcapRecord", "PcapRecords", "CaptureFile", "parse",
           "CaptureParser", "flow", "Context"]


class Endianness:
    """nom::Endianness"""
    Little = LITTLE
    Big = BIG


# ---- crate::errors::Error (src/errors.rs:3-11) ----------------------------------------------
class Error(Exception):
    pass


class Incomplete(Error):
    def __init__(self, size=None):
        super().__init__(f"Incomplete: {size!r}")
        self.size = size


class Failure(Error):
    pass


class Custom(Error):
    pass


class DeviceError(Error):
    """Boundary errors the Rust API cannot produce (negative npr_status)."""


Error.Incomplete, Error.Failure, Error.Custom = Incomplete, Failure, Custom


class Context:
    """One libnpr context (device + stream + workspaces).  One per thread, like npr_ctx."""

    def __init__(self, device=0):
        self.lib = _abi.load_library()
        h = ctypes.c_void_p()
        st = self.lib.npr_ctx_create(device, ctypes.byref(h))
        if st != 0:
            raise DeviceError(f"npr_ctx_create({device}) failed with status {st}: no usable HIP device")
        self.handle = h

    def check(self, st):
        if st == _abi.OK:
            return
        if st == _abi.INCOMPLETE:
            raise Incomplete()
        if st == _abi.FAILURE:
            raise Failure("Failure")
        if st == _abi.CUSTOM:
            raise Custom("Custom")
        msg = self.lib.npr_ctx_last_error(self.handle).decode()
        raise DeviceError(f"status {st}: {msg}")

    def release_stream(self, stream):
        """npr_stream_release: call before destroying a HIP stream (a raw handle, or an object with
        `cuda_stream`) that was passed to any device call; torch's pooled streams are never destroyed."""
        h = getattr(stream, "cuda_stream", stream)
        self.check(self.lib.npr_stream_release(self.handle, ctypes.c_void_p(h)))

    def close(self):
        if getattr(self, "handle", None):
            self.lib.npr_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def context(device=0):
    """The calling thread's Context for HIP device `device` (created on first use)."""
    d = getattr(_tls, "ctx", None)
    if d is None:
        d = _tls.ctx = {}
    c = d.get(device)
    if c is None:
        c = d[device] = Context(device)
    return c


def _as_array(data):
    if isinstance(data, np.ndarray):
        return np.ascontiguousarray(data, dtype=np.uint8).reshape(-1)
    return np.frombuffer(memoryview(data).cast("B"), dtype=np.uint8) if len(data) else np.zeros(0, np.uint8)


# ---- GlobalHeader (src/global_header.rs:13-70) -----------------------------------------------
class GlobalHeader:
    __slots__ = ("endianness", "version_major", "version_minor", "zone", "sig_figs", "snap_length", "network")

    def __init__(self, endianness=LITTLE, version_major=2, version_minor=4, zone=0, sig_figs=0,
                 snap_length=1500, network=1):  # Default (:25-37)
        self.endianness, self.version_major, self.version_minor = endianness, version_major, version_minor
        self.zone, self.sig_figs, self.snap_length, self.network = zone, sig_figs, snap_length, network

    @staticmethod
    def _from_c(h):
        return GlobalHeader(h.endianness, h.version_major, h.version_minor, h.zone, h.sig_figs,
                            h.snap_length, h.network)

    @staticmethod
    def parse(data):
        a = _as_array(data)
        h = _abi.GlobalHeaderC()
        used = ctypes.c_size_t(0)
        st = _abi.load_library().npr_global_header_parse(a.ctypes.data if a.size else None, a.size,
                                                        ctypes.byref(h), ctypes.byref(used))
        if st == _abi.INCOMPLETE:
            raise Incomplete(None)
        if st != 0:
            raise DeviceError(f"status {st}")
        return memoryview(a)[used.value:], GlobalHeader._from_c(h)


# ---- PcapRecord (src/record.rs:59-139) -------------------------------------------------------
class PcapRecord:
    __slots__ = ("_buf", "offset", "ts_sec", "ts_usec", "actual_length", "original_length")

    def __init__(self, buf, offset, ts_sec, ts_usec, actual_length, original_length):
        self._buf, self.offset = buf, int(offset)
        self.ts_sec, self.ts_usec = int(ts_sec), int(ts_usec)
        self.actual_length, self.original_length = int(actual_length), int(original_length)

    @property
    def payload(self):
        o = self.offset + 16
        return memoryview(self._buf)[o:o + self.actual_length]

    @property
    def timestamp_ns(self):
        """convert_packet_time (src/record.rs:82-86): UNIX_EPOCH + secs + micros."""
        return self.ts_sec * 1_000_000_000 + self.ts_usec * 1_000

    @staticmethod
    def convert_packet_time(ts_seconds, ts_microseconds):
        return ts_seconds * 1_000_000_000 + ts_microseconds * 1_000

    def __str__(self):  # Display (src/record.rs:123-139): "{secs}{millis}" unpadded
        ns = self.timestamp_ns
        return (f"Timestamp={ns // 1_000_000_000}{(ns % 1_000_000_000) // 1_000_000}   "
                f"Length={self.actual_length}   Original Length={self.original_length}")

    def __repr__(self):
        return f"PcapRecord(offset={self.offset}, {self})"

    @staticmethod
    def parse(data, endianness):
        a = _as_array(data)
        r = _abi.RecordC()
        used = ctypes.c_size_t(0)
        st = _abi.load_library().npr_record_parse(a.ctypes.data if a.size else None, a.size, endianness,
                                                 ctypes.byref(r), ctypes.byref(used))
        if st == _abi.INCOMPLETE:
            raise Incomplete(None)
        if st != 0:
            raise DeviceError(f"status {st}")
        return memoryview(a)[used.value:], PcapRecord(a, 0, r.ts_sec, r.ts_usec, r.actual_length,
                                                       r.original_length)

    def extract_flow(self):
        """FlowExtraction::extract_flow (src/flow/mod.rs:23-41); raises flow.FlowError on Err."""
        flows, v6, status = flow._extract(self._buf, [self])
        st = int(status[0])
        if st != 0:
            _, det = flow._details(self._buf, [self])
            raise flow.FlowError(st, det[0])
        return flow.Flow._from_row(flows[0], v6[0])


class PcapRecords:
    """Vec<PcapRecord> wrapper (src/record.rs:7-16), backed by a numpy npr_record table."""

    def __init__(self, buf, table):
        self._buf, self.table = buf, table

    def __len__(self):
        return len(self.table)

    def len(self):
        return len(self.table)

    def __getitem__(self, i):
        r = self.table[i]
        return PcapRecord(self._buf, r["offset"], r["ts_sec"], r["ts_usec"], r["actual_length"],
                          r["original_length"])

    def __iter__(self):
        return (self[i] for i in range(len(self.table)))

    def into_inner(self):
        return list(self)

    @staticmethod
    def parse(data, endianness):
        a = _as_array(data)
        ctx = context()
        cap = a.size // 16 + 1
        out = np.zeros(cap, dtype=_abi.RECORD_DTYPE)
        n = ctypes.c_size_t(0)
        cons = ctypes.c_size_t(0)
        ctx.check(ctx.lib.npr_records_parse(ctx.handle, a.ctypes.data if a.size else None, a.size, endianness,
                                            out.ctypes.data, cap, ctypes.byref(n), ctypes.byref(cons)))
        return memoryview(a)[cons.value:], PcapRecords(a, out[: n.value])


class CaptureFile:
    """CaptureFile (src/file.rs:4-35)."""

    def __init__(self, global_header, records):
        self.global_header, self.records = global_header, records

    @staticmethod
    def parse(data):
        a = _as_array(data)
        ctx = context()
        cap = a.size // 16 + 1
        out = np.zeros(cap, dtype=_abi.RECORD_DTYPE)
        h = _abi.GlobalHeaderC()
        n = ctypes.c_size_t(0)
        cons = ctypes.c_size_t(0)
        ctx.check(ctx.lib.npr_capture_file_parse(ctx.handle, a.ctypes.data if a.size else None, a.size,
                                                 ctypes.byref(h), out.ctypes.data, cap, ctypes.byref(n),
                                                 ctypes.byref(cons)))
        return memoryview(a)[cons.value:], CaptureFile(GlobalHeader._from_c(h), PcapRecords(a, out[: n.value]))


def parse(data):
    """net_parser_rs::parse (src/lib.rs:44-46)."""
    return CaptureFile.parse(data)


class CaptureParser:
    """The README facade (README.md:17-28; absent from the reference's code)."""

    @staticmethod
    def parse_file(data):
        return CaptureFile.parse(data)[1].records.into_inner()

    @staticmethod
    def parse_records(data, endianness=LITTLE):  # README passes no endianness: native default
        return PcapRecords.parse(data, endianness)[1].into_inner()

    @staticmethod
    def parse_record(data, endianness=LITTLE):
        return PcapRecord.parse(data, endianness)[1]


from . import flow  # noqa: E402  (flow needs the classes above)
from . import layers  # noqa: E402
