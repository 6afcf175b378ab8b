"""ctypes wrapper over oracle/build/liboracle.so — the parity CHECKER (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "net-parser-rs_amd"))
from net_parser_rs import _abi  # noqa: E402  (struct layouts only)

ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liboracle.so")

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_szp = ctypes.POINTER(ctypes.c_size_t)


class OrEth(ctypes.Structure):
    _fields_ = [("dst_mac", _vp), ("src_mac", _vp), ("ether_type", ctypes.c_uint16),
                ("vlan", ctypes.c_uint16), ("n_vlans", ctypes.c_uint32), ("payload_off", _sz)]


class OrVxlan(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint16), ("group_policy_id", ctypes.c_uint16),
                ("raw_network_identifier", ctypes.c_uint32), ("network_identifier", ctypes.c_uint32),
                ("payload_off", _sz)]


class OrIp(ctypes.Structure):
    _fields_ = [("src", _vp), ("dst", _vp), ("protocol", ctypes.c_uint8),
                ("payload_off", _sz), ("payload_len", _sz), ("rem", _sz)]


class OrArp(ctypes.Structure):
    _fields_ = [("operation", ctypes.c_uint16), ("sender_mac", _vp), ("sender_ip", _vp),
                ("target_mac", _vp), ("target_ip", _vp), ("rem", _sz)]


class OrL4(ctypes.Structure):
    _fields_ = [("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16),
                ("header_length", _sz), ("payload_off", _sz), ("payload_len", _sz), ("rem", _sz)]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.or_global_header_parse.argtypes = [_vp, _sz, ctypes.POINTER(_abi.GlobalHeaderC), _szp]
        L.or_record_parse.argtypes = [_vp, _sz, ctypes.c_int, ctypes.POINTER(_abi.RecordC), _szp]
        L.or_records_parse.argtypes = [_vp, _sz, ctypes.c_int, _vp, _sz, _szp]
        L.or_records_parse.restype = _sz
        L.or_capture_file_parse.argtypes = [_vp, _sz, ctypes.POINTER(_abi.GlobalHeaderC), _vp, _sz, _szp, _szp]
        L.or_extract_flow.argtypes = [_vp, _sz, ctypes.c_uint64, _vp, _vp]
        L.or_convert_records.argtypes = [_vp, _sz, _vp, _sz, _vp, _vp, _sz]
        L.or_convert_records.restype = _sz
        L.or_extract_flows.argtypes = [_vp, _sz, _vp, _sz, _vp, _vp, _vp]
        L.or_extract_flows.restype = None
        L.or_flow_details.argtypes = [_vp, _sz, _vp, _sz, _vp, _vp]
        L.or_flow_details.restype = None
        L.or_vxlan_flows.argtypes = [_vp, _sz, _vp, _sz, ctypes.c_uint32, ctypes.c_int, _vp, _vp, _vp, _vp]
        L.or_vxlan_flows.restype = None
        L.or_vxlan_parse.argtypes = [_vp, _sz, ctypes.c_int, ctypes.POINTER(OrVxlan)]
        L.or_vxlan_parse.restype = ctypes.c_int
        L.or_bench_extract.argtypes = [_vp, _sz, _vp, _sz, _vp, _vp, _sz, _szp]
        L.or_bench_extract.restype = _sz
        L.or_bench_extract_mt.argtypes = [_vp, _sz, _vp, _sz, _vp, _vp, _vp, _vp, _vp, _sz, _szp, ctypes.c_int]
        L.or_bench_extract_mt.restype = _sz
        L.or_eth_parse.argtypes = [_vp, _sz, ctypes.POINTER(OrEth)]
        L.or_ipv4_parse.argtypes = [_vp, _sz, ctypes.POINTER(OrIp)]
        L.or_ipv6_parse.argtypes = [_vp, _sz, ctypes.POINTER(OrIp)]
        L.or_arp_parse.argtypes = [_vp, _sz, ctypes.POINTER(OrArp)]
        L.or_tcp_parse.argtypes = [_vp, _sz, ctypes.POINTER(OrL4)]
        L.or_udp_parse.argtypes = [_vp, _sz, ctypes.POINTER(OrL4)]
        L.or_tcp_extract_length.argtypes = [ctypes.c_uint16]
        L.or_tcp_extract_length.restype = _sz
        _lib = L
    return _lib


def _buf(data):
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return a, (a.ctypes.data if a.size else None)


def global_header(data):
    a, p = _buf(data)
    h = _abi.GlobalHeaderC()
    used = _sz(0)
    rc = lib().or_global_header_parse(p, a.size, ctypes.byref(h), ctypes.byref(used))
    return rc, h, used.value


def record(data, endianness):
    a, p = _buf(data)
    r = _abi.RecordC()
    used = _sz(0)
    rc = lib().or_record_parse(p, a.size, endianness, ctypes.byref(r), ctypes.byref(used))
    return rc, r, used.value


def records_parse(data, endianness):
    a, p = _buf(data)
    cap = a.size // 16 + 1
    out = np.zeros(cap, dtype=_abi.RECORD_DTYPE)
    cons = _sz(0)
    n = lib().or_records_parse(p, a.size, endianness, out.ctypes.data, cap, ctypes.byref(cons))
    return out[:n], cons.value


def capture_file_parse(data):
    """-> (rc, header, records ndarray, consumed)"""
    a, p = _buf(data)
    cap = max(a.size // 16 + 1, 1)
    out = np.zeros(cap, dtype=_abi.RECORD_DTYPE)
    h = _abi.GlobalHeaderC()
    n = _sz(0)
    cons = _sz(0)
    rc = lib().or_capture_file_parse(p, a.size, ctypes.byref(h), out.ctypes.data, cap,
                                     ctypes.byref(n), ctypes.byref(cons))
    return rc, h, out[: n.value], cons.value


def extract_flow(payload, record_offset=0):
    a, p = _buf(payload)
    f = np.zeros(1, dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(1, dtype=_abi.FLOW_V6_DTYPE)
    st = lib().or_extract_flow(p, a.size, record_offset, f.ctypes.data, v6.ctypes.data)
    return st, f[0], v6[0]


def extract_flows(data, records):
    a, p = _buf(data)
    n = len(records)
    recs = np.ascontiguousarray(records, dtype=_abi.RECORD_DTYPE)
    flows = np.zeros(n, dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(n, dtype=_abi.FLOW_V6_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    lib().or_extract_flows(p, a.size, recs.ctypes.data, n, flows.ctypes.data, v6.ctypes.data, st.ctypes.data)
    return flows, v6, st


def flow_details(data, records):
    """Per-record status and error payload (include/npr.h npr_flow_details): (status, detail)."""
    a, p = _buf(data)
    n = len(records)
    recs = np.ascontiguousarray(records, dtype=_abi.RECORD_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    det = np.zeros(n, dtype=np.uint64)
    lib().or_flow_details(p, a.size, recs.ctypes.data, n, st.ctypes.data, det.ctypes.data)
    return st, det


def vxlan_flows(data, records, dst_port=0, big=True):
    """Row f3: the VXLAN inner flow of every record (dense): (flows, flows_v6, status, vni)."""
    a, p = _buf(data)
    n = len(records)
    recs = np.ascontiguousarray(records, dtype=_abi.RECORD_DTYPE)
    flows = np.zeros(n, dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(n, dtype=_abi.FLOW_V6_DTYPE)
    st = np.zeros(n, dtype=np.uint8)
    vni = np.zeros(n, dtype=np.uint32)
    lib().or_vxlan_flows(p, a.size, recs.ctypes.data, n, dst_port, 1 if big else 0, flows.ctypes.data,
                         v6.ctypes.data, st.ctypes.data, vni.ctypes.data)
    return flows, v6, st, vni


def vxlan_parse(data, big=True):
    """Vxlan::parse (src/layer4/vxlan.rs:31-48): (rc, OrVxlan)."""
    a, p = _buf(data)
    v = OrVxlan()
    return lib().or_vxlan_parse(p, a.size, 1 if big else 0, ctypes.byref(v)), v


def convert_records(data, records):
    a, p = _buf(data)
    n = len(records)
    recs = np.ascontiguousarray(records, dtype=_abi.RECORD_DTYPE)
    flows = np.zeros(max(n, 1), dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(max(n, 1), dtype=_abi.FLOW_V6_DTYPE)
    k = lib().or_convert_records(p, a.size, recs.ctypes.data, n, flows.ctypes.data, v6.ctypes.data, n)
    return flows[:k], v6[:k]


def bench_extract(data, rec_scratch, flow_scratch, v6_scratch):
    """CaptureFile::parse + convert_records (benches/benches.rs:56-62); returns (n_flows, n_records)."""
    a, p = _buf(data)
    nrec = _sz(0)
    k = lib().or_bench_extract(p, a.size, rec_scratch.ctypes.data, rec_scratch.size,
                               flow_scratch.ctypes.data, v6_scratch.ctypes.data, flow_scratch.size,
                               ctypes.byref(nrec))
    return k, nrec.value


class MtScratch:
    """Scratch of the multi-threaded bench leg for captures of up to n records."""

    def __init__(self, n):
        n = max(n, 1)
        self.rec = np.zeros(n, dtype=_abi.RECORD_DTYPE)
        self.dense = np.zeros(n, dtype=_abi.FLOW_DTYPE)
        self.dense6 = np.zeros(n, dtype=_abi.FLOW_V6_DTYPE)
        self.status = np.zeros(n, dtype=np.uint8)
        self.out = np.zeros(n, dtype=_abi.FLOW_DTYPE)
        self.out6 = np.zeros(n, dtype=_abi.FLOW_V6_DTYPE)


def bench_extract_mt(data, scratch, nthreads):
    """bench_extract on `nthreads` host threads; returns (n_flows, n_records); flows in scratch.out."""
    a, p = _buf(data)
    nrec = _sz(0)
    s = scratch
    k = lib().or_bench_extract_mt(p, a.size, s.rec.ctypes.data, s.rec.size, s.dense.ctypes.data, s.dense6.ctypes.data,
                                  s.status.ctypes.data, s.out.ctypes.data, s.out6.ctypes.data, s.out.size,
                                  ctypes.byref(nrec), int(nthreads))
    return k, nrec.value
