"""ctypes / numpy view of include/npr.h (the C-ABI of libnpr.so).

Loading is strict: if the HIP library is missing this raises instead of falling back to
anything else — there is no CPU path in the product.
"""
import ctypes
import os
import warnings

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)                 # net-parser-rs_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libnpr.so")

# ---- numpy record dtypes (byte-for-byte the C structs) ----------------------------------
RECORD_DTYPE = np.dtype(
    [("offset", "<u8"), ("ts_sec", "<u4"), ("ts_usec", "<u4"),
     ("actual_length", "<u4"), ("original_length", "<u4")], align=True)
FLOW_DTYPE = np.dtype(
    [("src_ip", "u1", (4,)), ("dst_ip", "u1", (4,)), ("src_port", "<u2"), ("dst_port", "<u2"),
     ("vlan", "<u2"), ("src_mac", "u1", (6,)), ("dst_mac", "u1", (6,)), ("kind", "u1"),
     ("record_offset", "u1", (5,))], align=True)
FLOW_V6_DTYPE = np.dtype([("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,))])
SUMMARY_DTYPE = np.dtype([("n_records", "<u8"), ("n_flows", "<u8"), ("consumed", "<u8"),
                          ("flags", "<u4"), ("epoch", "<u4"), ("entry", "<u8")])
assert RECORD_DTYPE.itemsize == 24 and FLOW_DTYPE.itemsize == 32 and FLOW_V6_DTYPE.itemsize == 32
assert SUMMARY_DTYPE.itemsize == 40
NO_ENTRY = 0xFFFFFFFFFFFFFFFF

KIND_IPV6 = 0x1
KIND_UDP = 0x2

# npr_status
OK, INCOMPLETE, FAILURE, CUSTOM = 0, 1, 2, 3
OPT_PARK_FLOWS = 1  # npr_ctx_set_option: accepted for ABI 2 callers, no effect
OPT_RESIDENT = 2    # npr_ctx_set_option: flows-only parses run the resident single pass (0 off, 1 auto, N>1 cap)
# row f3 statuses (include/npr.h): outer failures keep their npr_flow_status code
VXLAN_NOT_UDP = 32
VXLAN_PORT = 33
VXLAN_INCOMPLETE = 34
VXLAN_INNER = 64  # + the inner frame's npr_flow_status
VXLAN_PORT_IANA = 4789
OPT_PIPE = 4  # npr_ctx_set_option: the pipelined pass (an experiment) is not built: only 0 is accepted
OPT_DEVICE_WINDOW = 5  # npr_ctx_set_option: npr_parse_extract_pipelined's device window in chunks (0 auto, >= 3)
OPT_STREAM_CHUNK = 3  # npr_ctx_set_option: host flows-only parses copy in chunks of N KiB overlapped (0 off, default)
PASS_TWO_PASS, PASS_RESIDENT, PASS_SPARSE = 1, 2, 8  # npr_ctx_last_pass (4, the removed batched launch, no longer occurs)
OPT_SPARSE = 6      # npr_ctx_set_option: the sparse record walk (0 auto, 1 never, 2 always, N >= 64 lane bytes)
OPT_SPARSE_CAP = 7  # npr_ctx_set_option: record slots per sparse lane (0 = default 96, at most 128)
ERR_ARG, ERR_DEVICE, ERR_CAPACITY, ERR_TIMEOUT, ERR_NOMEM = -1, -2, -3, -4, -5
LITTLE, BIG = 0, 1

# npr_flow_status (include/npr.h), name -> code
FLOW_STATUS = {
    "OK": 0, "ETH_INCOMPLETE": 1, "ETH_FAILURE": 2, "L2_ETHERTYPE": 3,
    "L2_IPV4_INCOMPLETE": 4, "L2_IPV4_FAILURE": 5, "L2_IPV4_CUSTOM": 6,
    "L2_IPV6_INCOMPLETE": 7, "L2_IPV6_FAILURE": 8, "L2_IPV6_CUSTOM": 9,
    "L2_ARP_INCOMPLETE": 10, "L2_IPV4_REMAINDER": 11, "L2_IPV6_REMAINDER": 12,
    "L2_ARP_REMAINDER": 13, "L3_ARP": 14, "L3_IPV4_PROTOCOL": 15, "L3_IPV6_PROTOCOL": 16,
    "L3_IPV4_TCP_INCOMPLETE": 17, "L3_IPV4_TCP_FAILURE": 18, "L3_IPV4_UDP_INCOMPLETE": 19,
    "L3_IPV6_TCP_INCOMPLETE": 20, "L3_IPV6_TCP_FAILURE": 21, "L3_IPV6_UDP_INCOMPLETE": 22,
    "L3_IPV4_UDP_REMAINDER": 23, "L3_IPV6_UDP_REMAINDER": 24,
}
FLOW_STATUS_NAME = {v: k for k, v in FLOW_STATUS.items()}


class GlobalHeaderC(ctypes.Structure):
    _fields_ = [("endianness", ctypes.c_int32), ("version_major", ctypes.c_uint16),
                ("version_minor", ctypes.c_uint16), ("zone", ctypes.c_int32),
                ("sig_figs", ctypes.c_int32), ("snap_length", ctypes.c_uint32),
                ("network", ctypes.c_uint32)]


class RecordC(ctypes.Structure):
    _fields_ = [("offset", ctypes.c_uint64), ("ts_sec", ctypes.c_uint32),
                ("ts_usec", ctypes.c_uint32), ("actual_length", ctypes.c_uint32),
                ("original_length", ctypes.c_uint32)]


class DevOutputsC(ctypes.Structure):
    _fields_ = [("record_offsets", ctypes.c_void_p), ("records", ctypes.c_void_p),
                ("record_status", ctypes.c_void_p),
                ("record_cap", ctypes.c_uint64), ("flows", ctypes.c_void_p),
                ("flows_v6", ctypes.c_void_p), ("flow_cap", ctypes.c_uint64),
                ("summary", ctypes.c_void_p)]


class BatchItemC(ctypes.Structure):
    """npr_batch_item: one capture of npr_dev_parse_extract_batch."""
    _fields_ = [("input", ctypes.c_void_p), ("len", ctypes.c_uint64), ("start", ctypes.c_uint64),
                ("endianness", ctypes.c_int32), ("reserved", ctypes.c_int32), ("out", DevOutputsC)]


class ShardC(ctypes.Structure):
    _fields_ = [("base", ctypes.c_uint64), ("start", ctypes.c_uint64), ("stop", ctypes.c_uint64),
                ("speculative_start", ctypes.c_int32), ("usec_magic", ctypes.c_int32),
                ("ts_ref", ctypes.c_uint64), ("chunk_bytes", ctypes.c_uint64)]


class SummaryC(ctypes.Structure):
    _fields_ = [("n_records", ctypes.c_uint64), ("n_flows", ctypes.c_uint64),
                ("consumed", ctypes.c_uint64), ("flags", ctypes.c_uint32),
                ("epoch", ctypes.c_uint32), ("entry", ctypes.c_uint64)]


# ---- host-side per-layer header objects (npr.h "host-side per-layer header objects") -------------
_u64 = ctypes.c_uint64


class VlanTagC(ctypes.Structure):
    _fields_ = [("vlan_type", ctypes.c_uint16), ("vlan_value", ctypes.c_uint16), ("prio", ctypes.c_uint8),
                ("dei", ctypes.c_uint8), ("id", ctypes.c_uint16)]


class EthernetC(ctypes.Structure):
    _fields_ = [("dst_mac", ctypes.c_uint8 * 6), ("src_mac", ctypes.c_uint8 * 6), ("ether_type", ctypes.c_uint16),
                ("reserved", ctypes.c_uint16), ("n_vlans", ctypes.c_uint32), ("payload_offset", _u64),
                ("payload_length", _u64)]


class IPv4C(ctypes.Structure):
    _fields_ = [("version_and_length", ctypes.c_uint8), ("tos", ctypes.c_uint8), ("raw_length", ctypes.c_uint16),
                ("id", ctypes.c_uint16), ("flags", ctypes.c_uint16), ("ttl", ctypes.c_uint8),
                ("protocol", ctypes.c_uint8), ("checksum", ctypes.c_uint16), ("src_ip", ctypes.c_uint8 * 4),
                ("dst_ip", ctypes.c_uint8 * 4), ("payload_offset", _u64), ("payload_length", _u64),
                ("options_offset", _u64), ("options_length", _u64), ("padding_offset", _u64),
                ("padding_length", _u64)]


class IPv6C(ctypes.Structure):
    _fields_ = [("dst_ip", ctypes.c_uint8 * 16), ("src_ip", ctypes.c_uint8 * 16), ("protocol", ctypes.c_uint8),
                ("reserved", ctypes.c_uint8 * 7), ("payload_offset", _u64), ("payload_length", _u64)]


class ArpC(ctypes.Structure):
    _fields_ = [("sender_ip", ctypes.c_uint8 * 4), ("sender_mac", ctypes.c_uint8 * 6),
                ("target_ip", ctypes.c_uint8 * 4), ("target_mac", ctypes.c_uint8 * 6),
                ("operation", ctypes.c_uint16)]


class TcpC(ctypes.Structure):
    _fields_ = [("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16), ("sequence_number", ctypes.c_uint32),
                ("acknowledgement_number", ctypes.c_uint32), ("header_length_and_flags", ctypes.c_uint16),
                ("flags", ctypes.c_uint16), ("header_length", ctypes.c_uint32), ("window", ctypes.c_uint16),
                ("check", ctypes.c_uint16), ("urgent", ctypes.c_uint16), ("reserved", ctypes.c_uint16),
                ("options_offset", _u64), ("options_length", _u64), ("payload_offset", _u64),
                ("payload_length", _u64)]


class UdpC(ctypes.Structure):
    _fields_ = [("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16), ("checksum", ctypes.c_uint16),
                ("reserved", ctypes.c_uint16), ("payload_offset", _u64), ("payload_length", _u64)]


class VxlanC(ctypes.Structure):
    _fields_ = [("flags", ctypes.c_uint16), ("group_policy_id", ctypes.c_uint16),
                ("raw_network_identifier", ctypes.c_uint32), ("network_identifier", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("payload_offset", _u64), ("payload_length", _u64)]


assert ctypes.sizeof(GlobalHeaderC) == 24 and ctypes.sizeof(RecordC) == 24 and ctypes.sizeof(ShardC) == 48
assert (ctypes.sizeof(VlanTagC), ctypes.sizeof(EthernetC), ctypes.sizeof(IPv4C), ctypes.sizeof(IPv6C),
        ctypes.sizeof(ArpC), ctypes.sizeof(TcpC), ctypes.sizeof(UdpC), ctypes.sizeof(VxlanC)) == \
    (8, 40, 72, 56, 22, 64, 24, 32)

# Every symbol include/npr.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "npr_version", "npr_abi_version", "npr_ctx_create", "npr_ctx_destroy", "npr_ctx_last_error",
    "npr_ctx_set_stats", "npr_ctx_read_stats", "npr_ctx_read_stamps", "npr_ctx_set_option", "npr_ctx_last_pass",
    "npr_workspace_bytes", "npr_global_header_parse", "npr_record_parse", "npr_records_parse",
    "npr_capture_file_parse", "npr_extract_flows", "npr_convert_records", "npr_parse_extract",
    "npr_parse_extract_pipelined", "npr_host_alloc", "npr_host_free",
    "npr_dev_parse_extract", "npr_dev_parse_extract_range", "npr_dev_parse_extract_chain",
    "npr_dev_parse_extract_chunked", "npr_dev_parse_extract_shard", "npr_dev_check", "npr_dev_extract_flows",
    "npr_dev_convert_records", "npr_dev_vxlan_flows", "npr_vxlan_flows", "npr_dev_flow_aggregate",
    "npr_flow_details", "npr_dev_flow_details", "npr_dev_parse_extract_batch", "npr_shm_all_gather",
    "npr_stream_release", "npr_ctx_forget_density",
    "npr_ethernet_parse", "npr_ipv4_parse", "npr_ipv6_parse", "npr_arp_parse", "npr_tcp_parse", "npr_udp_parse",
    "npr_vxlan_parse",
]

_c_size_p = ctypes.POINTER(ctypes.c_size_t)
_vp = ctypes.c_void_p
_u8p = ctypes.c_void_p

_SIGNATURES = {
    "npr_version": (ctypes.c_char_p, []),
    "npr_abi_version": (ctypes.c_int, []),
    "npr_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "npr_ctx_destroy": (None, [_vp]),
    "npr_ctx_last_error": (ctypes.c_char_p, [_vp]),
    "npr_workspace_bytes": (ctypes.c_uint64, [ctypes.c_uint64]),
    "npr_ctx_set_stats": (ctypes.c_int, [_vp, ctypes.c_int]),
    "npr_ctx_set_option": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    "npr_ctx_last_pass": (ctypes.c_int, [_vp]),
    "npr_ctx_read_stats": (ctypes.c_int, [_vp, _vp, ctypes.c_int, ctypes.c_int]),
    "npr_ctx_read_stamps": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]),
    "npr_global_header_parse": (ctypes.c_int, [_u8p, ctypes.c_size_t, ctypes.POINTER(GlobalHeaderC), _c_size_p]),
    "npr_record_parse": (ctypes.c_int, [_u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(RecordC), _c_size_p]),
    "npr_records_parse": (ctypes.c_int, [_vp, _u8p, ctypes.c_size_t, ctypes.c_int, _vp, ctypes.c_size_t,
                                         _c_size_p, _c_size_p]),
    "npr_capture_file_parse": (ctypes.c_int, [_vp, _u8p, ctypes.c_size_t, ctypes.POINTER(GlobalHeaderC), _vp,
                                              ctypes.c_size_t, _c_size_p, _c_size_p]),
    "npr_extract_flows": (ctypes.c_int, [_vp, _u8p, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp, _vp, _vp]),
    "npr_convert_records": (ctypes.c_int, [_vp, _u8p, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp, _vp,
                                           ctypes.c_size_t, _c_size_p]),
    "npr_parse_extract": (ctypes.c_int, [_vp, _u8p, ctypes.c_size_t, ctypes.POINTER(GlobalHeaderC), _vp,
                                         ctypes.c_size_t, _c_size_p, _vp, _vp, ctypes.c_size_t, _c_size_p,
                                         _c_size_p]),
    "npr_parse_extract_pipelined": (ctypes.c_int, [_vp, _u8p, ctypes.c_size_t, ctypes.POINTER(GlobalHeaderC), _vp, _vp,
                                                   ctypes.c_size_t, _c_size_p, _c_size_p, ctypes.c_uint64]),
    "npr_host_alloc": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "npr_host_free": (ctypes.c_int, [_vp, _vp]),
    "npr_dev_parse_extract": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                             ctypes.POINTER(DevOutputsC), _vp]),
    "npr_dev_parse_extract_range": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                   ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                                   ctypes.POINTER(DevOutputsC), _vp]),
    "npr_dev_parse_extract_chain": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                   ctypes.c_int, _vp, ctypes.c_uint64,
                                                   ctypes.POINTER(DevOutputsC), _vp]),
    "npr_dev_parse_extract_chunked": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                                     ctypes.POINTER(DevOutputsC), ctypes.c_uint64, _vp]),
    "npr_dev_parse_extract_shard": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ShardC),
                                                   ctypes.POINTER(DevOutputsC), _vp]),
    "npr_dev_check": (ctypes.c_int, [_vp, ctypes.POINTER(DevOutputsC), _vp, ctypes.POINTER(SummaryC)]),
    "npr_dev_extract_flows": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                             _vp, _vp, _vp, _vp]),
    "npr_dev_convert_records": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                               _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "npr_dev_vxlan_flows": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "npr_dev_flow_aggregate": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp, _vp, ctypes.c_uint64,
                                              _vp, _vp]),
    "npr_vxlan_flows": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, ctypes.c_uint32,
                                       ctypes.c_int, _vp, _vp, _vp, _vp]),
    "npr_flow_details": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp, ctypes.c_size_t, _vp, _vp]),
    "npr_dev_flow_details": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp, _vp, _vp]),
    "npr_dev_parse_extract_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
    "npr_stream_release": (ctypes.c_int, [_vp, _vp]),
    "npr_ctx_forget_density": (ctypes.c_int, [_vp, _vp]),
    "npr_ethernet_parse": (ctypes.c_int, [_u8p, ctypes.c_size_t, ctypes.POINTER(EthernetC), _vp, ctypes.c_size_t,
                                          _c_size_p, ctypes.POINTER(ctypes.c_uint64)]),
    **{f"npr_{k}_parse": (ctypes.c_int, [_u8p, ctypes.c_size_t, ctypes.POINTER(c), _c_size_p,
                                         ctypes.POINTER(ctypes.c_uint64)])
       for k, c in (("ipv4", IPv4C), ("ipv6", IPv6C), ("arp", ArpC), ("tcp", TcpC), ("udp", UdpC))},
    "npr_vxlan_parse": (ctypes.c_int, [_u8p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(VxlanC), _c_size_p,
                                       ctypes.POINTER(ctypes.c_uint64)]),
    "npr_shm_all_gather": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.c_uint64, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
}

ABI_VERSION = 5  # include/npr.h NPR_ABI_VERSION: the layout these bindings assume

_lib = None


def load_library(path=None):
    """Load libnpr.so (built by __graft_entry__.build()); raise loudly if it is absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("NPR_LIB") or LIB_PATH  # NPR_LIB: an alternative in-tree build (experiments)
    if not os.path.exists(p):
        raise ImportError(
            f"libnpr.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (the parser has no CPU fallback)")
    lib = ctypes.CDLL(p)
    # An A/B build of an older revision (NPR_LIB) may predate a symbol or the ABI: that is refused
    # unless NPR_LIB_ALLOW_OLD=1 says the experiment expects it; the product library
    # must match exactly.
    allow_old = p != LIB_PATH and os.environ.get("NPR_LIB_ALLOW_OLD") == "1"
    abi_fn = getattr(lib, "npr_abi_version", None)
    abi = abi_fn() if abi_fn is not None else None
    if abi != ABI_VERSION:
        msg = f"{p}: ABI {abi}, this package binds ABI {ABI_VERSION}"
        if not allow_old:
            raise ImportError(msg + " (set NPR_LIB_ALLOW_OLD=1 to load an older A/B build anyway)")
        warnings.warn(msg)
    missing = []
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            missing.append(name)
            continue
        fn.restype = res
        fn.argtypes = args
    if missing:
        msg = f"{p} does not export {', '.join(missing)}"
        if not allow_old:
            raise ImportError(msg)
        warnings.warn(msg)
    if path is None:
        _lib = lib
    return lib


def ptr(a):
    """Address of a numpy array / bytes-like (None -> NULL)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(a, dtype=np.uint8).ctypes.data
    raise TypeError(type(a))
