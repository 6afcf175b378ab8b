"""net_parser_rs.flow — mirror of src/flow/ (Flow, Device, errors, convert_records) over libnpr.so."""
import ctypes
import ipaddress

import struct

import numpy as np

from . import _abi

__all__ = ["Flow", "Device", "MacAddress", "FlowError", "convert_records", "FlowExtraction"]


class MacAddress(bytes):
    """common::MacAddress (src/common.rs:3-26)."""

    def __str__(self):
        return ":".join(f"{b:02x}" for b in self)


class Device:
    """flow::device::Device (src/flow/device.rs:7-27)."""
    __slots__ = ("mac", "ip", "port")

    def __init__(self, mac, ip, port):
        self.mac, self.ip, self.port = MacAddress(mac), ip, int(port)

    def __eq__(self, o):
        return isinstance(o, Device) and (self.mac, self.ip, self.port) == (o.mac, o.ip, o.port)

    def __str__(self):
        return f"Mac={self.mac}   Ip={_ip_str(self.ip)}   Port={self.port}"


def _ip_str(ip):
    if isinstance(ip, ipaddress.IPv6Address):
        return str(ip)  # RFC 5952 form, as std::net::Ipv6Addr's Display for ordinary addresses
    return str(ip)


class Flow:
    """flow::Flow (src/flow/mod.rs:53-96).  layer2 is always "Ethernet"."""
    __slots__ = ("source", "destination", "layer2", "layer3", "layer4", "vlan", "record_offset")

    def __init__(self, source, destination, layer3, layer4, vlan, layer2="Ethernet", record_offset=None):
        self.source, self.destination = source, destination
        self.layer2, self.layer3, self.layer4, self.vlan = layer2, layer3, layer4, int(vlan)
        self.record_offset = record_offset

    def __eq__(self, o):
        return isinstance(o, Flow) and (self.source, self.destination, self.layer2, self.layer3, self.layer4,
                                        self.vlan) == (o.source, o.destination, o.layer2, o.layer3, o.layer4, o.vlan)

    def __str__(self):
        return f"Source=[{self.source}]   Destination=[{self.destination}]   Vlan={self.vlan}"

    @staticmethod
    def _from_row(row, v6row=None):
        kind = int(row["kind"])
        if kind & _abi.KIND_IPV6:
            src = ipaddress.IPv6Address(bytes(v6row["src_ip"]))
            dst = ipaddress.IPv6Address(bytes(v6row["dst_ip"]))
        else:
            src = ipaddress.IPv4Address(bytes(row["src_ip"]))
            dst = ipaddress.IPv4Address(bytes(row["dst_ip"]))
        off = int.from_bytes(bytes(row["record_offset"]), "little")
        return Flow(Device(bytes(row["src_mac"]), src, row["src_port"]),
                    Device(bytes(row["dst_mac"]), dst, row["dst_port"]),
                    "IPv6" if kind & _abi.KIND_IPV6 else "IPv4",
                    "Udp" if kind & _abi.KIND_UDP else "Tcp", row["vlan"], record_offset=off)


# npr_flow_status leaves whose variant carries a size (include/npr.h npr_flow_details): nom-level
# Incomplete (Needed::Size) and the flow-level remainders (rem.len())
_SIZED = {1, 4, 7, 10, 17, 19, 20, 22} | {11, 12, 13, 23, 24}


class FlowError(Exception):
    """flow::errors::Error (src/flow/errors.rs:5-19); `.code` is the npr_flow_status leaf, `.detail`
    the payload its variant carries (npr_flow_details: a size, an offset, a version, an EtherType
    or a protocol id; None when not computed) and `.size` the `size` field of the sized variants."""

    def __init__(self, code, detail=None):
        self.code = int(code)
        self.detail = None if detail is None else int(detail)
        self.name = _abi.FLOW_STATUS_NAME.get(self.code, f"UNKNOWN_{code}")
        super().__init__(self.name if self.detail is None else f"{self.name}({self.detail})")

    @property
    def size(self):
        return self.detail if self.code in _SIZED else None


def _details(buf, records):
    """(status, detail) of extract_flow over records indexing into `buf` (npr_flow_details)."""
    from . import context
    ctx = context()
    a = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    t = _table(records)
    n = len(t)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    detail = np.zeros(max(n, 1), dtype=np.uint64)
    ctx.check(ctx.lib.npr_flow_details(ctx.handle, a.ctypes.data if a.size else None, a.size, t.ctypes.data, n,
                                       status.ctypes.data, detail.ctypes.data))
    return status[:n], detail[:n]


def _table(records):
    t = np.zeros(len(records), dtype=_abi.RECORD_DTYPE)
    for i, r in enumerate(records):
        t[i] = (r.offset, r.ts_sec, r.ts_usec, r.actual_length, r.original_length)
    return t


def _extract(buf, records):
    """Dense extract over records that all index into `buf` (one device launch)."""
    from . import context
    ctx = context()
    a = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    t = _table(records)
    n = len(t)
    flows = np.zeros(max(n, 1), dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(max(n, 1), dtype=_abi.FLOW_V6_DTYPE)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    ctx.check(ctx.lib.npr_extract_flows(ctx.handle, a.ctypes.data if a.size else None, a.size, t.ctypes.data, n,
                                        flows.ctypes.data, v6.ctypes.data, status.ctypes.data))
    return flows[:n], v6[:n], status[:n]


def convert_records(records):
    """flow::convert_records (src/flow/mod.rs:101-123): [(record, Flow)] for Ok records, in REVERSE
    record order (the reference pops from the end)."""
    from . import context
    records = list(records)
    if not records:
        return []
    # group by backing buffer (records from one parse share it); keep the global reverse order
    out = []
    bufs = {}
    for r in records:
        bufs.setdefault(id(r._buf), r._buf)
    if len(bufs) == 1:
        buf = next(iter(bufs.values()))
        ctx = context()
        a = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
        t = _table(records)
        n = len(t)
        flows = np.zeros(n, dtype=_abi.FLOW_DTYPE)
        v6 = np.zeros(n, dtype=_abi.FLOW_V6_DTYPE)
        k = ctypes.c_size_t(0)
        ctx.check(ctx.lib.npr_convert_records(ctx.handle, a.ctypes.data if a.size else None, a.size, t.ctypes.data,
                                              n, flows.ctypes.data, v6.ctypes.data, n, ctypes.byref(k)))
        # rows are the Ok records in reverse list order: pair each with the next record (walking the
        # list backwards) at its offset, so a record listed twice yields two pairs, as in the reference
        j = n - 1
        for i in range(k.value):
            f = Flow._from_row(flows[i], v6[i])
            while records[j].offset != f.record_offset:
                j -= 1
            out.append((records[j], f))
            j -= 1
        return out
    for r in reversed(records):
        try:
            out.append((r, r.extract_flow()))
        except FlowError:
            pass
    return out


class Vxlan:
    """layer4::Vxlan (src/layer4/vxlan.rs:7-49): the 8-byte VXLAN header and the rest as payload."""
    __slots__ = ("flags", "group_policy_id", "raw_network_identifier", "network_identifier", "payload")

    def __init__(self, flags, group_policy_id, raw_network_identifier, payload):
        self.flags, self.group_policy_id = int(flags), int(group_policy_id)
        self.raw_network_identifier = int(raw_network_identifier)
        self.network_identifier = self.raw_network_identifier >> 8  # only 3 bytes are the VNI (:45)
        self.payload = bytes(payload)

    @staticmethod
    def parse(data, endianness):
        """Vxlan::parse (:31-48) by npr_vxlan_parse: (remainder, Vxlan); a short header raises
        net_parser_rs.Incomplete with nom's Needed::Size (u16!: 2, u32!: 4); the remainder is always
        empty (rest)."""
        from . import Incomplete, DeviceError
        buf = bytes(data)
        arr = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
        o, used, det = _abi.VxlanC(), ctypes.c_size_t(0), ctypes.c_uint64(0)
        st = _abi.load_library().npr_vxlan_parse(ctypes.addressof(arr), len(buf), int(endianness), ctypes.byref(o),
                                                 ctypes.byref(used), ctypes.byref(det))
        if st == _abi.INCOMPLETE:
            raise Incomplete(det.value)
        if st != _abi.OK:
            raise DeviceError(f"npr_vxlan_parse status {st}")
        return buf[used.value:], Vxlan(o.flags, o.group_policy_id, o.raw_network_identifier,
                                       buf[o.payload_offset:o.payload_offset + o.payload_length])

    def as_bytes(self):
        """Vxlan::as_bytes (:18-29): big-endian header + payload."""
        return struct.pack(">HHI", self.flags, self.group_policy_id, self.raw_network_identifier) + self.payload


def vxlan_flows(records, dst_port=0, big=True):
    """Row f3: the VXLAN inner flow of each record (one device launch): a list of (record, Flow |
    FlowError, vni).  A record whose outer frame is not an Ok UDP flow to dst_port (0: any) or whose
    UDP payload is shorter than a VXLAN header gets a FlowError with the npr.h VXLAN code."""
    from . import context
    records = list(records)
    if not records:
        return []
    bufs = {id(r._buf): r._buf for r in records}
    if len(bufs) != 1:
        out = []
        for b in bufs.values():
            out += vxlan_flows([r for r in records if r._buf is b], dst_port, big)
        return out
    ctx = context()
    a = np.ascontiguousarray(next(iter(bufs.values())), dtype=np.uint8).reshape(-1)
    t = _table(records)
    n = len(t)
    flows = np.zeros(n, dtype=_abi.FLOW_DTYPE)
    v6 = np.zeros(n, dtype=_abi.FLOW_V6_DTYPE)
    status = np.zeros(n, dtype=np.uint8)
    vni = np.zeros(n, dtype=np.uint32)
    ctx.check(ctx.lib.npr_vxlan_flows(ctx.handle, a.ctypes.data if a.size else None, a.size, t.ctypes.data, n,
                                      int(dst_port), _abi.BIG if big else _abi.LITTLE, flows.ctypes.data,
                                      v6.ctypes.data, status.ctypes.data, vni.ctypes.data))
    return [(r, Flow._from_row(flows[i], v6[i]) if status[i] == 0 else FlowError(status[i]), int(vni[i]))
            for i, r in enumerate(records)]


class FlowExtraction:
    """Trait marker (src/flow/mod.rs:20-42): PcapRecord implements extract_flow()."""
