"""net_parser_rs.layers — the reference's per-layer header objects:
Ethernet (src/layer2/ethernet.rs), IPv4 / IPv6 / Arp (src/layer3/{ipv4,ipv6,arp}.rs), Tcp / Udp
(src/layer4/{tcp,udp}.rs) and the Layer4 dispatch (src/layer4/mod.rs:14-27), with their `as_bytes`
serializers where the reference has them.

Each `parse` reads ONE header object through libnpr's host-side layer parsers (npr_ethernet_parse,
npr_ipv4_parse, ... in csrc/npr_layers.hip; no device work): an object API for callers that inspect
or rebuild frames.  The flows of whole captures never come from here; they come from the device
(extract_flow / convert_records).  The parsers follow the reference's nom 4 chains in order, with
its quirks (release-build wrapping arithmetic):
- Ethernet: a VLAN tag's prio / dei are `(total & 0x7000) as u8` / `(total & 0x8000) as u8`, i.e. 0;
- IPv4: the payload is `total_length - header_length` (u16, wrapping) bytes taken right after the
  20-byte header, THEN the options, then trailing padding; as_bytes writes them in that order;
- IPv6: one next-header byte per "extension" header (quirk Q11);
- Udp: the payload is `length - 8` bytes (usize, wrapping: a length below 8 asks for ~2^64 bytes).
Errors are the reference's (src/errors.rs:3-55): Incomplete(size) for nom's Needed::Size, Failure
"Error: Code(<input>, MapOpt|MapRes)" for a map_opt! / map_res! (an unknown EtherType / IP protocol,
a TCP header length outside 20..60), Custom for the IP version checks.
"""
import ipaddress
import struct

import ctypes

from . import Custom, DeviceError, Failure, Incomplete, _abi
from .flow import MacAddress, Vxlan

__all__ = ["EthernetTypeId", "VlanTag", "Ethernet", "InternetProtocolId", "IPv4", "IPv6", "Arp", "Tcp", "Udp",
           "Layer4"]

_U64 = (1 << 64) - 1


def _call(name, data, out, *mid):
    """libnpr's host parser `name` over `data`: (the input bytes, *consumed) or the reference's error.
    `mid` are the arguments between the output struct and (consumed, detail)."""
    buf = bytes(data)
    arr = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    used, det = ctypes.c_size_t(0), ctypes.c_uint64(0)
    st = getattr(_abi.load_library(), name)(ctypes.addressof(arr), len(buf), ctypes.byref(out), *mid,
                                           ctypes.byref(used), ctypes.byref(det))
    return buf, used.value, st, det.value


def _check(st, det, buf, kind, custom):
    if st == _abi.OK or st == -3:  # NPR_ERR_CAPACITY: the caller asks again with room
        return
    if st == _abi.INCOMPLETE:
        raise Incomplete(det)
    if st == _abi.FAILURE:  # nom's Context::Code(<the failing primitive's input>, kind)
        a, b = det & 0xFFFFFFFF, det >> 32
        raise Failure(f"Error: Code({list(buf[a:b])}, {kind})")
    if st == _abi.CUSTOM:
        raise Custom(custom.format(det))
    raise DeviceError(f"{_abi.load_library()} layer parser status {st}")


def _slice(buf, off, n):
    return buf[off:off + n]


# ---- layer 2 ------------------------------------------------------------------------------------
class EthernetTypeId:
    """EthernetTypeId (src/layer2/ethernet.rs:49-83): kind "PayloadLength" (value = the length),
    "Vlan" (name VlanTagId / ProviderBridging) or "L3" (name Lldp / IPv4 / IPv6 / Arp)."""
    _KNOWN = {0x8100: ("Vlan", "VlanTagId"), 0x88A8: ("Vlan", "ProviderBridging"), 0x88CC: ("L3", "Lldp"),
              0x0800: ("L3", "IPv4"), 0x86DD: ("L3", "IPv6"), 0x0806: ("L3", "Arp")}
    __slots__ = ("kind", "name", "_value")

    def __init__(self, kind, name, value):
        self.kind, self.name, self._value = kind, name, value

    @classmethod
    def new(cls, v):
        """EthernetTypeId::new (:57-72): None for anything else above 1500."""
        if v in cls._KNOWN:
            return cls(*cls._KNOWN[v], v)
        if v <= 1500:
            return cls("PayloadLength", None, v)
        return None

    def value(self):
        return self._value

    def __eq__(self, o):
        return isinstance(o, EthernetTypeId) and (self.kind, self._value) == (o.kind, o._value)

    def __repr__(self):
        return f"{self.kind}({self.name if self.name else self._value})"


class VlanTag:
    """VlanTag (src/layer2/ethernet.rs:85-98)."""
    __slots__ = ("vlan_type", "vlan_value", "prio", "dei", "id")

    def __init__(self, vlan_type, vlan_value):
        self.vlan_type, self.vlan_value = vlan_type, vlan_value
        self.prio = (vlan_value & 0x7000) & 0xFF  # `as u8` of a value whose low byte is 0: always 0
        self.dei = (vlan_value & 0x8000) & 0xFF   # likewise
        self.id = vlan_value & 0x0FFF

    def vlan(self):
        return self.id


class Ethernet:
    """Ethernet (src/layer2/ethernet.rs:100-216)."""
    __slots__ = ("dst_mac", "src_mac", "ether_type", "vlans", "payload")

    def __init__(self, dst_mac, src_mac, ether_type, vlans, payload):
        self.dst_mac, self.src_mac = MacAddress(dst_mac), MacAddress(src_mac)
        self.ether_type, self.vlans, self.payload = ether_type, list(vlans), bytes(payload)

    @staticmethod
    def parse(data):
        """Ethernet::parse (:204-216) by npr_ethernet_parse: two MACs, then EtherType / VLAN tags until
        a non-VLAN type, then the rest as payload.  -> (remainder, Ethernet); the remainder is always
        empty."""
        cap = 8
        while True:
            out, tags = _abi.EthernetC(), (_abi.VlanTagC * cap)()
            buf, used, st, det = _call("npr_ethernet_parse", data, out, ctypes.addressof(tags), cap)
            _check(st, det, buf, "MapOpt", "")
            if out.n_vlans <= cap:
                break
            cap = out.n_vlans
        vlans = [VlanTag(EthernetTypeId.new(t.vlan_type), t.vlan_value) for t in tags[:out.n_vlans]]
        return buf[used:], Ethernet(bytes(out.dst_mac), bytes(out.src_mac), EthernetTypeId.new(out.ether_type), vlans,
                                    _slice(buf, out.payload_offset, out.payload_length))

    def as_bytes(self):
        """Ethernet::as_bytes (:116-132)."""
        out = bytes(self.dst_mac) + bytes(self.src_mac)
        for v in self.vlans:
            out += struct.pack(">HH", v.vlan_type.value(), v.vlan_value)
        return out + struct.pack(">H", self.ether_type.value()) + self.payload

    @staticmethod
    def vlans_to_vlan(vlans):
        return vlans[0].vlan() if vlans else 0

    def vlan(self):
        return Ethernet.vlans_to_vlan(self.vlans)


# ---- layer 3 ------------------------------------------------------------------------------------
class InternetProtocolId:
    """InternetProtocolId (src/layer3/mod.rs:24-72)."""
    _NAMES = {0: "HopByHop", 1: "ICMP", 6: "Tcp", 17: "Udp", 43: "IPv6Route", 44: "IPv6Fragment",
              50: "AuthenticationHeader", 51: "EncapsulatingSecurityPayload", 59: "IPv6NoNext", 60: "IPv6Options"}
    __slots__ = ("name", "_value")

    def __init__(self, value):
        self._value, self.name = value, self._NAMES[value]

    @classmethod
    def new(cls, v):
        return cls(v) if v in cls._NAMES else None

    def value(self):
        return self._value

    def __eq__(self, o):
        return isinstance(o, InternetProtocolId) and self._value == o._value

    def __repr__(self):
        return self.name


class IPv4:
    """IPv4 (src/layer3/ipv4.rs:14-160)."""
    __slots__ = ("version_and_length", "tos", "raw_length", "id", "flags", "ttl", "protocol", "checksum",
                 "src_ip", "dst_ip", "payload", "options", "padding")

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw[k])

    @staticmethod
    def parse(data):
        """IPv4::parse (:148-160) + parse_ipv4 (:76-146) by npr_ipv4_parse.  -> (remainder, IPv4)."""
        o = _abi.IPv4C()
        buf, used, st, det = _call("npr_ipv4_parse", data, o)
        _check(st, det, buf, "MapOpt", "Expected version 4, was {}")
        return buf[used:], IPv4(version_and_length=o.version_and_length, tos=o.tos, raw_length=o.raw_length, id=o.id,
                                flags=o.flags, ttl=o.ttl, protocol=InternetProtocolId(o.protocol), checksum=o.checksum,
                                src_ip=ipaddress.IPv4Address(bytes(o.src_ip)),
                                dst_ip=ipaddress.IPv4Address(bytes(o.dst_ip)),
                                payload=_slice(buf, o.payload_offset, o.payload_length),
                                options=_slice(buf, o.options_offset, o.options_length) if o.options_length else None,
                                padding=_slice(buf, o.padding_offset, o.padding_length) if o.padding_length else None)

    def as_bytes(self):
        """IPv4::as_bytes (:42-74): header fields, addresses, payload, options, padding."""
        out = struct.pack(">BBHHHBBH", self.version_and_length, self.tos, self.raw_length, self.id, self.flags,
                          self.ttl, self.protocol.value(), self.checksum)
        out += self.src_ip.packed + self.dst_ip.packed + self.payload
        return out + (self.options or b"") + (self.padding or b"")


class IPv6:
    """IPv6 (src/layer3/ipv6.rs:10-16).  The reference has no serializer for it."""
    __slots__ = ("dst_ip", "src_ip", "protocol", "payload")

    def __init__(self, dst_ip, src_ip, protocol, payload):
        self.dst_ip, self.src_ip, self.protocol, self.payload = dst_ip, src_ip, protocol, payload

    @staticmethod
    def parse(data):
        """IPv6::parse (:87-99) by npr_ipv6_parse: version 6, flow label, payload length, the next
        header (one byte per "extension" header), hop limit, the addresses, take!(payload length)."""
        o = _abi.IPv6C()
        buf, used, st, det = _call("npr_ipv6_parse", data, o)
        _check(st, det, buf, "MapOpt", "Expected version 6, version was {}")
        return buf[used:], IPv6(ipaddress.IPv6Address(bytes(o.dst_ip)), ipaddress.IPv6Address(bytes(o.src_ip)),
                                InternetProtocolId(o.protocol), _slice(buf, o.payload_offset, o.payload_length))


class Arp:
    """Arp (src/layer3/arp.rs:7-14).  The reference has no serializer for it."""
    __slots__ = ("sender_ip", "sender_mac", "target_ip", "target_mac", "operation")

    def __init__(self, sender_ip, sender_mac, target_ip, target_mac, operation):
        self.sender_ip, self.sender_mac, self.target_ip = sender_ip, MacAddress(sender_mac), target_ip
        self.target_mac, self.operation = MacAddress(target_mac), operation

    @staticmethod
    def parse(data):
        """Arp::parse (:54-76) by npr_arp_parse."""
        o = _abi.ArpC()
        buf, used, st, det = _call("npr_arp_parse", data, o)
        _check(st, det, buf, "MapOpt", "")
        return buf[used:], Arp(ipaddress.IPv4Address(bytes(o.sender_ip)), bytes(o.sender_mac),
                               ipaddress.IPv4Address(bytes(o.target_ip)), bytes(o.target_mac), o.operation)


# ---- layer 4 ------------------------------------------------------------------------------------
class Tcp:
    """Tcp (src/layer4/tcp.rs:11-101)."""
    __slots__ = ("src_port", "dst_port", "sequence_number", "acknowledgement_number", "header_length_and_flags",
                 "header_length", "flags", "window", "check", "urgent", "options", "payload")

    def __init__(self, **kw):
        for k in self.__slots__:
            setattr(self, k, kw[k])

    @staticmethod
    def extract_length(value):
        return (value >> 12) * 4

    @staticmethod
    def parse(data):
        """Tcp::parse (:54-101) by npr_tcp_parse: a header length outside 20..60 is a map_res!
        Failure; payload = rest.  -> (remainder, Tcp)."""
        o = _abi.TcpC()
        buf, used, st, det = _call("npr_tcp_parse", data, o)
        _check(st, det, buf, "MapRes", "")
        return buf[used:], Tcp(src_port=o.src_port, dst_port=o.dst_port, sequence_number=o.sequence_number,
                               acknowledgement_number=o.acknowledgement_number,
                               header_length_and_flags=o.header_length_and_flags, header_length=o.header_length,
                               flags=o.flags, window=o.window, check=o.check, urgent=o.urgent,
                               options=_slice(buf, o.options_offset, o.options_length),
                               payload=_slice(buf, o.payload_offset, o.payload_length))

    def as_bytes(self):
        """Tcp::as_bytes (:33-51)."""
        return struct.pack(">HHIIHHHH", self.src_port, self.dst_port, self.sequence_number,
                           self.acknowledgement_number, self.header_length_and_flags, self.window, self.check,
                           self.urgent) + self.options + self.payload


class Udp:
    """Udp (src/layer4/udp.rs:10-50)."""
    __slots__ = ("src_port", "dst_port", "checksum", "payload")

    def __init__(self, src_port, dst_port, checksum, payload):
        self.src_port, self.dst_port, self.checksum, self.payload = src_port, dst_port, checksum, bytes(payload)

    @staticmethod
    def parse(data):
        """Udp::parse (:33-50) by npr_udp_parse: payload = take!(length - 8), usize wrapping.
        -> (remainder, Udp)."""
        o = _abi.UdpC()
        buf, used, st, det = _call("npr_udp_parse", data, o)
        _check(st, det, buf, "MapOpt", "")
        return buf[used:], Udp(o.src_port, o.dst_port, o.checksum, _slice(buf, o.payload_offset, o.payload_length))

    def as_bytes(self):
        """Udp::as_bytes (:19-31): the length field is len(payload) + 8 (as u16)."""
        return struct.pack(">HHHH", self.src_port, self.dst_port, (len(self.payload) + 8) & 0xFFFF,
                           self.checksum) + self.payload


class Layer4:
    """Layer4 (src/layer4/mod.rs:8-27): Tcp, Udp or Vxlan; as_bytes of the one it holds."""
    __slots__ = ("inner",)

    def __init__(self, inner):
        assert isinstance(inner, (Tcp, Udp, Vxlan))
        self.inner = inner

    def as_bytes(self):
        return self.inner.as_bytes()
