"""net_parser_rs.layers — host mirror of the reference's per-layer header objects and their
`as_bytes` serializers: Ethernet (src/layer2/ethernet.rs), IPv4
(src/layer3/ipv4.rs), Tcp / Udp (src/layer4/{tcp,udp}.rs) and the Layer4 dispatch
(src/layer4/mod.rs:14-27).

These parse ONE header object from a byte string, like GlobalHeader::parse: an object API for
callers that inspect or rebuild frames.  The flows of whole captures never come from here; they come
from the device (extract_flow / convert_records over libnpr.so).  Each step follows the reference's
nom 4 chain in order, with its quirks (release-build wrapping arithmetic):
- Ethernet: a VLAN tag's prio / dei are `(total & 0x7000) as u8` / `(total & 0x8000) as u8`, i.e. 0;
- IPv4: the payload is `total_length - header_length` (u16, wrapping) bytes taken right after the
  20-byte header, THEN the options, then trailing padding; as_bytes writes them in that order;
- Udp: the payload is `length - 8` bytes (usize, wrapping: a length below 8 asks for ~2^64 bytes).
Errors are the reference's (src/errors.rs:3-55): Incomplete(size) for nom's Needed::Size, Failure
for a nom Error (an unknown EtherType / IP protocol, a TCP header length outside 20..60), Custom for
IPv4's version check.
"""
import ipaddress
import struct

from . import Custom, Failure, Incomplete
from .flow import MacAddress, Vxlan

__all__ = ["EthernetTypeId", "VlanTag", "Ethernet", "InternetProtocolId", "IPv4", "Tcp", "Udp", "Layer4"]

_U64 = (1 << 64) - 1


class _Reader:
    """nom 4's big-endian number parsers and take! over a byte string (Needed::Size on short input)."""
    __slots__ = ("b", "i")

    def __init__(self, data):
        self.b, self.i = bytes(data), 0

    def take(self, n):
        if len(self.b) - self.i < n:
            raise Incomplete(n)
        out = self.b[self.i:self.i + n]
        self.i += n
        return out

    def u8(self):
        return self.take(1)[0]

    def u16(self):
        return struct.unpack(">H", self.take(2))[0]

    def u32(self):
        return struct.unpack(">I", self.take(4))[0]

    def rest(self):
        out = self.b[self.i:]
        self.i = len(self.b)
        return out


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
        """Ethernet::parse (:206-216): two MACs, then EtherType / VLAN tags until a non-VLAN type,
        then the rest as payload.  -> (remainder, Ethernet); the remainder is always empty."""
        r = _Reader(data)
        dst, src = r.take(6), r.take(6)
        vlans = []
        while True:  # parse_vlan_tag (:163-204)
            t = EthernetTypeId.new(r.u16())
            if t is None:
                raise Failure("Error: MapOpt")
            if t.kind != "Vlan":
                return b"", Ethernet(dst, src, t, vlans, r.rest())  # parse_not_vlan_tag (:140-161)
            vlans.append(VlanTag(t, r.u16()))

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
        """IPv4::parse (:148-160) + parse_ipv4 (:76-146).  -> (remainder, IPv4)."""
        data = bytes(data)
        input_len = len(data)
        r = _Reader(data)
        vl = r.u8()
        if vl >> 4 != 4:
            raise Custom(f"Expected version 4, was {vl >> 4}")
        words = vl & 0x0F
        header_length = words * 4
        additional = (words - 5) * 4 if words > 5 else 0
        tos = r.u8()
        raw_length = r.u16()
        length = (raw_length - header_length) & 0xFFFF  # u16 subtraction, wrapping (:97-101)
        expected = header_length + additional + length
        ident, flags, ttl = r.u16(), r.u16(), r.u8()
        protocol = InternetProtocolId.new(r.u8())
        if protocol is None:
            raise Failure("Error: MapOpt")
        checksum = r.u16()
        src, dst = ipaddress.IPv4Address(r.take(4)), ipaddress.IPv4Address(r.take(4))
        payload = r.take(length)
        options = r.take(additional) if additional > 0 else None
        padding = r.take(input_len - expected) if input_len > expected else None
        return r.rest(), IPv4(version_and_length=vl, tos=tos, raw_length=raw_length, id=ident, flags=flags, ttl=ttl,
                              protocol=protocol, checksum=checksum, src_ip=src, dst_ip=dst, payload=payload,
                              options=options, padding=padding)

    def as_bytes(self):
        """IPv4::as_bytes (:42-74): header fields, addresses, payload, options, padding."""
        out = struct.pack(">BBHHHBBH", self.version_and_length, self.tos, self.raw_length, self.id, self.flags,
                          self.ttl, self.protocol.value(), self.checksum)
        out += self.src_ip.packed + self.dst_ip.packed + self.payload
        return out + (self.options or b"") + (self.padding or b"")


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
        """Tcp::parse (:54-101): a header length outside 20..60 is a nom Error; payload = rest."""
        r = _Reader(data)
        src, dst, seq, ack = r.u16(), r.u16(), r.u32(), r.u32()
        v = r.u16()
        hl = Tcp.extract_length(v)
        if not 20 <= hl <= 60:
            raise Failure("Error: MapRes")
        window, check, urgent = r.u16(), r.u16(), r.u16()
        options = r.take(hl - 20)
        return b"", Tcp(src_port=src, dst_port=dst, sequence_number=seq, acknowledgement_number=ack,
                        header_length_and_flags=v, header_length=hl, flags=v & 0x01FF, window=window, check=check,
                        urgent=urgent, options=options, payload=r.rest())

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
        """Udp::parse (:33-50): payload = take!(length - 8), usize wrapping.  -> (remainder, Udp)."""
        r = _Reader(data)
        src, dst = r.u16(), r.u16()
        length = (r.u16() - 8) & _U64
        checksum = r.u16()
        payload = r.take(length)
        return r.rest(), Udp(src, dst, checksum, payload)

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
