"""Row f3: the per-layer header objects and their as_bytes serializers (net_parser_rs.layers), on
the CPU.  Pinned by the reference's own tests: the KAT frames of src/layer2/ethernet.rs:263-315,
src/layer3/ipv4.rs:195-224, src/layer4/tcp.rs:133-156 and src/layer4/udp.rs:70-93 (tests/golden/
kat.json) parse to the expected fields and `as_bytes` gives the input back, as those tests assert
(ethernet.rs:287 and :314, ipv4.rs:223, tcp.rs:155, udp.rs:92).  The quirk cases (VLAN prio / dei,
wrapping IPv4 / UDP lengths, error kinds) restate the cited reference lines; no reference vector
covers them (parity unpinned there)."""
import json
import os
import struct

import pytest

import net_parser_rs as npr
from net_parser_rs import layers

KATS = {k["name"]: k for k in json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))["kats"]}


def kat_bytes(name):
    return bytes.fromhex(KATS[name]["input"])


@pytest.mark.parametrize("name,kind", [("parse_ethernet_payload", "PayloadLength"), ("parse_ethernet_tcp", "L3")])
def test_ethernet_kat_and_round_trip(name, kind):
    raw, want = kat_bytes(name), KATS[name]["expect"]
    rem, l2 = layers.Ethernet.parse(raw)
    assert len(rem) == want["rem"] and str(l2.dst_mac) == want["dst_mac"] and str(l2.src_mac) == want["src_mac"]
    assert len(l2.vlans) == want["n_vlans"] and l2.ether_type.kind == kind
    assert l2.as_bytes() == raw


def test_ipv4_kat_and_round_trip():
    raw, want = kat_bytes("parse_ipv4"), KATS["parse_ipv4"]["expect"]
    rem, l3 = layers.IPv4.parse(raw)
    assert len(rem) == want["rem"] and str(l3.src_ip) == want["src_ip"] and str(l3.dst_ip) == want["dst_ip"]
    assert l3.protocol.value() == want["protocol"]
    assert l3.as_bytes() == raw


def test_tcp_kat_and_round_trip():
    raw, want = kat_bytes("parse_tcp"), KATS["parse_tcp"]["expect"]
    rem, l4 = layers.Tcp.parse(raw)
    assert (l4.src_port, l4.dst_port, l4.payload.hex(), len(rem)) == \
        (want["src_port"], want["dst_port"], want["payload"], want["rem"])
    assert l4.as_bytes() == raw and layers.Layer4(l4).as_bytes() == raw


def test_udp_kat_and_round_trip():
    raw, want = kat_bytes("parse_udp"), KATS["parse_udp"]["expect"]
    rem, l4 = layers.Udp.parse(raw)
    assert (l4.src_port, l4.dst_port, l4.payload.hex(), len(rem)) == \
        (want["src_port"], want["dst_port"], want["payload"], want["rem"])
    assert l4.as_bytes() == raw and layers.Layer4(l4).as_bytes() == raw


def test_vxlan_through_layer4():
    rem, v = npr.flow.Vxlan.parse(bytes.fromhex("08000000007b0000") + b"inner", npr.Endianness.Big)
    assert layers.Layer4(v).as_bytes() == bytes.fromhex("08000000007b0000") + b"inner"


def test_ethernet_vlan_stack_round_trip():
    """Two tags (802.1ad then 802.1Q): ids from the low 12 bits, prio / dei always 0
    (`(total & 0x7000) as u8`, ethernet.rs:181-186), vlan() = the first tag's id."""
    frame = bytes(range(12)) + struct.pack(">HHHHH", 0x88A8, 0xE123, 0x8100, 0x2456, 0x0800) + b"\x45payload"
    rem, l2 = layers.Ethernet.parse(frame)
    assert [v.id for v in l2.vlans] == [0x123, 0x456] and l2.vlan() == 0x123
    assert all(v.prio == 0 and v.dei == 0 for v in l2.vlans)
    assert l2.ether_type.name == "IPv4" and l2.payload == b"\x45payload" and l2.as_bytes() == frame


def test_ethernet_errors():
    with pytest.raises(npr.Incomplete) as e:
        layers.Ethernet.parse(bytes(10))
    assert e.value.size == 6
    with pytest.raises(npr.Incomplete):
        layers.Ethernet.parse(bytes(12) + b"\x81\x00\x00")  # a VLAN tag cut short
    with pytest.raises(npr.Failure):
        layers.Ethernet.parse(bytes(12) + b"\x12\x34")  # above 1500 and not a known type


def test_ipv4_quirks():
    """IHL 6: the payload (total_length - 24, u16 wrapping) comes right after the 20-byte header,
    then 4 option bytes, then padding; as_bytes writes the same order back (ipv4.rs:42-74)."""
    hdr = struct.pack(">BBHHHBBH4s4s", 0x46, 0, 24 + 8, 1, 0, 64, 17, 0, b"\x01\x02\x03\x04", b"\x05\x06\x07\x08")
    raw = hdr + b"PAYLOAD!" + b"OPTS" + b"pad"
    rem, l3 = layers.IPv4.parse(raw)
    assert (l3.payload, l3.options, l3.padding, rem) == (b"PAYLOAD!", b"OPTS", None, b"pad")
    # total_length below the header length wraps: asks for ~64 KB of payload
    short = struct.pack(">BBHHHBBH4s4s", 0x45, 0, 10, 0, 0, 64, 6, 0, bytes(4), bytes(4))
    with pytest.raises(npr.Incomplete) as e:
        layers.IPv4.parse(short + bytes(8))
    assert e.value.size == (10 - 20) & 0xFFFF
    with pytest.raises(npr.Custom):
        layers.IPv4.parse(b"\x60" + bytes(39))
    with pytest.raises(npr.Failure):
        layers.IPv4.parse(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20, 0, 0, 64, 99, 0, bytes(4), bytes(4)))


def test_l4_quirks():
    with pytest.raises(npr.Failure):  # data offset 4 words: below 20 bytes
        layers.Tcp.parse(struct.pack(">HHIIHHHH", 1, 2, 3, 4, 0x4000, 0, 0, 0))
    rem, t = layers.Tcp.parse(struct.pack(">HHIIHHHH", 1, 2, 3, 4, 0x6012, 5, 6, 7) + b"OPTNdata")
    assert (t.header_length, t.flags, t.options, t.payload) == (24, 0x12, b"OPTN", b"data")
    assert t.as_bytes() == struct.pack(">HHIIHHHH", 1, 2, 3, 4, 0x6012, 5, 6, 7) + b"OPTNdata"
    with pytest.raises(npr.Incomplete) as e:  # UDP length below 8: usize wrap (udp.rs:40)
        layers.Udp.parse(struct.pack(">HHHH", 1, 2, 4, 0))
    assert e.value.size == (4 - 8) & ((1 << 64) - 1)
    rem, u = layers.Udp.parse(struct.pack(">HHHH", 1, 2, 12, 9) + b"abcdEXTRA")
    assert (u.payload, rem) == (b"abcd", b"EXTRA")
