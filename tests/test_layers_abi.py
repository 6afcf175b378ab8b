"""Row f2: libnpr's host-side per-layer parsers (npr_ethernet_parse, npr_ipv4_parse, npr_ipv6_parse,
npr_arp_parse, npr_tcp_parse, npr_udp_parse, npr_vxlan_parse; csrc/npr_layers.hip), on the CPU.

Pinned two ways:
- the reference's own KAT frames for IPv6 and ARP (src/layer3/ipv6.rs:133-161, src/layer3/arp.rs:96-122,
  tests/golden/kat.json; tests/test_layers.py covers the Ethernet / IPv4 / TCP / UDP ones);
- composed layer by layer as src/flow/layer{2,3,4}/*.rs compose them (Ethernet -> IPv4 | IPv6 | ARP ->
  TCP | UDP, with the flow-level remainder checks), every frame of the quirk corpora and of random
  byte strings gives the oracle's extract_flow result: the same flow, or the same error status and
  payload (npr.h npr_flow_details: Needed::Size, the map_opt! / map_res! input range, the version
  nibble, the remainder length)."""
import ctypes
import json
import os
import struct

import numpy as np
import pytest

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, layers, synth

KATS = {k["name"]: k for k in json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat.json")))["kats"]}
LIB = _abi.load_library()


def call(name, data, out, *mid):
    arr = (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0")
    used, det = ctypes.c_size_t(0), ctypes.c_uint64(0)
    st = getattr(LIB, name)(ctypes.addressof(arr), len(data), ctypes.byref(out), *mid, ctypes.byref(used),
                            ctypes.byref(det))
    return st, used.value, det.value


def test_ipv6_kat():
    raw, want = bytes.fromhex(KATS["parse_ipv6"]["input"]), KATS["parse_ipv6"]["expect"]
    rem, l3 = layers.IPv6.parse(raw)
    assert (l3.src_ip.exploded, l3.dst_ip.exploded, l3.protocol.value(), len(rem)) == \
        (want["src_ip"], want["dst_ip"], want["protocol"], want["rem"])


def test_arp_kat():
    raw, want = bytes.fromhex(KATS["parse_arp"]["input"]), KATS["parse_arp"]["expect"]
    rem, a = layers.Arp.parse(raw)
    assert (str(a.sender_ip), str(a.sender_mac), str(a.target_ip), str(a.target_mac), a.operation, len(rem)) == \
        (want["sender_ip"], want["sender_mac"], want["target_ip"], want["target_mac"], want["operation"], want["rem"])


def test_errors_carry_the_references_payloads():
    with pytest.raises(npr.Failure) as e:  # nom's Context::Code(<input at the EtherType>, MapOpt)
        layers.Ethernet.parse(bytes(12) + b"\x12\x34\x56")
    assert str(e.value) == "Error: Code([18, 52, 86], MapOpt)"
    with pytest.raises(npr.Custom) as e:
        layers.IPv6.parse(b"\x45" + bytes(60))
    assert str(e.value) == "Expected version 6, version was 4"
    with pytest.raises(npr.Incomplete) as e:  # the hop limit byte after a chain of extension bytes
        layers.IPv6.parse(b"\x60\x00\x00\x00\x00\x08\x00\x2b\x3c")
    assert e.value.size == 1
    with pytest.raises(npr.Failure):  # an unknown id inside the extension chain
        layers.IPv6.parse(b"\x60\x00\x00\x00\x00\x08\x00\x2b\x63" + bytes(40))
    with pytest.raises(npr.Incomplete) as e:
        layers.Arp.parse(bytes(27))
    assert e.value.size == 4
    with pytest.raises(npr.Incomplete) as e:  # u32! needs 4
        npr.flow.Vxlan.parse(bytes(6), npr.Endianness.Little)
    assert e.value.size == 4
    rem, v = npr.flow.Vxlan.parse(bytes.fromhex("0008000000007b00") + b"x", npr.Endianness.Little)
    assert (v.flags, v.raw_network_identifier, v.network_identifier, v.payload) == (0x800, 0x007B0000, 0x7B00, b"x")


def test_ethernet_vlan_capacity_contract():
    frame = bytes(12) + b"\x81\x00\x00\x01" * 11 + b"\x08\x00" + b"rest"
    out, tags = _abi.EthernetC(), (_abi.VlanTagC * 4)()
    st, used, _ = call("npr_ethernet_parse", frame, out, ctypes.addressof(tags), 4)
    assert st == -3 and out.n_vlans == 11 and [t.id for t in tags] == [1] * 4  # NPR_ERR_CAPACITY, exact count
    rem, e = layers.Ethernet.parse(frame)
    assert len(e.vlans) == 11 and e.payload == b"rest" and e.as_bytes() == frame


# ---- the flow, composed from the layer objects (src/flow/layer2/ethernet.rs:39-133,
#      src/flow/layer3/{ipv4,ipv6,arp}.rs, src/flow/layer4/{tcp,udp}.rs) ---------------------------
def shift(det, off):  # a Failure's input range, moved from the layer's input to the frame
    return ((det & 0xFFFFFFFF) + off) | (((det >> 32) + off) << 32)


def l4_flow(ip_payload, off, proto, codes):
    inc, fail, udp_inc, udp_rem, proto_code = codes
    if proto == 6:
        t = _abi.TcpC()
        st, used, det = call("npr_tcp_parse", ip_payload, t)
        if st == _abi.INCOMPLETE:
            return inc, det, None
        if st == _abi.FAILURE:
            return fail, shift(det, off), None
        return 0, 0, (t.src_port, t.dst_port, 0)
    if proto == 17:
        u = _abi.UdpC()
        st, used, det = call("npr_udp_parse", ip_payload, u)
        if st == _abi.INCOMPLETE:
            return udp_inc, det, None
        if used < len(ip_payload):
            return udp_rem, len(ip_payload) - used, None
        return 0, 0, (u.src_port, u.dst_port, 2)  # npr.h NPR_FLOW_KIND_UDP
    return proto_code, proto, None


def composed_flow(frame):
    """(status, detail, flow fields or None) as the reference's extract_flow composes the layers."""
    e, tags = _abi.EthernetC(), (_abi.VlanTagC * 64)()
    st, used, det = call("npr_ethernet_parse", frame, e, ctypes.addressof(tags), 64)
    if st == _abi.INCOMPLETE:
        return 1, det, None
    if st == _abi.FAILURE:
        return 2, det, None
    assert st == _abi.OK
    vlan = tags[0].id if e.n_vlans else 0
    t, off = e.ether_type, e.payload_offset
    pay = frame[off:off + e.payload_length]
    macs = (bytes(e.src_mac), bytes(e.dst_mac), vlan)
    if t == 0x0800:
        o = _abi.IPv4C()
        st, used, det = call("npr_ipv4_parse", pay, o)
        if st != _abi.OK:
            return {1: 4, 2: 5, 3: 6}[st], shift(det, off) if st == 2 else det, None
        if used < len(pay):
            return 11, len(pay) - used, None
        ipo = off + o.payload_offset
        s, d, ports = l4_flow(frame[ipo:ipo + o.payload_length], ipo, o.protocol, (17, 18, 19, 23, 15))
        return s, d, None if ports is None else (macs, (bytes(o.src_ip), bytes(o.dst_ip)), ports)
    if t == 0x86DD:
        o = _abi.IPv6C()
        st, used, det = call("npr_ipv6_parse", pay, o)
        if st != _abi.OK:
            return {1: 7, 2: 8, 3: 9}[st], shift(det, off) if st == 2 else det, None
        if used < len(pay):
            return 12, len(pay) - used, None
        ipo = off + o.payload_offset
        s, d, ports = l4_flow(frame[ipo:ipo + o.payload_length], ipo, o.protocol, (20, 21, 22, 24, 16))
        return s, d, None if ports is None else (macs, (bytes(o.src_ip), bytes(o.dst_ip)), ports)
    if t == 0x0806:
        a = _abi.ArpC()
        st, used, det = call("npr_arp_parse", pay, a)
        if st == _abi.INCOMPLETE:
            return 10, det, None
        if used < len(pay):
            return 13, len(pay) - used, None
        return 14, 0, None
    return 3, t, None  # LLDP or an 802.3 length


def check_corpus(blob):
    rc, hdr, recs, _ = _oracle.capture_file_parse(blob)
    assert rc == 0 and len(recs)
    st, det = _oracle.flow_details(blob, recs)
    flows, v6, _ = _oracle.extract_flows(blob, recs)
    for i, r in enumerate(recs):
        o = int(r["offset"]) + 16
        frame = blob[o:o + int(r["actual_length"])]
        s, d, f = composed_flow(frame)
        assert (s, d) == (int(st[i]), int(det[i])), (i, s, d, int(st[i]), int(det[i]))
        if s == 0:
            (smac, dmac, vlan), (sip, dip), (sp, dp, kind) = f
            want = flows[i]
            assert (bytes(want["src_mac"]), bytes(want["dst_mac"]), int(want["vlan"])) == (smac, dmac, vlan), i
            assert (int(want["src_port"]), int(want["dst_port"])) == (sp, dp), i
            if int(want["kind"]) & 1:  # IPv6: the addresses live in the side row
                assert (bytes(v6[i]["src_ip"]), bytes(v6[i]["dst_ip"])) == (sip, dip), i
            else:
                assert (bytes(want["src_ip"]), bytes(want["dst_ip"])) == (sip, dip), i
            assert int(want["kind"]) & 2 == kind, i


@pytest.mark.parametrize("seed", [3, 17, 99])
def test_composed_layers_match_the_oracle_flows_quirk_corpus(seed):
    check_corpus(synth.quirk_corpus(2500, seed=seed))


def test_composed_layers_match_the_oracle_flows_random_frames():
    rng = np.random.default_rng(5)
    recs = []
    for i in range(3000):
        n = int(rng.integers(0, 120))
        frame = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        if n >= 14 and i % 2:  # steer half of them past the EtherType into the L3 / L4 parsers
            frame[12:14] = [(0x08, 0x00), (0x86, 0xDD), (0x08, 0x06), (0x81, 0x00)][i % 4]
            if n > 14:
                frame[14] = (0x45, 0x60, 0x00, 0x08)[i % 4] | (frame[14] & 0x0F if i % 4 == 0 else 0)
            if n > 23 and i % 4 == 0:
                frame[23] = (6, 17)[(i // 4) % 2]
        recs.append(bytes(frame))
    body = b"".join(struct.pack("<IIII", 1_600_000_000, 0, len(f), len(f)) + f for f in recs)
    check_corpus(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, 1) + body)
