"""Generate tests/golden/kat.json: the reference's own known-answer tests as data.

Every vector below is a byte array (or Wireshark hex dump) held by a `#[test]` in
protectwise/net-parser-rs 0.3.0, together with the values that test asserts.  The reference
cannot be executed here (no Rust toolchain), so these KATs are what pins the CPU oracle
(oracle/npr_oracle.c).  `derived` entries are values the reference test does not assert but
that follow from the same bytes under the cited parse path; they are marked as such.

Run:  python tests/golden/make_golden.py   (rewrites kat.json next to this file)
"""
import json
import os
import re


def hexdump(text):
    """Bytes of a Wireshark "Hex + ASCII" dump (the format of src/lib.rs:93-104)."""
    out = bytearray()
    for line in text.strip().splitlines():
        m = re.match(r"^\s*[0-9a-fA-F]{3,}\s+((?:[0-9a-fA-F]{2}\s){1,16})", line + " ")
        if m:
            out += bytes.fromhex(m.group(1).replace(" ", ""))
    return bytes(out)


def h(s):
    return bytes.fromhex(s.replace(" ", "").replace("\n", ""))


ETH_HDR = "010203040506 FFFEFDFCFBFA"
IPV4_TCP = (
    "45 00 0048 0000 0000 64 06 0000 01020304 0A0B0C0D"
)
TCP_HDR = "C6B7 0050 00000001 00000002 5000 0000 0000 0000"
PAYLOAD32 = "01020304" + "00" * 24 + "fcfdfeff"

# src/record.rs:147-183 — big-endian record header + Ethernet/IPv4/TCP frame
RECORD_BE = h("5B116DE3 000251F5 00000056 000004D0" + ETH_HDR + "0800" + IPV4_TCP + TCP_HDR + PAYLOAD32)
# src/lib.rs:107-151 — global header with magic 4d 3c 2b 1a (=> Big) + the record above
FILE_BE = h("4d3c2b1a 0004 0002 00000000 00000004 00000613 00000002") + RECORD_BE
# src/global_header.rs:84-103 (little-endian host constants)
GH_NATIVE = h("D4C3B2A1 0400 0200 00000000 04000000 13060000 02000000")
GH_REVERSED = h("1A2B3C4D 0004 0002 00000000 00000004 00000613 00000002")
# src/layer2/ethernet.rs:223-229 / :231-261
ETH_PAYLOAD = h(ETH_HDR + "0004" + "01020304")
ETH_TCP = h(ETH_HDR + "0800" + IPV4_TCP + TCP_HDR + PAYLOAD32)
# src/layer3/ipv4.rs:167-193
IPV4_RAW = h(IPV4_TCP + TCP_HDR + PAYLOAD32)
# src/layer3/ipv6.rs:106-131
IPV6_RAW = h(
    "65 000000 0034 06 00"
    "0102030405060708090A0B0C0D0E0F0F"
    "0F000102030405060708090A0B0C0D0E" + TCP_HDR + PAYLOAD32
)
# src/layer3/arp.rs:83-94
ARP_RAW = h("0001 0800 06 04 0001 000adc6485c2 c0a85901 000000000000 c0a85902")
# src/layer4/tcp.rs:110-125
TCP_RAW = h(TCP_HDR + PAYLOAD32)
# src/layer4/udp.rs:59-68
UDP_RAW = h("C6B7 0050 0028 0000" + PAYLOAD32)
# src/layer4/vxlan.rs:66-85 (148-byte frame) and :113-122 (44-byte frame)
VXLAN_ENCAP = hexdump(
    """
            0000   08 00 27 f2 1d 8c 08 00 27 ae 4d 62 08 00 45 00  ..'.....'.Mb..E.
            0010   00 86 d9 99 40 00 40 11 6f 65 c0 a8 38 0b c0 a8  ....@.@.oe..8...
            0020   38 0c bc 06 12 b5 00 72 00 00 08 00 00 00 00 00  8......r........
            0030   7b 00 4a 7f 01 3b a2 71 ba 09 2b 6e f8 be 08 00  {.J..;.q..+n....
            0040   45 00 00 54 2f 4f 40 00 40 01 f7 57 0a 00 00 01  E..T/O@.@..W....
            0050   0a 00 00 02 08 00 4c 8a 0d 3d 00 01 a3 8c 7c 57  ......L..=....|W
            0060   00 00 00 00 b5 80 0a 00 00 00 00 00 10 11 12 13  ................
            0070   14 15 16 17 18 19 1a 1b 1c 1d 1e 1f 20 21 22 23  ............ !"#
            0080   24 25 26 27 28 29 2a 2b 2c 2d 2e 2f 30 31 32 33  $%&'()*+,-./0123
            0090   34 35 36 37                                      4567
    """
)
VXLAN_PLAIN = hexdump(
    """
            0000   00 86 9c 66 13 11 68 5b 35 b2 43 ff 08 00 45 00  ...f..h[5.C...E.
            0010   00 1e e2 7c 00 00 40 11 00 00 c0 a8 00 d8 01 01  ...|..@.........
            0020   01 01 eb f6 14 b4 00 0a c3 9d 20 0a              .......... .
    """
)
assert len(RECORD_BE) == 16 + 86 and len(FILE_BE) == 24 + 16 + 86
assert len(VXLAN_ENCAP) == 148 and len(VXLAN_PLAIN) == 44  # vxlan.rs:87, :124

KATS = [
    {"name": "global_header_native_endian", "ref": "src/global_header.rs:118-129", "api": "global_header",
     "input": GH_NATIVE.hex(),
     "expect": {"endianness": "little", "version_major": 4, "version_minor": 2, "snap_length": 1555, "rem": 0}},
    {"name": "global_header_not_native_endian", "ref": "src/global_header.rs:131-145", "api": "global_header",
     "input": GH_REVERSED.hex(),
     "expect": {"endianness": "big", "version_major": 4, "version_minor": 2, "snap_length": 1555, "rem": 0}},
    {"name": "parse_record", "ref": "src/record.rs:218-232", "api": "record", "endianness": "big",
     "input": RECORD_BE.hex(),
     "expect": {"ts_sec": 1527868899, "ts_usec": 152053, "actual_length": 86, "original_length": 1232, "rem": 0}},
    {"name": "display_record", "ref": "src/record.rs:185-196", "api": "record_display", "endianness": "big",
     "input": RECORD_BE.hex(),
     "expect": {"display": "Timestamp=1527868899152   Length=86   Original Length=1232"}},
    {"name": "convert_timestamp", "ref": "src/record.rs:198-207", "api": "timestamp",
     "input": "", "expect": {"ts_sec": 1527868899, "ts_usec": 152053, "timestamp_ns": 1527868899152053000}},
    {"name": "convert_record", "ref": "src/record.rs:234-238", "api": "record_flow", "endianness": "big",
     "input": RECORD_BE.hex(),
     "expect": {"status": 0, "src_port": 50871, "dst_port": 80},
     "derived": {"src_ip": "1.2.3.4", "dst_ip": "10.11.12.13", "src_mac": "ff:fe:fd:fc:fb:fa",
                 "dst_mac": "01:02:03:04:05:06", "vlan": 0, "layer3": "IPv4", "layer4": "Tcp"}},
    {"name": "file_bytes_parse", "ref": "src/lib.rs:153-165", "api": "file",
     "input": FILE_BE.hex(),
     "expect": {"endianness": "big", "n_records": 1, "rem": 0},
     "derived": {"record_offsets": [24], "actual_lengths": [86]}},
    {"name": "convert_packet", "ref": "src/lib.rs:167-180", "api": "file_flows",
     "input": FILE_BE.hex(),
     "expect": {"n_flows": 1, "src_port": 50871, "dst_port": 80}},
    {"name": "parse_ethernet_payload", "ref": "src/layer2/ethernet.rs:263-289", "api": "ethernet",
     "input": ETH_PAYLOAD.hex(),
     "expect": {"dst_mac": "01:02:03:04:05:06", "src_mac": "ff:fe:fd:fc:fb:fa", "n_vlans": 0,
                "ether_type": "payload_length", "rem": 0},
     "derived": {"flow_status": "L2_ETHERTYPE"}},
    {"name": "parse_ethernet_tcp", "ref": "src/layer2/ethernet.rs:291-315", "api": "ethernet",
     "input": ETH_TCP.hex(),
     "expect": {"dst_mac": "01:02:03:04:05:06", "src_mac": "ff:fe:fd:fc:fb:fa", "n_vlans": 0,
                "ether_type": "ipv4", "rem": 0}},
    {"name": "convert_ethernet_tcp", "ref": "src/flow/layer2/ethernet.rs:143-156", "api": "flow",
     "input": ETH_TCP.hex(),
     "expect": {"status": 0, "layer2": "Ethernet", "src_port": 50871, "dst_port": 80}},
    {"name": "parse_ipv4", "ref": "src/layer3/ipv4.rs:195-224", "api": "ipv4",
     "input": IPV4_RAW.hex(),
     "expect": {"src_ip": "1.2.3.4", "dst_ip": "10.11.12.13", "protocol": 6, "rem": 0}},
    {"name": "convert_ipv4", "ref": "src/flow/layer3/ipv4.rs:115-145", "api": "ipv4_flow",
     "input": IPV4_RAW.hex(),
     "expect": {"layer3": "IPv4", "src_ip": "1.2.3.4", "dst_ip": "10.11.12.13", "src_port": 50871, "dst_port": 80}},
    {"name": "parse_ipv6", "ref": "src/layer3/ipv6.rs:133-161", "api": "ipv6",
     "input": IPV6_RAW.hex(),
     "expect": {"src_ip": "0102:0304:0506:0708:090a:0b0c:0d0e:0f0f", "dst_ip": "0f00:0102:0304:0506:0708:090a:0b0c:0d0e",
                "protocol": 6, "rem": 0}},
    {"name": "convert_ipv6", "ref": "src/flow/layer3/ipv6.rs:114-144", "api": "ipv6_flow",
     "input": IPV6_RAW.hex(),
     "expect": {"layer3": "IPv6", "src_ip": "0102:0304:0506:0708:090a:0b0c:0d0e:0f0f",
                "dst_ip": "0f00:0102:0304:0506:0708:090a:0b0c:0d0e", "src_port": 50871, "dst_port": 80}},
    {"name": "parse_arp", "ref": "src/layer3/arp.rs:96-122", "api": "arp",
     "input": ARP_RAW.hex(),
     "expect": {"sender_ip": "192.168.89.1", "sender_mac": "00:0a:dc:64:85:c2", "target_ip": "192.168.89.2",
                "target_mac": "00:00:00:00:00:00", "operation": 1, "rem": 0}},
    {"name": "convert_length", "ref": "src/layer4/tcp.rs:127-131", "api": "tcp_length",
     "input": "", "expect": {"0x0000": 0, "0x3000": 12}},
    {"name": "parse_tcp", "ref": "src/layer4/tcp.rs:133-156", "api": "tcp",
     "input": TCP_RAW.hex(),
     "expect": {"src_port": 50871, "dst_port": 80, "payload": PAYLOAD32.lower(), "rem": 0}},
    {"name": "convert_tcp", "ref": "src/flow/layer4/tcp.rs:48-76", "api": "tcp",
     "input": TCP_RAW.hex(),
     "expect": {"src_port": 50871, "dst_port": 80, "layer4": "Tcp"}},
    {"name": "parse_udp", "ref": "src/layer4/udp.rs:70-93", "api": "udp",
     "input": UDP_RAW.hex(),
     "expect": {"src_port": 50871, "dst_port": 80, "payload": PAYLOAD32.lower(), "rem": 0}},
    {"name": "convert_udp", "ref": "src/flow/layer4/udp.rs:48-76", "api": "udp",
     "input": UDP_RAW.hex(),
     "expect": {"src_port": 50871, "dst_port": 80, "layer4": "Udp"}},
    {"name": "encapsulated", "ref": "src/layer4/vxlan.rs:63-104", "api": "frame_layers",
     "input": VXLAN_ENCAP.hex(),
     "expect": {"dst_mac": "08:00:27:f2:1d:8c", "dst_ip": "192.168.56.12", "udp_dst_port": 4789,
                # Vxlan::parse(udp.payload, Big) (:91-101): no remainder, flags, VNI, as_bytes
                # round trip, then the inner Ethernet / IPv4 (:99-103)
                "vxlan": {"ok": True, "remainder": 0, "flags": 0x0800, "network_identifier": 123,
                          "as_bytes_is_udp_payload": True, "inner_dst_mac": "4a:7f:01:3b:a2:71",
                          "inner_dst_ip": "10.0.0.2"}},
     "derived": {"flow_status": 0, "src_ip": "192.168.56.11", "src_port": 48134, "layer4": "Udp",
                 # the inner frame is ICMP: its Ethernet flow is Err(L3 IPv4 protocol)
                 "vxlan_inner_flow_status": 15}},
    {"name": "not_encapsulated", "ref": "src/layer4/vxlan.rs:106-137", "api": "frame_layers",
     "input": VXLAN_PLAIN.hex(),
     "expect": {"dst_mac": "00:86:9c:66:13:11", "dst_ip": "1.1.1.1", "udp_dst_port": 5300,
                "vxlan": {"ok": False}},  # Vxlan::parse is Err on the 2-byte payload (:134-135)
     "derived": {"flow_status": 0, "src_ip": "192.168.0.216", "src_port": 60406, "layer4": "Udp"}},
    {"name": "format_flow", "ref": "src/flow/mod.rs:136-156", "api": "display_flow", "input": "",
     "flow": {"src_mac": "00:01:02:03:04:05", "src_ip": "0.1.2.3", "src_port": 80,
              "dst_mac": "0b:0a:09:08:07:06", "dst_ip": "100.99.98.97", "dst_port": 52436, "vlan": 0},
     "expect": {"display": "Source=[Mac=00:01:02:03:04:05   Ip=0.1.2.3   Port=80]   Destination=[Mac=0b:0a:09:08:07:06   Ip=100.99.98.97   Port=52436]   Vlan=0"}},
    {"name": "format_device", "ref": "src/flow/device.rs:33-45", "api": "display_device", "input": "",
     "device": {"mac": "00:01:02:03:04:05", "ip": "0.1.2.3", "port": 80},
     "expect": {"display": "Mac=00:01:02:03:04:05   Ip=0.1.2.3   Port=80"}},
    {"name": "format_mac_address", "ref": "src/common.rs:32-37", "api": "display_mac", "input": "000102030405",
     "expect": {"display": "00:01:02:03:04:05"}},
    {"name": "test_hex_dump", "ref": "src/lib.rs:59-66", "api": "hexdump", "input": "34353637",
     "expect": {"len": 4}},
    {"name": "file_parse", "ref": "src/lib.rs:182-202", "api": "blob", "input": "",
     "blob": "resources/4SICS-GeekLounge-151020.pcap",
     "expect": {"endianness": "little", "n_records": 246137}},
    {"name": "file_convert", "ref": "src/flow/mod.rs:158-183", "api": "blob", "input": "",
     "blob": "resources/4SICS-GeekLounge-151020.pcap",
     "expect": {"endianness": "little", "n_records": 246137, "n_flows": 236527}},
]


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")
    with open(path, "w") as f:
        json.dump({"source": "protectwise/net-parser-rs 0.3.0 #[test] vectors", "kats": KATS}, f, indent=1)
        f.write("\n")
    print(f"wrote {len(KATS)} KATs to {path}")


if __name__ == "__main__":
    main()
