"""Row f3: VXLAN (src/layer4/vxlan.rs:31-48) and its inner flow (src/flow/layer4/vxlan.rs:32-50).

CPU: the oracle and the Python mirror against the reference's own VXLAN tests (the two frames of
src/layer4/vxlan.rs:63-138, tests/golden/kat.json).  GPU: npr_dev_vxlan_flows / npr_vxlan_flows
bit-exact against the oracle on a synthetic VXLAN corpus (valid inner TCP/UDP over IPv4/IPv6,
inner frames from the quirk generator, truncated VXLAN headers, other ports, IPv6 underlays).
"""
import json
import os

import numpy as np
import pytest

import _oracle
import net_parser_rs as npr
from net_parser_rs import _abi, flow, synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KATS = {k["name"]: k for k in json.load(open(os.path.join(REPO, "tests", "golden", "kat.json")))["kats"]}
UDP_PAYLOAD = 14 + 20 + 8  # both KAT frames: untagged Ethernet / IPv4 IHL 5 / UDP


def kat_pcap(names):
    """The KAT frames as one capture (records in the given order)."""
    import struct
    out = synth.global_header()
    for i, nm in enumerate(names):
        f = bytes.fromhex(KATS[nm]["input"])
        out += struct.pack("<IIII", 1, i, len(f), len(f)) + f
    return out


def test_oracle_vxlan_kat():
    k = KATS["encapsulated"]
    b = bytes.fromhex(k["input"])
    x = k["expect"]["vxlan"]
    rc, v = _oracle.vxlan_parse(b[UDP_PAYLOAD:], big=True)
    assert rc == 0 and v.flags == x["flags"] and v.network_identifier == x["network_identifier"]
    assert v.payload_off == 8 and len(b) - UDP_PAYLOAD - 8 > 0
    inner = b[UDP_PAYLOAD + 8:]  # Ethernet::parse(vxlan.payload), IPv4::parse(enet2.payload) (:99-103)
    assert ":".join(f"{c:02x}" for c in inner[:6]) == x["inner_dst_mac"]
    assert ".".join(str(c) for c in inner[14 + 16:14 + 20]) == x["inner_dst_ip"]
    assert _oracle.extract_flow(inner)[0] == k["derived"]["vxlan_inner_flow_status"]  # ICMP: no flow
    rc, _ = _oracle.vxlan_parse(bytes.fromhex(KATS["not_encapsulated"]["input"])[UDP_PAYLOAD:], big=True)
    assert rc != 0  # Incomplete: 2-byte UDP payload (src/layer4/vxlan.rs:134-135)


def test_mirror_vxlan_kat():
    b = bytes.fromhex(KATS["encapsulated"]["input"])
    rem, v = flow.Vxlan.parse(b[UDP_PAYLOAD:], npr.Endianness.Big)
    x = KATS["encapsulated"]["expect"]["vxlan"]
    assert len(rem) == x["remainder"] and v.flags == x["flags"] and v.network_identifier == x["network_identifier"]
    assert v.as_bytes() == b[UDP_PAYLOAD:]  # as_bytes round trip (:98)
    with pytest.raises(npr.Incomplete):
        flow.Vxlan.parse(bytes.fromhex(KATS["not_encapsulated"]["input"])[UDP_PAYLOAD:], npr.Endianness.Big)


def test_oracle_vxlan_flow_statuses():
    blob = kat_pcap(["encapsulated", "not_encapsulated", "convert_ethernet_tcp"])
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    assert rc == 0 and len(recs) == 3
    _, _, st, vni = _oracle.vxlan_flows(blob, recs, dst_port=_abi.VXLAN_PORT_IANA)
    # inner ICMP -> Err(L3 IPv4 protocol); port 5300; outer TCP
    assert list(st) == [_abi.VXLAN_INNER + KATS["encapsulated"]["derived"]["vxlan_inner_flow_status"],
                        _abi.VXLAN_PORT, _abi.VXLAN_NOT_UDP]
    assert list(vni) == [123, 0, 0]
    _, _, st0, _ = _oracle.vxlan_flows(blob, recs, dst_port=0)
    assert st0[1] == _abi.VXLAN_INCOMPLETE


def test_oracle_vxlan_corpus_has_every_class():
    blob = synth.vxlan_corpus(4000)
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    f, v6, st, vni = _oracle.vxlan_flows(blob, recs, dst_port=_abi.VXLAN_PORT_IANA)
    codes = set(int(c) for c in st)
    assert {0, _abi.VXLAN_NOT_UDP, _abi.VXLAN_PORT, _abi.VXLAN_INCOMPLETE} <= codes
    assert any(c > _abi.VXLAN_INNER for c in codes)
    ok = st == 0
    assert (f["kind"][ok] & _abi.KIND_IPV6).any() and (f["kind"][ok] & _abi.KIND_UDP).any()


# ---- device ---------------------------------------------------------------------------------
def _check_device(blob, dst_port, big):
    import torch
    from net_parser_rs import device
    rc, hdr, recs, cons = _oracle.capture_file_parse(blob)
    want = _oracle.vxlan_flows(blob, recs, dst_port=dst_port, big=big)
    buf = torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).cuda()
    drecs = torch.from_numpy(recs.view(np.uint8).copy()).cuda()
    got = device.dev_vxlan_flows(buf, drecs, dst_port=dst_port, big=big)
    torch.cuda.synchronize()
    n = len(recs)
    assert np.array_equal(got[2][:n].cpu().numpy(), want[2])
    assert np.array_equal(got[3][: 4 * n].cpu().numpy().view(np.uint32), want[3])
    assert got[0][: 32 * n].cpu().numpy().tobytes() == want[0].tobytes()
    assert got[1][: 32 * n].cpu().numpy().tobytes() == want[1].tobytes()
    return want


@pytest.mark.gpu
@pytest.mark.parametrize("dst_port", [0, 4789])
@pytest.mark.parametrize("big", [True, False])
def test_device_vxlan_corpus(dst_port, big):
    want = _check_device(synth.vxlan_corpus(20_000), dst_port, big)
    assert (want[2] == 0).sum() > 1000


@pytest.mark.gpu
def test_device_vxlan_kats_and_host_api():
    blob = kat_pcap(["encapsulated", "not_encapsulated", "convert_ethernet_tcp", "encapsulated"])
    _check_device(blob, _abi.VXLAN_PORT_IANA, True)
    rem, f = npr.parse(blob)
    out = flow.vxlan_flows(f.records.into_inner(), dst_port=_abi.VXLAN_PORT_IANA)
    codes = [o[1].code if isinstance(o[1], flow.FlowError) else 0 for o in out]
    assert codes == [_abi.VXLAN_INNER + 15, _abi.VXLAN_PORT, _abi.VXLAN_NOT_UDP, _abi.VXLAN_INNER + 15]
    assert [o[2] for o in out] == [123, 0, 0, 123]
    # a corpus through the host entry point: inner flows equal the oracle's
    blob = synth.vxlan_corpus(3000, seed=5)
    rem, f = npr.parse(blob)
    recs = f.records.into_inner()
    got = flow.vxlan_flows(recs, dst_port=0)
    rc, hdr, orecs, cons = _oracle.capture_file_parse(blob)
    wf, wv6, wst, wvni = _oracle.vxlan_flows(blob, orecs, dst_port=0)
    for i, (r, fl, vni) in enumerate(got):
        assert vni == wvni[i]
        if wst[i] == 0:
            assert fl == flow.Flow._from_row(wf[i], wv6[i]) and fl.record_offset == r.offset
        else:
            assert isinstance(fl, flow.FlowError) and fl.code == wst[i]
