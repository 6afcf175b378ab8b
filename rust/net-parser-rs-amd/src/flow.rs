//! Flow extraction on the device (src/flow/mod.rs): the FlowExtraction trait, convert_records,
//! and a fused parse + convert_records.  Flow, Device, info and the error tree are the
//! reference's own types.
//!
//! A flow error is rebuilt from the device's per-record status code, one code per leaf of the
//! reference's error tree (include/npr.h npr_flow_status).  The variant path is exact; the
//! `size` / `msg` payloads inside it are not computed on the device (`size: None` / `0`,
//! `msg: ""`), which SURVEY.md §8 a16 leaves out of scope.
pub use net_parser_rs::flow::{device, errors, info, layer2, layer3, layer4, Flow};

use crate::common::MacAddress;
use crate::ffi;
use crate::{check, to_record, with_ctx, PcapRecord};
use device::Device;
use errors::Error;
use std::borrow::Cow;
use std::net::{IpAddr, Ipv4Addr, Ipv6Addr};

///
/// Trait that provides necessary information to indicate a flow (src/flow/mod.rs:20-42); the
/// default `extract_flow` runs the decode tree on the device.
///
pub trait FlowExtraction {
    fn payload(&self) -> &[u8];

    fn extract_flow(&self) -> Result<Flow, Error> {
        let mut v = extract_payloads(&[self.payload()], None);
        v.pop().unwrap_or_else(|| Err(Error::Incomplete { size: 0 }))
    }
}

impl<'a> FlowExtraction for PcapRecord<'a> {
    fn payload(&self) -> &[u8] {
        self.payload
    }
}

/// extract_flow for a batch of records in ONE device call (file order kept).
pub fn extract_flows<'b>(records: &[PcapRecord<'b>]) -> Vec<Result<Flow, Error>> {
    let payloads: Vec<&[u8]> = records.iter().map(|r| r.payload).collect();
    extract_payloads(&payloads, None)
}

///
/// Utility function to convert a vector of records to flows, unless an error is encountered
/// in stream conversion (src/flow/mod.rs:101-123): Ok flows in REVERSE record order.
///
pub fn convert_records<'b>(records: Vec<PcapRecord<'b>>) -> Vec<(PcapRecord<'b>, Flow)> {
    convert(records, None)
}

/// convert_records when the records borrow from `input` (e.g. CaptureFile::parse(input)): the
/// device reads the payloads from one staged copy of `input`, with no per-record gathering.
pub fn convert_records_in<'b>(input: &'b [u8], records: Vec<PcapRecord<'b>>) -> Vec<(PcapRecord<'b>, Flow)> {
    convert(records, Some(input))
}

fn convert<'b>(records: Vec<PcapRecord<'b>>, input: Option<&[u8]>) -> Vec<(PcapRecord<'b>, Flow)> {
    let payloads: Vec<&[u8]> = records.iter().map(|r| r.payload).collect();
    let res = extract_payloads(&payloads, input);
    let mut out = Vec::with_capacity(records.len());
    for (r, f) in records.into_iter().zip(res.into_iter()).rev() {
        if let Ok(f) = f {
            out.push((r, f));
        }
    }
    out
}

/// The reference's `extract` bench step (benches/benches.rs:56-62: CaptureFile::parse then
/// convert_records) fused into one device pass with the PCIe transfers pipelined
/// (npr_parse_extract_pipelined).  Returns the unparsed remainder and the (record, flow) pairs
/// in convert_records order.
pub fn parse_and_convert<'b>(input: &'b [u8]) -> Result<(&'b [u8], Vec<(PcapRecord<'b>, Flow)>), crate::Error> {
    let (_, header) = crate::GlobalHeader::parse(input)?;
    let big = header.endianness == nom::Endianness::Big;
    let (rows, rows6, consumed) = with_ctx(|ctx| {
        let cap = input.len().saturating_sub(24) / 16 + 1;
        let mut rows = vec![ffi::npr_flow::default(); cap];
        let mut rows6 = vec![ffi::npr_flow_v6::default(); cap];
        let mut hdr = ffi::npr_global_header::default();
        let (mut n, mut consumed) = (0usize, 0usize);
        let st = unsafe {
            ffi::npr_parse_extract_pipelined(
                ctx,
                input.as_ptr(),
                input.len(),
                &mut hdr,
                rows.as_mut_ptr(),
                rows6.as_mut_ptr(),
                cap,
                &mut n,
                &mut consumed,
                0,
            )
        };
        check(ctx, st)?;
        let k = n.min(cap);
        // right-aligned: rows[cap - n .. cap] in convert_records order
        rows.drain(..cap - k);
        rows6.drain(..cap - k);
        Ok((rows, rows6, consumed))
    })?;
    let rd = |b: &[u8]| {
        let a = [b[0], b[1], b[2], b[3]];
        if big {
            u32::from_be_bytes(a)
        } else {
            u32::from_le_bytes(a)
        }
    };
    let mut out = Vec::with_capacity(rows.len());
    for (f, f6) in rows.iter().zip(rows6.iter()) {
        let mut o = [0u8; 8];
        o[..5].copy_from_slice(&f.record_offset);
        let off = u64::from_le_bytes(o) as usize;
        let h = &input[off..off + 16];
        let r = ffi::npr_record {
            offset: off as u64,
            ts_sec: rd(&h[0..4]),
            ts_usec: rd(&h[4..8]),
            actual_length: rd(&h[8..12]),
            original_length: rd(&h[12..16]),
        };
        out.push((to_record(input, &r), to_flow(f, f6)));
    }
    Ok((&input[consumed..], out))
}

/// Row f3 (off the reference's flow path, which never yields a Vxlan flow): for each record, the
/// outer frame's UDP payload (to `dst_port`, 0 = any; 4789 is the IANA port) parsed as
/// `layer4::Vxlan::parse(.., endianness)` (src/layer4/vxlan.rs:31-48) and the inner Ethernet
/// frame's flow, as `<Vxlan as FlowExtraction>::extract_flow` (src/flow/layer4/vxlan.rs:32-50),
/// with the VXLAN network identifier (0 when the header was not reached).  One device call.
/// Errors: an outer failure as extract_flow's; an inner Ethernet parse failure as
/// `Error::L4(Vxlan(NetParser(..)))`; other inner failures as the inner frame's own flow error; a
/// payload shorter than the VXLAN header as `Error::NetParser(Incomplete)`; an outer flow that is
/// not UDP to `dst_port` as `Error::NetParser(Custom)`.
pub fn vxlan_flows<'b>(
    input: Option<&'b [u8]>,
    records: &[PcapRecord<'b>],
    dst_port: u16,
    endianness: nom::Endianness,
) -> Vec<(Result<Flow, Error>, u32)> {
    let payloads: Vec<&[u8]> = records.iter().map(|r| r.payload).collect();
    let n = payloads.len();
    if n == 0 {
        return Vec::new();
    }
    let (buf, recs) = stage(&payloads, input);
    let mut flows = vec![ffi::npr_flow::default(); n];
    let mut flows6 = vec![ffi::npr_flow_v6::default(); n];
    let mut status = vec![0u8; n];
    let mut vni = vec![0u32; n];
    let r = with_ctx(|ctx| {
        let st = unsafe {
            ffi::npr_vxlan_flows(
                ctx,
                buf.as_ptr(),
                buf.len(),
                recs.as_ptr(),
                n,
                dst_port as u32,
                crate::endian(endianness),
                flows.as_mut_ptr(),
                flows6.as_mut_ptr(),
                status.as_mut_ptr(),
                vni.as_mut_ptr(),
            )
        };
        check(ctx, st)
    });
    if let Err(e) = r {
        let msg = format!("{}", e);
        return (0..n).map(|_| (Err(Error::NetParser(crate::Error::Custom { msg: msg.clone() })), 0)).collect();
    }
    (0..n)
        .map(|i| {
            let st = status[i];
            let res = match st {
                0 => Ok(to_flow(&flows[i], &flows6[i])),
                ffi::NPR_VXLAN_NOT_UDP | ffi::NPR_VXLAN_PORT => Err(Error::NetParser(crate::Error::Custom {
                    msg: String::from("the outer flow is not UDP to the requested port"),
                })),
                ffi::NPR_VXLAN_INCOMPLETE => Err(Error::NetParser(crate::Error::Incomplete { size: None })),
                s if s > ffi::NPR_VXLAN_INNER => {
                    let inner = vxlan_inner(payloads[i]);
                    match s - ffi::NPR_VXLAN_INNER {
                        1 => Err(vxlan_eth_error(crate::Error::Incomplete { size: None })),
                        2 => Err(vxlan_eth_error(crate::Error::Failure { msg: String::new() })),
                        k => Err(flow_error(k, inner)),
                    }
                }
                s => Err(flow_error(s, payloads[i])),
            };
            (res, vni[i])
        })
        .collect()
}

/// Error::L4(Vxlan(NetParser(e))) (src/flow/layer4/vxlan.rs:35-38)
fn vxlan_eth_error(e: crate::Error) -> Error {
    let v: layer4::vxlan::errors::Error = layer4::vxlan::errors::Error::NetParser(e);
    let l4: layer4::errors::Error = v.into();
    Error::L4(l4)
}

/// The inner Ethernet frame of an Ok outer Ethernet / IP / UDP frame carrying VXLAN: after the
/// UDP header (8 B) and the VXLAN header (8 B); the L4 header starts 20 bytes into IPv4 (quirk Q7)
/// and after one byte per extension in IPv6 (quirk Q11).
fn vxlan_inner(p: &[u8]) -> &[u8] {
    use crate::layer2::ethernet::{EthernetTypeId, Layer3Id};
    let (et, l3) = l2_etype(p);
    let l4 = match et {
        EthernetTypeId::L3(Layer3Id::IPv6) => {
            let get = |i: usize| p.get(l3 + i).copied().unwrap_or(0);
            let mut k = 7;
            let mut id = get(6);
            while matches!(id, 0 | 43 | 44 | 50 | 51 | 60) {
                id = get(k);
                k += 1;
            }
            l3 + k + 33
        }
        _ => l3 + 20,
    };
    p.get(l4 + 16..).unwrap_or(&[])
}

// ---- device call ----------------------------------------------------------------------------
/// The buffer and record rows one device call reads: `input` itself when every payload lies
/// inside it behind its 16-byte record header, else a staged buffer of [16 header bytes | payload]...
fn stage<'a>(payloads: &[&[u8]], input: Option<&'a [u8]>) -> (Cow<'a, [u8]>, Vec<ffi::npr_record>) {
    let n = payloads.len();
    let inside = |buf: &[u8]| {
        let b = buf.as_ptr() as usize;
        payloads.iter().all(|p| {
            let a = p.as_ptr() as usize;
            a >= b + 16 && a + p.len() <= b + buf.len()
        })
    };
    match input {
        Some(buf) if inside(buf) => {
            let b = buf.as_ptr() as usize;
            let recs = payloads
                .iter()
                .map(|p| ffi::npr_record {
                    offset: (p.as_ptr() as usize - b - 16) as u64,
                    actual_length: p.len() as u32,
                    ..Default::default()
                })
                .collect();
            (Cow::Borrowed(buf), recs)
        }
        _ => {
            let total: usize = payloads.iter().map(|p| 16 + p.len()).sum();
            let mut staged = Vec::with_capacity(total);
            let mut recs = Vec::with_capacity(n);
            for p in payloads {
                recs.push(ffi::npr_record {
                    offset: staged.len() as u64,
                    actual_length: p.len() as u32,
                    ..Default::default()
                });
                staged.extend_from_slice(&[0u8; 16]);
                staged.extend_from_slice(p);
            }
            (Cow::Owned(staged), recs)
        }
    }
}

/// One npr_extract_flows call over `payloads` (read from `input` when they lie inside it).
fn extract_payloads(payloads: &[&[u8]], input: Option<&[u8]>) -> Vec<Result<Flow, Error>> {
    let n = payloads.len();
    if n == 0 {
        return Vec::new();
    }
    let (buf, recs) = stage(payloads, input);
    let mut flows = vec![ffi::npr_flow::default(); n];
    let mut flows6 = vec![ffi::npr_flow_v6::default(); n];
    let mut status = vec![0u8; n];
    let r = with_ctx(|ctx| {
        let st = unsafe {
            ffi::npr_extract_flows(
                ctx,
                buf.as_ptr(),
                buf.len(),
                recs.as_ptr(),
                n,
                flows.as_mut_ptr(),
                flows6.as_mut_ptr(),
                status.as_mut_ptr(),
            )
        };
        check(ctx, st)
    });
    if let Err(e) = r {
        let msg = format!("{}", e);
        return (0..n).map(|_| Err(Error::NetParser(crate::Error::Custom { msg: msg.clone() }))).collect();
    }
    (0..n)
        .map(|i| if status[i] == 0 { Ok(to_flow(&flows[i], &flows6[i])) } else { Err(flow_error(status[i], payloads[i])) })
        .collect()
}

/// Flow::new (src/flow/mod.rs:64-86) from a 32-byte device row (+ its IPv6 side row).
fn to_flow(f: &ffi::npr_flow, f6: &ffi::npr_flow_v6) -> Flow {
    let v6 = f.kind & ffi::NPR_FLOW_KIND_IPV6 != 0;
    let (src, dst) = if v6 {
        (IpAddr::V6(Ipv6Addr::from(f6.src_ip)), IpAddr::V6(Ipv6Addr::from(f6.dst_ip)))
    } else {
        (IpAddr::V4(Ipv4Addr::from(f.src_ip)), IpAddr::V4(Ipv4Addr::from(f.dst_ip)))
    };
    Flow {
        source: Device { mac: MacAddress(f.src_mac), ip: src, port: f.src_port },
        destination: Device { mac: MacAddress(f.dst_mac), ip: dst, port: f.dst_port },
        layer2: info::layer2::Id::Ethernet,
        layer3: if v6 { info::layer3::Id::IPv6 } else { info::layer3::Id::IPv4 },
        layer4: if f.kind & ffi::NPR_FLOW_KIND_UDP != 0 { info::layer4::Id::Udp } else { info::layer4::Id::Tcp },
        vlan: f.vlan,
    }
}

// ---- npr_flow_status -> the reference's flow error tree ------------------------------------------
/// The first EtherType after the 802.1Q/ad tags (src/layer2/ethernet.rs:163-216), as the
/// reference's EthernetTypeId: only LLDP / an 802.3 length reach flow status 3.
fn l2_etype(p: &[u8]) -> (crate::layer2::ethernet::EthernetTypeId, usize) {
    use crate::layer2::ethernet::{EthernetTypeId, Layer3Id, VlanTypeId};
    let mut pos = 12;
    loop {
        if p.len() < pos + 2 {
            return (EthernetTypeId::PayloadLength(0), pos);
        }
        let t = u16::from_be_bytes([p[pos], p[pos + 1]]);
        match t {
            0x8100 | 0x88a8 => pos += 4,
            0x88cc => return (EthernetTypeId::L3(Layer3Id::Lldp), pos + 2),
            0x0800 => return (EthernetTypeId::L3(Layer3Id::IPv4), pos + 2),
            0x86dd => return (EthernetTypeId::L3(Layer3Id::IPv6), pos + 2),
            0x0806 => return (EthernetTypeId::L3(Layer3Id::Arp), pos + 2),
            x if x <= 1500 => return (EthernetTypeId::PayloadLength(x), pos + 2),
            _ => return (EthernetTypeId::Vlan(VlanTypeId::VlanTagId), pos + 2),
        }
    }
}

/// The L3 protocol id the reference rejects at flow status 15 / 16 (src/layer3/ipv4.rs:119,
/// src/layer3/ipv6.rs:29-56: one next-header byte per extension).
fn l3_proto(p: &[u8], v6: bool) -> crate::layer3::InternetProtocolId {
    use crate::layer3::InternetProtocolId;
    let (_, l3) = l2_etype(p);
    let get = |i: usize| p.get(l3 + i).copied().unwrap_or(0);
    let mut id = if v6 { get(6) } else { get(9) };
    if v6 {
        let mut k = 7;
        while matches!(id, 0 | 43 | 44 | 50 | 51 | 60) {
            id = get(k);
            k += 1;
        }
    }
    InternetProtocolId::new(id).unwrap_or(InternetProtocolId::ICMP)
}

fn flow_error(st: u8, p: &[u8]) -> Error {
    use crate::layer2::ethernet::{EthernetTypeId as E, Layer3Id as L3};
    use crate::layer3::InternetProtocolId as P;
    use layer2::ethernet::errors::Error as Eth;
    use layer3::{arp, ipv4, ipv6};
    type NP = crate::Error;
    let inc = || NP::Incomplete { size: None };
    let fail = || NP::Failure { msg: String::new() };
    let cust = || NP::Custom { msg: String::new() };
    let eth = |e: Eth| -> Error {
        let l2: layer2::errors::Error = e.into();
        l2.into()
    };
    let l3e = |e: layer3::errors::Error| -> Error { e.into() };
    match st {
        1 => Error::NetParser(inc()),
        2 => Error::NetParser(fail()),
        3 => eth(Eth::EthernetType { etype: l2_etype(p).0 }),
        4 => eth(Eth::NetParser { l3: E::L3(L3::IPv4), err: inc() }),
        5 => eth(Eth::NetParser { l3: E::L3(L3::IPv4), err: fail() }),
        6 => eth(Eth::NetParser { l3: E::L3(L3::IPv4), err: cust() }),
        7 => eth(Eth::NetParser { l3: E::L3(L3::IPv6), err: inc() }),
        8 => eth(Eth::NetParser { l3: E::L3(L3::IPv6), err: fail() }),
        9 => eth(Eth::NetParser { l3: E::L3(L3::IPv6), err: cust() }),
        10 => eth(Eth::NetParser { l3: E::L3(L3::Arp), err: inc() }),
        11 => eth(Eth::Incomplete { l3: E::L3(L3::IPv4), size: 0 }),
        12 => eth(Eth::Incomplete { l3: E::L3(L3::IPv6), size: 0 }),
        13 => eth(Eth::Incomplete { l3: E::L3(L3::Arp), size: 0 }),
        14 => l3e(arp::errors::Error::Flow.into()),
        15 => l3e(ipv4::errors::Error::InternetProtocolId { id: l3_proto(p, false) }.into()),
        16 => l3e(ipv6::errors::Error::InternetProtocolId { id: l3_proto(p, true) }.into()),
        17 => l3e(ipv4::errors::Error::NetParser { l4: P::Tcp, err: inc() }.into()),
        18 => l3e(ipv4::errors::Error::NetParser { l4: P::Tcp, err: fail() }.into()),
        19 => l3e(ipv4::errors::Error::NetParser { l4: P::Udp, err: inc() }.into()),
        20 => l3e(ipv6::errors::Error::NetParser { l4: P::Tcp, err: inc() }.into()),
        21 => l3e(ipv6::errors::Error::NetParser { l4: P::Tcp, err: fail() }.into()),
        22 => l3e(ipv6::errors::Error::NetParser { l4: P::Udp, err: inc() }.into()),
        23 => l3e(ipv4::errors::Error::Incomplete { l4: P::Udp, size: 0 }.into()),
        24 => l3e(ipv6::errors::Error::Incomplete { l4: P::Udp, size: 0 }.into()),
        _ => Error::NetParser(NP::Custom { msg: format!("record not inside the buffer (status {})", st) }),
    }
}
