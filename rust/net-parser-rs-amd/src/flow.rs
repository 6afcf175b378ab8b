//! Flow extraction on the device (src/flow/mod.rs): the FlowExtraction trait, convert_records, and
//! a fused parse + convert_records.  Flow, Device, info and the error tree are this crate's
//! restatements of the reference's types (types.rs).
//!
//! A flow error is rebuilt from the device's per-record status code (one code per leaf of the
//! reference's error tree, include/npr.h npr_flow_status) and the payload its variant carries
//! (npr_flow_details: nom's Needed sizes, the bytes a layer left over, the failing primitive's
//! input, the version, EtherType or protocol id), so `Debug`, `Display` and the `size` fields
//! compare equal to the reference's.
pub use crate::types::flow_types::{device, errors, info, layer2, layer3, layer4};

use crate::common::MacAddress;
use crate::ffi;
use crate::{check, to_record, with_ctx, PcapRecord};
use device::Device;
use errors::Error;
use std::borrow::Cow;
use std::net::{IpAddr, Ipv4Addr, Ipv6Addr};

///
/// Flow that was built from a record moved (src/flow/mod.rs:50-96)
///
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq, Hash)]
pub struct Flow {
    pub source: Device,
    pub destination: Device,
    pub layer2: info::layer2::Id,
    pub layer3: info::layer3::Id,
    pub layer4: info::layer4::Id,
    pub vlan: crate::common::Vlan,
}

impl Flow {
    pub fn new(l2: info::layer2::Info, l3: info::layer3::Info, l4: info::layer4::Info) -> Flow {
        Flow {
            source: Device { mac: l2.src_mac, ip: l3.src_ip, port: l4.src_port },
            destination: Device { mac: l2.dst_mac, ip: l3.dst_ip, port: l4.dst_port },
            layer2: l2.id,
            layer3: l3.id,
            layer4: l4.id,
            vlan: l2.vlan,
        }
    }
}

impl std::fmt::Display for Flow {
    fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
        write!(f, "Source=[{}]   Destination=[{}]   Vlan={}", self.source, self.destination, self.vlan)
    }
}

///
/// Trait that provides necessary information to indicate a flow (src/flow/mod.rs:20-42); the
/// default `extract_flow` runs the decode tree on the device.  One call per record pays a
/// host->device->host round trip: for many records use [`extract_flows`] / [`convert_records`],
/// which take the whole batch in one device call.
///
/// A device failure (no usable GPU, a lost HIP context) is not a flow error: `extract_flow` and
/// [`convert_records`] panic with the device's message, as the reference would on an allocation
/// failure, rather than answer with an error payload or a flow list the reference never produces
/// for that input.  `try_extract_flow` / [`try_convert_records`] return it instead.
pub trait FlowExtraction {
    fn payload(&self) -> &[u8];

    fn extract_flow(&self) -> Result<Flow, Error> {
        self.try_extract_flow().unwrap_or_else(|e| panic!("net-parser-rs-amd: device failure: {}", e))
    }

    /// extract_flow, with a device failure as the outer error
    fn try_extract_flow(&self) -> Result<Result<Flow, Error>, crate::Error> {
        let mut v = extract_payloads(&[self.payload()], None)?;
        Ok(v.pop().expect("one result per payload"))
    }
}

impl<'a> FlowExtraction for PcapRecord<'a> {
    fn payload(&self) -> &[u8] {
        self.payload
    }
}

/// extract_flow for a batch of records in ONE device call (file order kept).  Panics on a device
/// failure (see [`FlowExtraction`]); [`try_extract_flows`] returns it.
pub fn extract_flows<'b>(records: &[PcapRecord<'b>]) -> Vec<Result<Flow, Error>> {
    try_extract_flows(records).unwrap_or_else(|e| panic!("net-parser-rs-amd: device failure: {}", e))
}

pub fn try_extract_flows<'b>(records: &[PcapRecord<'b>]) -> Result<Vec<Result<Flow, Error>>, crate::Error> {
    let payloads: Vec<&[u8]> = records.iter().map(|r| r.payload).collect();
    extract_payloads(&payloads, None)
}

///
/// Utility function to convert a vector of records to flows, unless an error is encountered
/// in stream conversion (src/flow/mod.rs:101-123): Ok flows in REVERSE record order.  A device
/// failure panics with the device's message (the reference drops only the records whose
/// extract_flow failed: an empty list here would be a wrong answer); [`try_convert_records`]
/// returns it.
///
pub fn convert_records<'b>(records: Vec<PcapRecord<'b>>) -> Vec<(PcapRecord<'b>, Flow)> {
    try_convert_records(records).unwrap_or_else(|e| panic!("net-parser-rs-amd: device failure: {}", e))
}

pub fn try_convert_records<'b>(records: Vec<PcapRecord<'b>>) -> Result<Vec<(PcapRecord<'b>, Flow)>, crate::Error> {
    convert(records, None)
}

/// convert_records when the records borrow from `input` (e.g. CaptureFile::parse(input)): the
/// device reads the payloads from one staged copy of `input`, with no per-record gathering.
pub fn convert_records_in<'b>(input: &'b [u8], records: Vec<PcapRecord<'b>>) -> Vec<(PcapRecord<'b>, Flow)> {
    convert(records, Some(input)).unwrap_or_else(|e| panic!("net-parser-rs-amd: device failure: {}", e))
}

fn convert<'b>(records: Vec<PcapRecord<'b>>, input: Option<&[u8]>) -> Result<Vec<(PcapRecord<'b>, Flow)>, crate::Error> {
    let payloads: Vec<&[u8]> = records.iter().map(|r| r.payload).collect();
    let res = flows_only(&payloads, input)?;
    let mut out = Vec::with_capacity(records.len());
    for (r, f) in records.into_iter().zip(res.into_iter()).rev() {
        if let Some(f) = f {
            out.push((r, f));
        }
    }
    Ok(out)
}

/// The reference's `extract` bench step (benches/benches.rs:56-62: CaptureFile::parse then
/// convert_records) fused into one device pass with the PCIe transfers pipelined
/// (npr_parse_extract_pipelined).  Returns the unparsed remainder and the (record, flow) pairs
/// in convert_records order.
/// Rows to reserve for a capture's flows: its record count predicted from the mean size of the
/// records in its first 256 KiB (the record chain walked on the host, 16 + incl_len each), +1/16
/// and +64 of slack; one row per 80 B (a 64-B frame) when fewer than 16 records fit there.
fn rows_for(input: &[u8], big: bool) -> usize {
    let body = &input[24.min(input.len())..];
    let head = &body[..body.len().min(256 << 10)];
    let (mut off, mut n) = (0usize, 0usize);
    while off + 16 <= head.len() {
        let b = [head[off + 8], head[off + 9], head[off + 10], head[off + 11]];
        let incl = if big { u32::from_be_bytes(b) } else { u32::from_le_bytes(b) } as usize;
        if incl > head.len() - off - 16 {
            break;
        }
        off += 16 + incl;
        n += 1;
    }
    let mean = if n >= 16 { (off / n).max(16) } else { 80 };
    let est = body.len() / mean + 1;
    est + est / 16 + 64
}

pub fn parse_and_convert<'b>(input: &'b [u8]) -> Result<(&'b [u8], Vec<(PcapRecord<'b>, Flow)>), crate::Error> {
    let (_, header) = crate::GlobalHeader::parse(input)?;
    let big = header.endianness == nom::Endianness::Big;
    let (rows, rows6, consumed) = with_ctx(|ctx| {
        // Rows for the flows the capture's first records predict (rows_for: their mean size over
        // at most 256 KiB, +1/16 and +64 of slack), uninitialised -- the device writes the Ok
        // flows' rows right-aligned, and only those are read back, so no zero fill and no
        // resident pages beyond what the call touches.  A capture whose later records
        // are smaller makes the call report NPR_ERR_CAPACITY with its exact flow count, and it
        // runs once more into exactly that many rows.
        let cap_all = input.len().saturating_sub(24) / 16 + 1;
        let mut cap = rows_for(input, big).min(cap_all);
        loop {
            let mut rows: Vec<std::mem::MaybeUninit<ffi::npr_flow>> = Vec::with_capacity(cap);
            let mut rows6: Vec<std::mem::MaybeUninit<ffi::npr_flow_v6>> = Vec::with_capacity(cap);
            // SAFETY: MaybeUninit elements need no initialisation
            unsafe {
                rows.set_len(cap);
                rows6.set_len(cap);
            }
            let mut hdr = ffi::npr_global_header::default();
            let (mut n, mut consumed) = (0usize, 0usize);
            let st = unsafe {
                ffi::npr_parse_extract_pipelined(
                    ctx,
                    input.as_ptr(),
                    input.len(),
                    &mut hdr,
                    rows.as_mut_ptr() as *mut ffi::npr_flow,
                    rows6.as_mut_ptr() as *mut ffi::npr_flow_v6,
                    cap,
                    &mut n,
                    &mut consumed,
                    0,
                )
            };
            if st == ffi::NPR_ERR_CAPACITY && n > cap && n <= cap_all {
                cap = n;
                continue;
            }
            check(ctx, st)?;
            // right-aligned: rows[cap - k .. cap] in convert_records order, written by the call;
            // a side row is written (and read) only where the flow is IPv6
            let k = n.min(cap);
            // SAFETY: the call wrote rows[cap - k .. cap], and side rows of IPv6 flows among them
            let tail: Vec<ffi::npr_flow> = rows[cap - k..cap].iter().map(|r| unsafe { r.assume_init_read() }).collect();
            let tail6: Vec<ffi::npr_flow_v6> = rows6[cap - k..cap]
                .iter()
                .zip(tail.iter())
                .map(|(f6, f)| {
                    if f.kind & ffi::NPR_FLOW_KIND_IPV6 != 0 {
                        unsafe { f6.assume_init_read() }
                    } else {
                        ffi::npr_flow_v6::default()
                    }
                })
                .collect();
            return Ok((tail, tail6, consumed));
        }
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
/// outer frame's UDP payload (to `dst_port`, 0 = any; 4789 is the IANA port) parsed as the
/// reference's `layer4::Vxlan::parse(.., endianness)` (src/layer4/vxlan.rs:31-48) and the inner
/// Ethernet frame's flow, as `<Vxlan as FlowExtraction>::extract_flow` (src/flow/layer4/vxlan.rs:
/// 32-50), with the VXLAN network identifier (0 when the header was not reached).  One device call.
/// Errors: an outer failure as extract_flow's; an inner Ethernet parse failure as
/// `Error::L4(Vxlan(NetParser(..)))`; other inner failures as the inner frame's own flow error; a
/// payload shorter than the VXLAN header as `Error::NetParser(Incomplete)`; an outer flow that is
/// not UDP to `dst_port` as `Error::NetParser(Custom)`.  (The payloads of the inner errors are not
/// computed: sizes 0 / None.)
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
    with_ctx(|ctx| {
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
    })
    .unwrap_or_else(|e| panic!("net-parser-rs-amd: device failure: {}", e));
    let outer = details(&payloads, input, &status);
    (0..n)
        .map(|i| {
            let st = status[i];
            let res = match st {
                0 => Ok(to_flow(&flows[i], &flows6[i])),
                ffi::NPR_VXLAN_NOT_UDP | ffi::NPR_VXLAN_PORT => Err(Error::NetParser(crate::Error::Custom {
                    msg: String::from("the outer flow is not UDP to the requested port"),
                })),
                ffi::NPR_VXLAN_INCOMPLETE => Err(Error::NetParser(crate::Error::Incomplete { size: None })),
                s if s > ffi::NPR_VXLAN_INNER => match s - ffi::NPR_VXLAN_INNER {
                    1 => Err(vxlan_eth_error(crate::Error::Incomplete { size: None })),
                    2 => Err(vxlan_eth_error(crate::Error::Failure { msg: String::new() })),
                    k => Err(flow_error(k, None, &[])),
                },
                s => Err(flow_error(s, outer.as_ref().map(|d| d[i]), payloads[i])),
            };
            (res, vni[i])
        })
        .collect()
}

/// Error::L4(Vxlan(NetParser(e))) (src/flow/layer4/vxlan.rs:35-38)
fn vxlan_eth_error(e: crate::Error) -> Error {
    let v = layer4::vxlan::errors::Error::NetParser(e);
    let l4: layer4::errors::Error = v.into();
    Error::L4(l4)
}

// ---- device calls -----------------------------------------------------------------------------
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

/// One npr_extract_flows call: per payload Some(flow) or None, and the status codes.
fn extract_raw(payloads: &[&[u8]], input: Option<&[u8]>) -> Result<(Vec<Option<Flow>>, Vec<u8>), crate::Error> {
    let n = payloads.len();
    let (buf, recs) = stage(payloads, input);
    let mut flows = vec![ffi::npr_flow::default(); n];
    let mut flows6 = vec![ffi::npr_flow_v6::default(); n];
    let mut status = vec![0u8; n];
    with_ctx(|ctx| {
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
    })?;
    let out = (0..n).map(|i| if status[i] == 0 { Some(to_flow(&flows[i], &flows6[i])) } else { None }).collect();
    Ok((out, status))
}

/// The error payloads (npr_flow_details) of the payloads whose status is not Ok: one more device
/// call over those records only.  None when that call failed: the errors then carry no payload
/// (size None, an explicit message) instead of a zero one.
fn details(payloads: &[&[u8]], input: Option<&[u8]>, status: &[u8]) -> Option<Vec<u64>> {
    let n = payloads.len();
    let mut det = vec![0u64; n];
    let bad: Vec<usize> = (0..n).filter(|&i| status[i] != 0 && status[i] < ffi::NPR_VXLAN_NOT_UDP).collect();
    if bad.is_empty() {
        return Some(det);
    }
    let sub: Vec<&[u8]> = bad.iter().map(|&i| payloads[i]).collect();
    let (buf, recs) = stage(&sub, input);
    let mut got = vec![0u64; sub.len()];
    let r = with_ctx(|ctx| {
        let st = unsafe {
            ffi::npr_flow_details(
                ctx,
                buf.as_ptr(),
                buf.len(),
                recs.as_ptr(),
                sub.len(),
                std::ptr::null_mut(),
                got.as_mut_ptr(),
            )
        };
        check(ctx, st)
    });
    r.ok()?;
    for (k, &i) in bad.iter().enumerate() {
        det[i] = got[k];
    }
    Some(det)
}

/// Per payload Some(flow) or None; a device failure is the error (never "no flows").
fn flows_only(payloads: &[&[u8]], input: Option<&[u8]>) -> Result<Vec<Option<Flow>>, crate::Error> {
    if payloads.is_empty() {
        return Ok(Vec::new());
    }
    extract_raw(payloads, input).map(|(f, _)| f)
}

/// extract_flow over `payloads` (read from `input` when they lie inside it): one device call, plus
/// one for the error payloads of the records that failed.
pub(crate) fn extract_payloads(payloads: &[&[u8]], input: Option<&[u8]>) -> Result<Vec<Result<Flow, Error>>, crate::Error> {
    let n = payloads.len();
    if n == 0 {
        return Ok(Vec::new());
    }
    let (flows, status) = extract_raw(payloads, input)?;
    let det = details(payloads, input, &status);
    Ok(flows
        .into_iter()
        .enumerate()
        .map(|(i, f)| match f {
            Some(f) => Ok(f),
            None => Err(flow_error(status[i], det.as_ref().map(|d| d[i]), payloads[i])),
        })
        .collect())
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

// ---- npr_flow_status + npr_flow_details -> the reference's flow error tree ----------------------------
/// nom's message for a map_opt! / map_res! failure: "Error: " + the Debug form of
/// Context::Code(<the failing primitive's input>, kind) (src/errors.rs:43-47); the detail word holds
/// the input's frame offsets start | end << 32.
fn nom_failure(p: &[u8], det: u64, kind: nom::ErrorKind<u32>) -> crate::Error {
    let (a, b) = ((det & 0xffff_ffff) as usize, (det >> 32) as usize);
    let input = if a <= b && b <= p.len() { &p[a..b] } else { &[][..] };
    crate::Error::Failure { msg: format!("Error: {:?}", nom::Context::Code(input, kind)) }
}

/// The reference's error for status `st`; `det` its payload (npr_flow_details), None when it could
/// not be computed: sizes become None and failure messages say so.
fn flow_error(st: u8, det: Option<u64>, p: &[u8]) -> Error {
    let known = det.is_some();
    let det = det.unwrap_or(0);
    use crate::layer2::ethernet::{EthernetTypeId as E, Layer3Id as L3};
    use crate::layer3::InternetProtocolId as P;
    use layer2::ethernet::errors::Error as Eth;
    use layer3::{arp, ipv4, ipv6};
    type NP = crate::Error;
    let inc = || NP::Incomplete { size: if known { Some(det as usize) } else { None } };
    let unknown = || NP::Custom { msg: String::from("the error payload could not be computed (device call failed)") };
    let opt = || if known { nom_failure(p, det, nom::ErrorKind::MapOpt) } else { unknown() };
    let eth = |e: Eth| -> Error {
        let l2: layer2::errors::Error = e.into();
        l2.into()
    };
    let l3e = |e: layer3::errors::Error| -> Error { e.into() };
    let v4 = || E::L3(L3::IPv4);
    let v6 = || E::L3(L3::IPv6);
    let proto = || P::new(det as u8).unwrap_or(P::ICMP);
    let size = det as usize;
    if !known && matches!(st, 3 | 6 | 9 | 11 | 12 | 13 | 15 | 16 | 23 | 24) {
        // the error's fields ARE the payload: no guessed etype / version / protocol / size
        return Error::NetParser(unknown());
    }
    match st {
        1 => Error::NetParser(inc()),
        2 => Error::NetParser(opt()),
        3 => eth(Eth::EthernetType { etype: E::from_value(det as u16).unwrap_or(E::PayloadLength(0)) }),
        4 => eth(Eth::NetParser { l3: v4(), err: inc() }),
        5 => eth(Eth::NetParser { l3: v4(), err: opt() }),
        6 => eth(Eth::NetParser { l3: v4(), err: NP::Custom { msg: format!("Expected version 4, was {}", det) } }),
        7 => eth(Eth::NetParser { l3: v6(), err: inc() }),
        8 => eth(Eth::NetParser { l3: v6(), err: opt() }),
        9 => eth(Eth::NetParser { l3: v6(), err: NP::Custom { msg: format!("Expected version 6, version was {}", det) } }),
        10 => eth(Eth::NetParser { l3: E::L3(L3::Arp), err: inc() }),
        11 => eth(Eth::Incomplete { l3: v4(), size }),
        12 => eth(Eth::Incomplete { l3: v6(), size }),
        13 => eth(Eth::Incomplete { l3: E::L3(L3::Arp), size }),
        14 => l3e(arp::errors::Error::Flow.into()),
        15 => l3e(ipv4::errors::Error::InternetProtocolId { id: proto() }.into()),
        16 => l3e(ipv6::errors::Error::InternetProtocolId { id: proto() }.into()),
        17 => l3e(ipv4::errors::Error::NetParser { l4: P::Tcp, err: inc() }.into()),
        18 => l3e(ipv4::errors::Error::NetParser { l4: P::Tcp, err: if known { nom_failure(p, det, nom::ErrorKind::MapRes) } else { unknown() } }.into()),
        19 => l3e(ipv4::errors::Error::NetParser { l4: P::Udp, err: inc() }.into()),
        20 => l3e(ipv6::errors::Error::NetParser { l4: P::Tcp, err: inc() }.into()),
        21 => l3e(ipv6::errors::Error::NetParser { l4: P::Tcp, err: if known { nom_failure(p, det, nom::ErrorKind::MapRes) } else { unknown() } }.into()),
        22 => l3e(ipv6::errors::Error::NetParser { l4: P::Udp, err: inc() }.into()),
        23 => l3e(ipv4::errors::Error::Incomplete { l4: P::Udp, size }.into()),
        24 => l3e(ipv6::errors::Error::Incomplete { l4: P::Udp, size }.into()),
        _ => Error::NetParser(NP::Custom { msg: format!("record not inside the buffer (status {})", st) }),
    }
}
