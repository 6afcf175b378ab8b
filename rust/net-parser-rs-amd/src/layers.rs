//! The reference's per-layer header objects (src/layer2, src/layer3, src/layer4): the same structs,
//! fields, `as_bytes` serializers and `parse` signatures, re-exported under the reference's paths
//! (`layer2::ethernet::Ethernet`, `layer3::ipv4::IPv4`, ..., `layer4::Layer4`).  Each `parse` runs
//! libnpr's host-side layer parser (include/npr.h, csrc/npr_layers.hip: the nom chain step by step,
//! no device work) and borrows its slices from the caller's input, as the reference does.  Errors
//! are the reference's (src/errors.rs:16-55): Incomplete with nom's Needed::Size, Failure with
//! nom's `Code(<input>, MapOpt|MapRes)` message, Custom for the IP version checks.
//!
//! `flow::layer2::FlowExtraction` for `Ethernet` (src/flow/layer2/ethernet.rs:39-133) runs the frame
//! through the device decoder (one record, one call), which is what the reference's flow path
//! composes from these objects.  The layer-3 / layer-4 `FlowExtraction` traits, which take the
//! outer layers' flow info, are restated on the host exactly as the reference composes them:
//! `IPv4` / `IPv6` parse their payload with `Tcp::parse` / `Udp::parse` (libnpr's host parsers),
//! reject a remainder, and hand their info to the layer-4 object, which builds the `Flow`
//! (src/flow/layer3/{ipv4,ipv6,arp}.rs, src/flow/layer4/{tcp,udp}.rs).  No device work: these are
//! per-object calls on objects the caller already parsed.

use std::net::{IpAddr, Ipv4Addr, Ipv6Addr};

use crate::common::{MacAddress, Vlan};
use crate::errors::Error;
use crate::ffi;
use crate::layer2::ethernet::{EthernetTypeId, VlanTypeId};
use crate::layer3::InternetProtocolId;

/// The reference's error for a layer parser's status and detail word (include/npr.h)
fn check(st: ffi::npr_status, det: u64, input: &[u8], kind: nom::ErrorKind<u32>, custom: &str) -> Result<(), Error> {
    match st {
        ffi::NPR_OK | ffi::NPR_ERR_CAPACITY => Ok(()),
        ffi::NPR_INCOMPLETE => Err(Error::Incomplete { size: Some(det as usize) }),
        ffi::NPR_FAILURE => {
            let (a, b) = ((det & 0xffff_ffff) as usize, (det >> 32) as usize);
            let at = if a <= b && b <= input.len() { &input[a..b] } else { &input[input.len()..] };
            Err(Error::Failure { msg: format!("Error: {:?}", nom::Context::Code(at, kind)) })
        }
        ffi::NPR_CUSTOM => Err(Error::Custom { msg: custom.replace("{}", &det.to_string()) }),
        st => Err(Error::Custom { msg: format!("libnpr layer parser: status {}", st) }),
    }
}

fn range(input: &[u8], off: u64, len: u64) -> &[u8] {
    &input[off as usize..(off + len) as usize]
}

fn be16(out: &mut Vec<u8>, v: u16) {
    out.extend_from_slice(&v.to_be_bytes());
}

fn be32(out: &mut Vec<u8>, v: u32) {
    out.extend_from_slice(&v.to_be_bytes());
}

fn v4(ip: &IpAddr) -> [u8; 4] {
    match ip {
        IpAddr::V4(v) => v.octets(),
        IpAddr::V6(_) => [0; 4],
    }
}

// ---- layer 2: src/layer2/ethernet.rs --------------------------------------------------------------
/// src/layer2/ethernet.rs:85-98
#[allow(unused)]
#[derive(Clone, Copy, Debug)]
pub struct VlanTag {
    pub vlan_type: VlanTypeId,
    pub vlan_value: u16,
    pub prio: u8,
    pub dei: u8,
    pub id: u16,
}

impl VlanTag {
    pub fn vlan(&self) -> u16 {
        self.id
    }
}

/// src/layer2/ethernet.rs:100-107
#[derive(Clone, Debug)]
pub struct Ethernet<'a> {
    pub dst_mac: MacAddress,
    pub src_mac: MacAddress,
    pub ether_type: EthernetTypeId,
    pub vlans: std::vec::Vec<VlanTag>,
    pub payload: &'a [u8],
}

impl<'a> Ethernet<'a> {
    /// the MACs, each tag's type and value, the EtherType, the payload (src/layer2/ethernet.rs:116-133)
    pub fn as_bytes(&self) -> Vec<u8> {
        let mut out = Vec::with_capacity(14 + 4 * self.vlans.len() + self.payload.len());
        out.extend_from_slice(&self.dst_mac.0);
        out.extend_from_slice(&self.src_mac.0);
        for v in &self.vlans {
            be16(&mut out, v.vlan_type.value());
            be16(&mut out, v.vlan_value);
        }
        be16(&mut out, self.ether_type.value());
        out.extend_from_slice(self.payload);
        out
    }

    pub fn vlans_to_vlan(vlans: &std::vec::Vec<VlanTag>) -> Vlan {
        vlans.first().map(|v| v.vlan()).unwrap_or(0)
    }

    pub fn vlan(&self) -> Vlan {
        Ethernet::vlans_to_vlan(&self.vlans)
    }

    /// Ethernet::parse (src/layer2/ethernet.rs:204-216) by npr_ethernet_parse
    pub fn parse<'b>(input: &'b [u8]) -> Result<(&'b [u8], Ethernet<'b>), Error> {
        let mut cap = 8usize;
        loop {
            let mut e = ffi::npr_ethernet::default();
            let mut tags = vec![ffi::npr_vlan_tag::default(); cap];
            let (mut used, mut det) = (0usize, 0u64);
            let st = unsafe {
                ffi::npr_ethernet_parse(input.as_ptr(), input.len(), &mut e, tags.as_mut_ptr(), cap, &mut used, &mut det)
            };
            check(st, det, input, nom::ErrorKind::MapOpt, "")?;
            if e.n_vlans as usize > cap {
                cap = e.n_vlans as usize;
                continue;
            }
            let vlans = tags[..e.n_vlans as usize]
                .iter()
                .map(|t| VlanTag {
                    vlan_type: if t.vlan_type == 0x88a8 { VlanTypeId::ProviderBridging } else { VlanTypeId::VlanTagId },
                    vlan_value: t.vlan_value,
                    prio: t.prio,
                    dei: t.dei,
                    id: t.id,
                })
                .collect();
            let ether_type = EthernetTypeId::from_value(e.ether_type).expect("libnpr returns a known EtherType");
            let payload = range(input, e.payload_offset, e.payload_length);
            return Ok((
                &input[used..],
                Ethernet { dst_mac: MacAddress(e.dst_mac), src_mac: MacAddress(e.src_mac), ether_type, vlans, payload },
            ));
        }
    }
}

/// src/layer2/mod.rs: the layer-2 representations
#[derive(Clone, Debug)]
pub enum Layer2<'a> {
    Ethernet(Ethernet<'a>),
}

impl<'a> crate::flow::layer2::FlowExtraction for Ethernet<'a> {
    /// the flow of the frame this object serializes to (as_bytes), by the device decoder: what the
    /// reference's `Ethernet::extract_flow` (src/flow/layer2/ethernet.rs:39-133) composes from the
    /// layer objects.  Panics on a device failure, as `FlowExtraction::extract_flow` does.
    fn extract_flow(&self) -> Result<crate::flow::Flow, crate::flow::errors::Error> {
        let frame = self.as_bytes();
        let mut v = crate::flow::extract_payloads(&[&frame[..]], None)
            .unwrap_or_else(|e| panic!("net-parser-rs-amd: device failure: {}", e));
        v.pop().expect("one result per frame")
    }
}

// ---- layer 3: src/layer3/{ipv4,ipv6,arp}.rs -------------------------------------------------------
/// src/layer3/ipv4.rs:14-29
#[derive(Clone, Copy, Debug)]
pub struct IPv4<'a> {
    pub version_and_length: u8,
    pub tos: u8,
    pub raw_length: u16,
    pub id: u16,
    pub flags: u16,
    pub ttl: u8,
    pub protocol: InternetProtocolId,
    pub checksum: u16,
    pub src_ip: IpAddr,
    pub dst_ip: IpAddr,
    pub payload: &'a [u8],
    pub options: Option<&'a [u8]>,
    pub padding: Option<&'a [u8]>,
}

impl<'a> IPv4<'a> {
    /// the header fields, the addresses, then payload, options, padding (src/layer3/ipv4.rs:42-74)
    pub fn as_bytes(&self) -> Vec<u8> {
        let mut out = Vec::with_capacity(20 + self.payload.len());
        out.push(self.version_and_length);
        out.push(self.tos);
        be16(&mut out, self.raw_length);
        be16(&mut out, self.id);
        be16(&mut out, self.flags);
        out.push(self.ttl);
        out.push(self.protocol.value());
        be16(&mut out, self.checksum);
        if let IpAddr::V4(_) = self.src_ip {
            out.extend_from_slice(&v4(&self.src_ip));
        }
        if let IpAddr::V4(_) = self.dst_ip {
            out.extend_from_slice(&v4(&self.dst_ip));
        }
        out.extend_from_slice(self.payload);
        if let Some(o) = self.options {
            out.extend_from_slice(o);
        }
        if let Some(p) = self.padding {
            out.extend_from_slice(p);
        }
        out
    }

    /// IPv4::parse (src/layer3/ipv4.rs:148-160) by npr_ipv4_parse
    pub fn parse<'b>(input: &'b [u8]) -> Result<(&'b [u8], IPv4<'b>), Error> {
        let mut o = ffi::npr_ipv4::default();
        let (mut used, mut det) = (0usize, 0u64);
        let st = unsafe { ffi::npr_ipv4_parse(input.as_ptr(), input.len(), &mut o, &mut used, &mut det) };
        check(st, det, input, nom::ErrorKind::MapOpt, "Expected version 4, was {}")?;
        let opt = |off, len| if len > 0 { Some(range(input, off, len)) } else { None };
        Ok((
            &input[used..],
            IPv4 {
                version_and_length: o.version_and_length,
                tos: o.tos,
                raw_length: o.raw_length,
                id: o.id,
                flags: o.flags,
                ttl: o.ttl,
                protocol: InternetProtocolId::new(o.protocol).expect("libnpr returns a known protocol"),
                checksum: o.checksum,
                src_ip: IpAddr::V4(Ipv4Addr::from(o.src_ip)),
                dst_ip: IpAddr::V4(Ipv4Addr::from(o.dst_ip)),
                payload: range(input, o.payload_offset, o.payload_length),
                options: opt(o.options_offset, o.options_length),
                padding: opt(o.padding_offset, o.padding_length),
            },
        ))
    }
}

/// src/layer3/ipv6.rs:10-16
#[derive(Clone, Copy, Debug)]
pub struct IPv6<'a> {
    pub dst_ip: IpAddr,
    pub src_ip: IpAddr,
    pub protocol: InternetProtocolId,
    pub payload: &'a [u8],
}

impl<'a> IPv6<'a> {
    /// src/layer3/ipv6.rs:73-85
    pub fn new(dst_ip: Ipv6Addr, src_ip: Ipv6Addr, protocol: InternetProtocolId, payload: &'a [u8]) -> IPv6<'a> {
        IPv6 { dst_ip: IpAddr::V6(dst_ip), src_ip: IpAddr::V6(src_ip), protocol, payload }
    }

    /// IPv6::parse (src/layer3/ipv6.rs:87-99) by npr_ipv6_parse (one byte per "extension" header)
    pub fn parse<'b>(input: &'b [u8]) -> Result<(&'b [u8], IPv6<'b>), Error> {
        let mut o = ffi::npr_ipv6::default();
        let (mut used, mut det) = (0usize, 0u64);
        let st = unsafe { ffi::npr_ipv6_parse(input.as_ptr(), input.len(), &mut o, &mut used, &mut det) };
        check(st, det, input, nom::ErrorKind::MapOpt, "Expected version 6, version was {}")?;
        Ok((
            &input[used..],
            IPv6::new(
                Ipv6Addr::from(o.dst_ip),
                Ipv6Addr::from(o.src_ip),
                InternetProtocolId::new(o.protocol).expect("libnpr returns a known protocol"),
                range(input, o.payload_offset, o.payload_length),
            ),
        ))
    }
}

/// src/layer3/arp.rs:7-14
#[derive(Clone, Copy, Debug)]
pub struct Arp {
    pub sender_ip: IpAddr,
    pub sender_mac: MacAddress,
    pub target_ip: IpAddr,
    pub target_mac: MacAddress,
    pub operation: u16,
}

impl Arp {
    /// src/layer3/arp.rs:38-52
    pub fn new(sender_ip: Ipv4Addr, sender_mac: [u8; 6], target_ip: Ipv4Addr, target_mac: [u8; 6], operation: u16) -> Arp {
        Arp {
            sender_ip: IpAddr::V4(sender_ip),
            sender_mac: MacAddress(sender_mac),
            target_ip: IpAddr::V4(target_ip),
            target_mac: MacAddress(target_mac),
            operation,
        }
    }

    /// Arp::parse (src/layer3/arp.rs:54-76) by npr_arp_parse
    pub fn parse(input: &[u8]) -> Result<(&[u8], Arp), Error> {
        let mut o = ffi::npr_arp::default();
        let (mut used, mut det) = (0usize, 0u64);
        let st = unsafe { ffi::npr_arp_parse(input.as_ptr(), input.len(), &mut o, &mut used, &mut det) };
        check(st, det, input, nom::ErrorKind::MapOpt, "")?;
        Ok((
            &input[used..],
            Arp::new(Ipv4Addr::from(o.sender_ip), o.sender_mac, Ipv4Addr::from(o.target_ip), o.target_mac, o.operation),
        ))
    }
}

/// src/layer3/mod.rs: the layer-3 representations
#[derive(Clone, Copy, Debug)]
pub enum Layer3<'a> {
    Arp(Arp),
    IPv4(IPv4<'a>),
    IPv6(IPv6<'a>),
}

// ---- the layer-3 flow dispatch: src/flow/layer3/{ipv4,ipv6,arp}.rs ---------------------------------
use crate::flow::info::layer2::Info as L2Info;
use crate::flow::info::layer3::{Id as L3Id, Info as L3Info};
use crate::flow::info::layer4::{Id as L4Id, Info as L4Info};
use crate::flow::layer3::errors::Error as L3Error;
use crate::flow::layer4::FlowExtraction as Layer4Extraction;

// IPv4 / IPv6 share the reference's dispatch (src/flow/layer3/ipv4.rs:49-101, ipv6.rs:49-100):
// TCP and UDP parse their payload and must leave no remainder, any other protocol is an error.
// `wrap` makes the IP version's layer-3 error (IPv4 / IPv6 variant) of an ip_errors-shaped error.
macro_rules! ip_flow {
    ($payload:expr, $protocol:expr, $l2:expr, $l3:expr, $errs:ident, $wrap:expr) => {{
        let proto: InternetProtocolId = $protocol;
        let wrap = $wrap;
        let l4_err = |e: crate::flow::layer3::$errs::errors::Error| -> crate::flow::errors::Error {
            let e: L3Error = wrap(e);
            e.into()
        };
        match proto {
            InternetProtocolId::Tcp => match Tcp::parse($payload) {
                Err(err) => Err(l4_err(crate::flow::layer3::$errs::errors::Error::NetParser { l4: proto, err })),
                Ok((rem, l4)) if rem.is_empty() => l4.extract_flow($l2, $l3),
                Ok((rem, _)) => Err(l4_err(crate::flow::layer3::$errs::errors::Error::Incomplete { l4: proto, size: rem.len() })),
            },
            InternetProtocolId::Udp => match Udp::parse($payload) {
                Err(err) => Err(l4_err(crate::flow::layer3::$errs::errors::Error::NetParser { l4: proto, err })),
                Ok((rem, l4)) if rem.is_empty() => l4.extract_flow($l2, $l3),
                Ok((rem, _)) => Err(l4_err(crate::flow::layer3::$errs::errors::Error::Incomplete { l4: proto, size: rem.len() })),
            },
            _ => Err(l4_err(crate::flow::layer3::$errs::errors::Error::InternetProtocolId { id: proto })),
        }
    }};
}

/// <IPv4 as FlowExtraction>::extract_flow (src/flow/layer3/ipv4.rs:40-103)
impl<'a> crate::flow::layer3::FlowExtraction for IPv4<'a> {
    fn extract_flow(&self, l2: L2Info) -> Result<crate::flow::Flow, crate::flow::errors::Error> {
        let l3 = L3Info { id: L3Id::IPv4, src_ip: self.src_ip, dst_ip: self.dst_ip };
        ip_flow!(self.payload, self.protocol, l2, l3, ipv4, L3Error::IPv4)
    }
}

/// <IPv6 as FlowExtraction>::extract_flow (src/flow/layer3/ipv6.rs:40-102)
impl<'a> crate::flow::layer3::FlowExtraction for IPv6<'a> {
    fn extract_flow(&self, l2: L2Info) -> Result<crate::flow::Flow, crate::flow::errors::Error> {
        let l3 = L3Info { id: L3Id::IPv6, src_ip: self.src_ip, dst_ip: self.dst_ip };
        ip_flow!(self.payload, self.protocol, l2, l3, ipv6, L3Error::IPv6)
    }
}

/// <Arp as FlowExtraction>::extract_flow (src/flow/layer3/arp.rs:23-27): never a flow
impl crate::flow::layer3::FlowExtraction for Arp {
    fn extract_flow(&self, _l2: L2Info) -> Result<crate::flow::Flow, crate::flow::errors::Error> {
        let e: L3Error = crate::flow::layer3::arp::errors::Error::Flow.into();
        Err(e.into())
    }
}

// ---- the layer-4 flow: src/flow/layer4/{tcp,udp}.rs ------------------------------------------------
/// <Tcp as FlowExtraction>::extract_flow (src/flow/layer4/tcp.rs:23-35)
impl<'a> Layer4Extraction for Tcp<'a> {
    fn extract_flow(&self, l2: L2Info, l3: L3Info) -> Result<crate::flow::Flow, crate::flow::errors::Error> {
        Ok(crate::flow::Flow::new(l2, l3, L4Info { id: L4Id::Tcp, dst_port: self.dst_port, src_port: self.src_port }))
    }
}

/// <Udp as FlowExtraction>::extract_flow (src/flow/layer4/udp.rs:23-35)
impl<'a> Layer4Extraction for Udp<'a> {
    fn extract_flow(&self, l2: L2Info, l3: L3Info) -> Result<crate::flow::Flow, crate::flow::errors::Error> {
        Ok(crate::flow::Flow::new(l2, l3, L4Info { id: L4Id::Udp, dst_port: self.dst_port, src_port: self.src_port }))
    }
}

// ---- layer 4: src/layer4/{tcp,udp,vxlan}.rs -------------------------------------------------------
/// src/layer4/tcp.rs:11-16
#[derive(Clone, Copy, Debug)]
pub struct HeaderLengthAndFlags {
    pub inner: u16,
    pub header_length: usize,
    pub flags: u16,
}

/// src/layer4/tcp.rs:18-30
#[derive(Clone, Copy, Debug)]
pub struct Tcp<'a> {
    pub src_port: u16,
    pub dst_port: u16,
    pub sequence_number: u32,
    pub acknowledgement_number: u32,
    pub header_length_and_flags: HeaderLengthAndFlags,
    pub window: u16,
    pub check: u16,
    pub urgent: u16,
    pub options: &'a [u8],
    pub payload: &'a [u8],
}

impl<'a> Tcp<'a> {
    /// src/layer4/tcp.rs:33-51
    pub fn as_bytes(&self) -> Vec<u8> {
        let mut out = Vec::with_capacity(20 + self.options.len() + self.payload.len());
        be16(&mut out, self.src_port);
        be16(&mut out, self.dst_port);
        be32(&mut out, self.sequence_number);
        be32(&mut out, self.acknowledgement_number);
        be16(&mut out, self.header_length_and_flags.inner);
        be16(&mut out, self.window);
        be16(&mut out, self.check);
        be16(&mut out, self.urgent);
        out.extend_from_slice(self.options);
        out.extend_from_slice(self.payload);
        out
    }

    /// the data offset in bytes (src/layer4/tcp.rs:54-57)
    pub fn extract_length(value: u16) -> usize {
        ((value >> 12) * 4) as usize
    }

    /// Tcp::parse (src/layer4/tcp.rs:59-101) by npr_tcp_parse
    pub fn parse<'b>(input: &'b [u8]) -> Result<(&'b [u8], Tcp<'b>), Error> {
        let mut o = ffi::npr_tcp::default();
        let (mut used, mut det) = (0usize, 0u64);
        let st = unsafe { ffi::npr_tcp_parse(input.as_ptr(), input.len(), &mut o, &mut used, &mut det) };
        check(st, det, input, nom::ErrorKind::MapRes, "")?;
        Ok((
            &input[used..],
            Tcp {
                src_port: o.src_port,
                dst_port: o.dst_port,
                sequence_number: o.sequence_number,
                acknowledgement_number: o.acknowledgement_number,
                header_length_and_flags: HeaderLengthAndFlags {
                    inner: o.header_length_and_flags,
                    header_length: o.header_length as usize,
                    flags: o.flags,
                },
                window: o.window,
                check: o.check,
                urgent: o.urgent,
                options: range(input, o.options_offset, o.options_length),
                payload: range(input, o.payload_offset, o.payload_length),
            },
        ))
    }
}

/// src/layer4/udp.rs:10-16
#[derive(Clone, Copy, Debug)]
pub struct Udp<'a> {
    pub src_port: u16,
    pub dst_port: u16,
    pub checksum: u16,
    pub payload: &'a [u8],
}

impl<'a> Udp<'a> {
    /// the length field is the payload length + 8 (src/layer4/udp.rs:19-31)
    pub fn as_bytes(&self) -> Vec<u8> {
        let mut out = Vec::with_capacity(8 + self.payload.len());
        be16(&mut out, self.src_port);
        be16(&mut out, self.dst_port);
        be16(&mut out, (self.payload.len() + 8) as u16);
        be16(&mut out, self.checksum);
        out.extend_from_slice(self.payload);
        out
    }

    /// Udp::parse (src/layer4/udp.rs:33-50) by npr_udp_parse (a length below 8 wraps as usize)
    pub fn parse<'b>(input: &'b [u8]) -> Result<(&'b [u8], Udp<'b>), Error> {
        let mut o = ffi::npr_udp::default();
        let (mut used, mut det) = (0usize, 0u64);
        let st = unsafe { ffi::npr_udp_parse(input.as_ptr(), input.len(), &mut o, &mut used, &mut det) };
        check(st, det, input, nom::ErrorKind::MapOpt, "")?;
        Ok((
            &input[used..],
            Udp {
                src_port: o.src_port,
                dst_port: o.dst_port,
                checksum: o.checksum,
                payload: range(input, o.payload_offset, o.payload_length),
            },
        ))
    }
}

/// src/layer4/vxlan.rs:7-14
#[derive(Clone, Copy, Debug)]
pub struct Vxlan<'a> {
    pub flags: u16,
    pub group_policy_id: u16,
    pub raw_network_identifier: u32,
    pub network_identifier: u32,
    pub payload: &'a [u8],
}

impl<'a> Vxlan<'a> {
    /// big-endian header, then the payload (src/layer4/vxlan.rs:17-29)
    pub fn as_bytes(&self) -> Vec<u8> {
        let mut out = Vec::with_capacity(8 + self.payload.len());
        be16(&mut out, self.flags);
        be16(&mut out, self.group_policy_id);
        be32(&mut out, self.raw_network_identifier);
        out.extend_from_slice(self.payload);
        out
    }

    /// Vxlan::parse (src/layer4/vxlan.rs:31-48) by npr_vxlan_parse
    pub fn parse<'b>(input: &'b [u8], endianness: nom::Endianness) -> Result<(&'b [u8], Vxlan<'b>), Error> {
        let mut o = ffi::npr_vxlan::default();
        let (mut used, mut det) = (0usize, 0u64);
        let e = crate::endian(endianness);
        let st = unsafe { ffi::npr_vxlan_parse(input.as_ptr(), input.len(), e, &mut o, &mut used, &mut det) };
        check(st, det, input, nom::ErrorKind::MapOpt, "")?;
        Ok((
            &input[used..],
            Vxlan {
                flags: o.flags,
                group_policy_id: o.group_policy_id,
                raw_network_identifier: o.raw_network_identifier,
                network_identifier: o.network_identifier,
                payload: range(input, o.payload_offset, o.payload_length),
            },
        ))
    }
}

/// src/layer4/mod.rs:8-27: the layer-4 representations
#[derive(Clone, Copy, Debug)]
pub enum Layer4<'a> {
    Tcp(Tcp<'a>),
    Udp(Udp<'a>),
    Vxlan(Vxlan<'a>),
}

impl<'a> Layer4<'a> {
    pub fn as_bytes(&self) -> Vec<u8> {
        match self {
            Layer4::Tcp(v) => v.as_bytes(),
            Layer4::Udp(v) => v.as_bytes(),
            Layer4::Vxlan(v) => v.as_bytes(),
        }
    }
}
