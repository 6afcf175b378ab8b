//! `extern "C"` view of include/npr.h (ABI 5): the entry points this crate binds, with the
//! reference functions they replace.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub type npr_status = c_int;
pub const NPR_OK: npr_status = 0;
pub const NPR_INCOMPLETE: npr_status = 1; // crate::errors::Error::Incomplete (src/errors.rs:5)
pub const NPR_FAILURE: npr_status = 2; // Error::Failure (src/errors.rs:7)
pub const NPR_CUSTOM: npr_status = 3; // Error::Custom (src/errors.rs:9)
pub const NPR_ERR_CAPACITY: npr_status = -3;
pub const NPR_LITTLE: c_int = 0;
pub const NPR_BIG: c_int = 1;
pub const NPR_ABI_VERSION: c_int = 5;
pub const NPR_FLOW_KIND_IPV6: u8 = 0x1;
pub const NPR_FLOW_KIND_UDP: u8 = 0x2;

#[repr(C)]
pub struct npr_ctx {
    _private: [u8; 0],
}

/// GlobalHeader (src/global_header.rs:13-23)
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_global_header {
    pub endianness: i32,
    pub version_major: u16,
    pub version_minor: u16,
    pub zone: i32,
    pub sig_figs: i32,
    pub snap_length: u32,
    pub network: u32,
}

/// PcapRecord (src/record.rs:59-65) as a byte offset into the caller's buffer
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_record {
    pub offset: u64,
    pub ts_sec: u32,
    pub ts_usec: u32,
    pub actual_length: u32,
    pub original_length: u32,
}

/// Flow (src/flow/mod.rs:53-61) in the fixed 32-byte encoding
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_flow {
    pub src_ip: [u8; 4],
    pub dst_ip: [u8; 4],
    pub src_port: u16,
    pub dst_port: u16,
    pub vlan: u16,
    pub src_mac: [u8; 6],
    pub dst_mac: [u8; 6],
    pub kind: u8,
    pub record_offset: [u8; 5],
}

// VXLAN statuses (include/npr.h): an outer failure keeps its flow status code
pub const NPR_VXLAN_NOT_UDP: u8 = 32;
pub const NPR_VXLAN_PORT: u8 = 33;
pub const NPR_VXLAN_INCOMPLETE: u8 = 34;
pub const NPR_VXLAN_INNER: u8 = 64;

#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_flow_v6 {
    pub src_ip: [u8; 16],
    pub dst_ip: [u8; 16],
}

// ---- host-side per-layer header objects (include/npr.h): byte ranges are {offset, length} ----------
/// VlanTag (src/layer2/ethernet.rs:85-98)
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_vlan_tag {
    pub vlan_type: u16,
    pub vlan_value: u16,
    pub prio: u8,
    pub dei: u8,
    pub id: u16,
}

/// Ethernet (src/layer2/ethernet.rs:100-107); the first min(n_vlans, cap) tags go to the tag array
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_ethernet {
    pub dst_mac: [u8; 6],
    pub src_mac: [u8; 6],
    pub ether_type: u16,
    pub reserved: u16,
    pub n_vlans: u32,
    pub payload_offset: u64,
    pub payload_length: u64,
}

/// IPv4 (src/layer3/ipv4.rs:14-29); options / padding length 0 = None
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_ipv4 {
    pub version_and_length: u8,
    pub tos: u8,
    pub raw_length: u16,
    pub id: u16,
    pub flags: u16,
    pub ttl: u8,
    pub protocol: u8,
    pub checksum: u16,
    pub src_ip: [u8; 4],
    pub dst_ip: [u8; 4],
    pub payload_offset: u64,
    pub payload_length: u64,
    pub options_offset: u64,
    pub options_length: u64,
    pub padding_offset: u64,
    pub padding_length: u64,
}

/// IPv6 (src/layer3/ipv6.rs:10-16)
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_ipv6 {
    pub dst_ip: [u8; 16],
    pub src_ip: [u8; 16],
    pub protocol: u8,
    pub reserved: [u8; 7],
    pub payload_offset: u64,
    pub payload_length: u64,
}

/// Arp (src/layer3/arp.rs:7-14)
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_arp {
    pub sender_ip: [u8; 4],
    pub sender_mac: [u8; 6],
    pub target_ip: [u8; 4],
    pub target_mac: [u8; 6],
    pub operation: u16,
}

/// Tcp (src/layer4/tcp.rs:11-30) with its HeaderLengthAndFlags
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_tcp {
    pub src_port: u16,
    pub dst_port: u16,
    pub sequence_number: u32,
    pub acknowledgement_number: u32,
    pub header_length_and_flags: u16,
    pub flags: u16,
    pub header_length: u32,
    pub window: u16,
    pub check: u16,
    pub urgent: u16,
    pub reserved: u16,
    pub options_offset: u64,
    pub options_length: u64,
    pub payload_offset: u64,
    pub payload_length: u64,
}

/// Udp (src/layer4/udp.rs:10-16)
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_udp {
    pub src_port: u16,
    pub dst_port: u16,
    pub checksum: u16,
    pub reserved: u16,
    pub payload_offset: u64,
    pub payload_length: u64,
}

/// Vxlan (src/layer4/vxlan.rs:7-14)
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct npr_vxlan {
    pub flags: u16,
    pub group_policy_id: u16,
    pub raw_network_identifier: u32,
    pub network_identifier: u32,
    pub reserved: u32,
    pub payload_offset: u64,
    pub payload_length: u64,
}

extern "C" {
    /// Ethernet::parse (src/layer2/ethernet.rs:204-216), host side.  Incomplete: *detail = nom's
    /// Needed::Size; Failure: *detail = start | end << 32 of the map_opt! input; more tags than
    /// vlan_cap: NPR_ERR_CAPACITY with the exact n_vlans
    pub fn npr_ethernet_parse(
        input: *const u8,
        len: usize,
        out: *mut npr_ethernet,
        vlans: *mut npr_vlan_tag,
        vlan_cap: usize,
        consumed: *mut usize,
        detail: *mut u64,
    ) -> npr_status;
    /// IPv4::parse (src/layer3/ipv4.rs:148-160); Custom: *detail = the version nibble
    pub fn npr_ipv4_parse(input: *const u8, len: usize, out: *mut npr_ipv4, consumed: *mut usize, detail: *mut u64) -> npr_status;
    /// IPv6::parse (src/layer3/ipv6.rs:87-99); Custom: *detail = the version nibble
    pub fn npr_ipv6_parse(input: *const u8, len: usize, out: *mut npr_ipv6, consumed: *mut usize, detail: *mut u64) -> npr_status;
    /// Arp::parse (src/layer3/arp.rs:54-76)
    pub fn npr_arp_parse(input: *const u8, len: usize, out: *mut npr_arp, consumed: *mut usize, detail: *mut u64) -> npr_status;
    /// Tcp::parse (src/layer4/tcp.rs:59-101); Failure = the map_res! on the header length
    pub fn npr_tcp_parse(input: *const u8, len: usize, out: *mut npr_tcp, consumed: *mut usize, detail: *mut u64) -> npr_status;
    /// Udp::parse (src/layer4/udp.rs:33-50)
    pub fn npr_udp_parse(input: *const u8, len: usize, out: *mut npr_udp, consumed: *mut usize, detail: *mut u64) -> npr_status;
    /// Vxlan::parse (src/layer4/vxlan.rs:31-48)
    pub fn npr_vxlan_parse(
        input: *const u8,
        len: usize,
        endianness: c_int,
        out: *mut npr_vxlan,
        consumed: *mut usize,
        detail: *mut u64,
    ) -> npr_status;

    /// GlobalHeader::parse (src/global_header.rs:40-70): 24 bytes, host side
    pub fn npr_global_header_parse(
        input: *const u8,
        len: usize,
        out: *mut npr_global_header,
        consumed: *mut usize,
    ) -> npr_status;

    /// PcapRecord::parse (src/record.rs:102-121): one 16-byte header + its payload, host side
    pub fn npr_record_parse(
        input: *const u8,
        len: usize,
        endianness: c_int,
        out: *mut npr_record,
        consumed: *mut usize,
    ) -> npr_status;

    pub fn npr_abi_version() -> c_int;
    pub fn npr_version() -> *const c_char;
    pub fn npr_ctx_create(device: c_int, out: *mut *mut npr_ctx) -> npr_status;
    pub fn npr_ctx_destroy(ctx: *mut npr_ctx);
    pub fn npr_ctx_last_error(ctx: *const npr_ctx) -> *const c_char;

    /// PcapRecords::parse (src/record.rs:21-54)
    pub fn npr_records_parse(
        ctx: *mut npr_ctx,
        input: *const u8,
        len: usize,
        endianness: c_int,
        out: *mut npr_record,
        cap: usize,
        n_out: *mut usize,
        consumed: *mut usize,
    ) -> npr_status;

    /// FlowExtraction::extract_flow (src/flow/mod.rs:20-48) over a batch of records: dense
    /// per-record status (npr_flow_status) and flow rows
    pub fn npr_extract_flows(
        ctx: *mut npr_ctx,
        input: *const u8,
        len: usize,
        records: *const npr_record,
        n: usize,
        flows: *mut npr_flow,
        flows_v6: *mut npr_flow_v6,
        status: *mut u8,
    ) -> npr_status;

    /// flow::convert_records (src/flow/mod.rs:101-123): Ok flows, reverse record order
    pub fn npr_convert_records(
        ctx: *mut npr_ctx,
        input: *const u8,
        len: usize,
        records: *const npr_record,
        n: usize,
        out: *mut npr_flow,
        out_v6: *mut npr_flow_v6,
        cap: usize,
        n_out: *mut usize,
    ) -> npr_status;

    /// CaptureFile::parse + convert_records, PCIe transfers pipelined; flows right-aligned in out
    pub fn npr_parse_extract_pipelined(
        ctx: *mut npr_ctx,
        input: *const u8,
        len: usize,
        header: *mut npr_global_header,
        out: *mut npr_flow,
        out_v6: *mut npr_flow_v6,
        flow_cap: usize,
        n_flows: *mut usize,
        consumed: *mut usize,
        chunk_bytes: u64,
    ) -> npr_status;

    /// Row f3: the VXLAN inner flow of each record (Vxlan::parse, src/layer4/vxlan.rs:31-48, then
    /// <Vxlan as FlowExtraction>::extract_flow, src/flow/layer4/vxlan.rs:32-50); dense outputs
    pub fn npr_vxlan_flows(
        ctx: *mut npr_ctx,
        input: *const u8,
        len: usize,
        records: *const npr_record,
        n: usize,
        dst_port: u32,
        endianness: c_int,
        flows: *mut npr_flow,
        flows_v6: *mut npr_flow_v6,
        status: *mut u8,
        vni: *mut u32,
    ) -> npr_status;

    /// The payload each record's extract_flow error variant carries (include/npr.h npr_flow_details)
    pub fn npr_flow_details(
        ctx: *mut npr_ctx,
        input: *const u8,
        len: usize,
        records: *const npr_record,
        n: usize,
        status: *mut u8,
        detail: *mut u64,
    ) -> npr_status;

    pub fn npr_host_alloc(ctx: *mut npr_ctx, bytes: usize, out: *mut *mut c_void) -> npr_status;
    pub fn npr_host_free(ctx: *mut npr_ctx, p: *mut c_void) -> npr_status;
}
