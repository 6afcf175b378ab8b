//! net-parser-rs-amd — a drop-in for net-parser-rs 0.3 whose record parse and flow extraction run
//! on an AMD MI355X (HIP kernels in libnpr.so, behind the C-ABI of include/npr.h).
//!
//! Switch a dependent crate over by renaming the dependency:
//!
//! ```toml
//! [dependencies]
//! net-parser-rs = { package = "net-parser-rs-amd", path = ".../rust/net-parser-rs-amd" }
//! ```
//!
//! The reference crate is neither a dependency nor linked: the types on the record-parse and
//! flow-extraction path are restated here (`types.rs`, field for field, same `Display` strings) and
//! every parse runs in libnpr.
//!
//! **Surface.**  This crate is a drop-in for the capture -> records -> flows path (the table below)
//! and the reference's per-layer header objects.  Code that uses those items compiles unchanged.
//! - The per-layer parsers and their structs, under the reference's paths:
//!   `layer2::ethernet::{Ethernet, VlanTag}` (src/layer2/ethernet.rs:84-217),
//!   `layer3::{Arp, IPv4, IPv6, Layer3}` (src/layer3/{arp,ipv4,ipv6}.rs),
//!   `layer4::{Tcp, Udp, Vxlan, Layer4}` (src/layer4/{tcp,udp,vxlan}.rs), with their `as_bytes`:
//!   each `parse` runs libnpr's host-side layer parser (npr_ethernet_parse ... npr_vxlan_parse).
//! - `flow::layer2::FlowExtraction` for `Ethernet` (src/flow/layer2/ethernet.rs:39): the frame's flow
//!   from the device decoder.  NOT restated: the layer-3 / layer-4 `FlowExtraction` traits
//!   (src/flow/layer3/mod.rs:9, src/flow/layer4/mod.rs:10), which build a flow from outer-layer
//!   info structs; [`flow::FlowExtraction`] on [`PcapRecord`] and [`flow::vxlan_flows`] cover the
//!   record path and the VXLAN inner flow.
//!
//! | reference (src file:line)                          | here                                            |
//! |----------------------------------------------------|-------------------------------------------------|
//! | `net_parser_rs::parse` (src/lib.rs:44-46)          | [`parse`]                                       |
//! | `CaptureFile::parse` (src/file.rs:14-35)           | [`CaptureFile::parse`]                          |
//! | `GlobalHeader::parse` (src/global_header.rs:40-70) | `npr_global_header_parse` (24 B, host side)     |
//! | `PcapRecords::parse` (src/record.rs:21-54)         | `npr_records_parse`: the record chain on the GPU |
//! | `PcapRecord::parse` (src/record.rs:102-121)        | `npr_record_parse` (16 B, host side)            |
//! | `FlowExtraction::extract_flow` (src/flow/mod.rs:23)| [`flow::FlowExtraction`]: `npr_extract_flows`   |
//! | `flow::convert_records` (src/flow/mod.rs:101-123)  | [`flow::convert_records`]                       |
//! | README `CaptureParser` facade (README.md:17-28)    | [`CaptureParser`]                               |
//!
//! Device errors (no GPU, a HIP failure): the parse functions return them as
//! `Error::Custom { msg }` (the reference's error enum, src/errors.rs:3-11, has no variant for
//! them).  `FlowExtraction::extract_flow`, `flow::extract_flows` and `flow::convert_records`,
//! whose reference signatures cannot carry them (a per-record flow error would misreport the
//! record, an empty flow list is a wrong answer), panic with the device's message; their `try_`
//! forms return it.
//!
//! Threading: the reference's functions are pure and reentrant (its errors are Send + Sync,
//! src/errors.rs:13-14).  Here every thread uses its own libnpr context (`thread_local!` below),
//! and libnpr orders the look-back launches of all contexts on a device, so any number of threads
//! may call in at once.
#![allow(clippy::needless_lifetimes)]

pub mod ffi;
pub mod flow;
mod layers;
mod types;

pub use types::{common, errors, layer2, layer3, layer4};

/// src/global_header.rs: the header type, its constants and GlobalHeader::parse (over the C-ABI)
pub mod global_header {
    pub use crate::types::global_header::{GlobalHeader, NATIVE_ENDIAN};
}

/// src/record.rs and src/file.rs paths
pub mod record {
    pub use crate::{PcapRecord, PcapRecords};
}
pub mod file {
    pub use crate::CaptureFile;
}

pub use errors::Error;
pub use global_header::GlobalHeader;

use std::cell::RefCell;
use std::ffi::CStr;
use std::time::{Duration, SystemTime, UNIX_EPOCH};

// ---- one libnpr context per thread ----------------------------------------------------------------
struct Ctx(*mut ffi::npr_ctx);

impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { ffi::npr_ctx_destroy(self.0) }
    }
}

thread_local! {
    static CTX: RefCell<Option<Ctx>> = RefCell::new(None);
}

/// Run `f` with this thread's context (created on first use on HIP device `$NPR_DEVICE`, 0).
pub(crate) fn with_ctx<T, F>(f: F) -> Result<T, Error>
where
    F: FnOnce(*mut ffi::npr_ctx) -> Result<T, Error>,
{
    CTX.with(|cell| {
        let mut slot = cell.borrow_mut();
        if slot.is_none() {
            let dev: i32 = std::env::var("NPR_DEVICE").ok().and_then(|s| s.parse().ok()).unwrap_or(0);
            let mut p: *mut ffi::npr_ctx = std::ptr::null_mut();
            let st = unsafe { ffi::npr_ctx_create(dev, &mut p) };
            if st != ffi::NPR_OK {
                return Err(Error::Custom {
                    msg: format!("npr_ctx_create({}) failed with status {}: no usable HIP device", dev, st),
                });
            }
            *slot = Some(Ctx(p));
        }
        let ctx = slot.as_ref().map(|c| c.0).unwrap_or(std::ptr::null_mut());
        f(ctx)
    })
}

/// A device-path npr_status as crate::errors::Error (codes 1..3 map 1:1, src/errors.rs:3-11).
pub(crate) fn check(ctx: *mut ffi::npr_ctx, st: ffi::npr_status) -> Result<(), Error> {
    match st {
        ffi::NPR_OK => Ok(()),
        ffi::NPR_INCOMPLETE => Err(Error::Incomplete { size: None }),
        ffi::NPR_FAILURE => Err(Error::Failure { msg: String::new() }),
        ffi::NPR_CUSTOM => Err(Error::Custom { msg: String::new() }),
        _ => {
            let m = if ctx.is_null() {
                String::new()
            } else {
                unsafe { CStr::from_ptr(ffi::npr_ctx_last_error(ctx)) }.to_string_lossy().into_owned()
            };
            Err(Error::Custom { msg: format!("npr status {}: {}", st, m) })
        }
    }
}

pub(crate) fn endian(e: nom::Endianness) -> std::os::raw::c_int {
    match e {
        nom::Endianness::Big => ffi::NPR_BIG,
        nom::Endianness::Little => ffi::NPR_LITTLE,
    }
}

/// nom's Needed::Size for an input of `have` bytes that stops a chain of fixed-size primitives
/// (`sizes`, in parse order): the size of the first primitive that does not fit (nom 4.2 reports a
/// primitive's full size, e.g. u32! -> 4).
pub(crate) fn needed(sizes: &[usize], have: usize) -> Option<usize> {
    let mut end = 0;
    for &k in sizes {
        end += k;
        if end > have {
            return Some(k);
        }
    }
    None
}

// ---- GlobalHeader::parse (src/global_header.rs:40-70) over npr_global_header_parse -----------------
impl GlobalHeader {
    /// The 24-byte libpcap file header: the magic read in native order decides the endianness
    /// (0xA1B2C3D4: native, anything else: the other order), then six fields in that order.
    pub fn parse<'a>(input: &'a [u8]) -> Result<(&'a [u8], GlobalHeader), Error> {
        let mut h = ffi::npr_global_header::default();
        let mut used = 0usize;
        let st = unsafe { ffi::npr_global_header_parse(input.as_ptr(), input.len(), &mut h, &mut used) };
        if st == ffi::NPR_INCOMPLETE {
            // u32! magic, u16! x2, i32! x2, u32! x2 (src/global_header.rs:43-59)
            return Err(Error::Incomplete { size: needed(&[4, 2, 2, 4, 4, 4, 4], input.len()) });
        }
        check(std::ptr::null_mut(), st)?;
        let header = GlobalHeader {
            endianness: if h.endianness == ffi::NPR_BIG { nom::Endianness::Big } else { nom::Endianness::Little },
            version_major: h.version_major,
            version_minor: h.version_minor,
            zone: h.zone,
            sig_figs: h.sig_figs,
            snap_length: h.snap_length,
            network: h.network,
        };
        Ok((&input[used..], header))
    }
}

// ---- PcapRecord (src/record.rs:56-139) ------------------------------------------------------------
/// One libpcap record: its header fields and the payload it borrows from the input
#[derive(Clone, Copy, Debug)]
pub struct PcapRecord<'a> {
    pub timestamp: SystemTime,
    pub actual_length: u32,
    pub original_length: u32,
    pub payload: &'a [u8],
}

impl<'a> Default for PcapRecord<'a> {
    fn default() -> Self {
        PcapRecord { timestamp: UNIX_EPOCH, actual_length: 0, original_length: 0, payload: &[] }
    }
}

impl<'a> PcapRecord<'a> {
    /// UNIX_EPOCH + seconds + microseconds (the microseconds are not bounded, src/record.rs:82-86)
    pub fn convert_packet_time(ts_seconds: u32, ts_microseconds: u32) -> SystemTime {
        UNIX_EPOCH + Duration::from_secs(ts_seconds as u64) + Duration::from_micros(ts_microseconds as u64)
    }

    pub fn new(timestamp: SystemTime, actual_length: u32, original_length: u32, payload: &'a [u8]) -> PcapRecord<'a> {
        PcapRecord { timestamp, actual_length, original_length, payload }
    }

    /// One record (16-byte header in `endianness`, then `actual_length` payload bytes) and the
    /// rest of the input, by npr_record_parse.
    pub fn parse<'b>(input: &'b [u8], endianness: nom::Endianness) -> Result<(&'b [u8], PcapRecord<'b>), Error> {
        let mut r = ffi::npr_record::default();
        let mut used = 0usize;
        let st = unsafe { ffi::npr_record_parse(input.as_ptr(), input.len(), endian(endianness), &mut r, &mut used) };
        if st == ffi::NPR_INCOMPLETE {
            // four u32! then take!(actual_length) (src/record.rs:106-111)
            let size = if input.len() < 16 {
                needed(&[4, 4, 4, 4], input.len())
            } else {
                let b = [input[8], input[9], input[10], input[11]];
                let incl = match endianness {
                    nom::Endianness::Big => u32::from_be_bytes(b),
                    nom::Endianness::Little => u32::from_le_bytes(b),
                };
                Some(incl as usize)
            };
            return Err(Error::Incomplete { size });
        }
        check(std::ptr::null_mut(), st)?;
        Ok((&input[used..], to_record(input, &r)))
    }
}

impl<'a> std::fmt::Display for PcapRecord<'a> {
    /// `Timestamp=<secs><millis>   Length=..   Original Length=..` (src/record.rs:123-139: the
    /// milliseconds are appended without padding)
    fn fmt(&self, f: &mut std::fmt::Formatter) -> std::fmt::Result {
        let d = self.timestamp.duration_since(UNIX_EPOCH).map_err(|_| std::fmt::Error)?;
        write!(
            f,
            "Timestamp={}{}   Length={}   Original Length={}",
            d.as_secs(),
            d.subsec_millis(),
            self.actual_length,
            self.original_length
        )
    }
}

/// A device record row as a PcapRecord borrowing `input`.
pub(crate) fn to_record<'b>(input: &'b [u8], r: &ffi::npr_record) -> PcapRecord<'b> {
    let o = r.offset as usize + 16;
    PcapRecord::new(
        PcapRecord::convert_packet_time(r.ts_sec, r.ts_usec),
        r.actual_length,
        r.original_length,
        &input[o..o + r.actual_length as usize],
    )
}

// ---- PcapRecords (src/record.rs:7-54) -------------------------------------------------------------
/// Collection of pcap records associated with a libpcap capture
#[derive(Clone, Debug)]
pub struct PcapRecords<'a> {
    inner: Vec<PcapRecord<'a>>,
}

impl<'a> PcapRecords<'a> {
    pub fn len(&self) -> usize {
        self.inner.len()
    }

    pub fn into_inner(self) -> Vec<PcapRecord<'a>> {
        self.inner
    }

    /// Records of `input` (no global header) in the given endianness, until the first incomplete
    /// record (src/record.rs:30-49); the remainder is returned like the reference's.  The record
    /// chain is found and verified on the device (npr_records_parse).
    pub fn parse<'b>(input: &'b [u8], endianness: nom::Endianness) -> Result<(&'b [u8], PcapRecords<'b>), Error> {
        let (rows, consumed) = with_ctx(|ctx| {
            // room for the most records the input can hold; not zero-filled, so only the pages of
            // the n rows the device writes are ever touched (the rest stays a virtual reservation)
            let cap = input.len() / 16 + 1;
            let mut rows: Vec<ffi::npr_record> = Vec::with_capacity(cap);
            let (mut n, mut consumed) = (0usize, 0usize);
            let st = unsafe {
                ffi::npr_records_parse(
                    ctx,
                    input.as_ptr(),
                    input.len(),
                    endian(endianness),
                    rows.as_mut_ptr(),
                    cap,
                    &mut n,
                    &mut consumed,
                )
            };
            check(ctx, st)?;
            unsafe { rows.set_len(n.min(cap)) };
            Ok((rows, consumed))
        })?;
        let inner = rows.iter().map(|r| to_record(input, r)).collect();
        Ok((&input[consumed..], PcapRecords { inner }))
    }
}

// ---- CaptureFile (src/file.rs:4-35) ---------------------------------------------------------------
#[derive(Clone, Debug)]
pub struct CaptureFile<'a> {
    pub global_header: GlobalHeader,
    pub records: PcapRecords<'a>,
}

impl<'a> CaptureFile<'a> {
    ///
    /// Parse a slice of bytes that start with libpcap file format header: the 24-byte header on the
    /// host (npr_global_header_parse), the record chain on the device.
    ///
    pub fn parse<'b>(input: &'b [u8]) -> Result<(&'b [u8], CaptureFile<'b>), Error> {
        let (rem, header) = GlobalHeader::parse(input)?;
        let (records_rem, records) = PcapRecords::parse(rem, header.endianness)?;
        Ok((records_rem, CaptureFile { global_header: header, records }))
    }
}

/// net_parser_rs::parse (src/lib.rs:44-46)
pub fn parse<'a>(data: &'a [u8]) -> Result<(&'a [u8], CaptureFile<'a>), Error> {
    CaptureFile::parse(data)
}

/// The README facade (README.md:17-28; the reference's code has no CaptureParser).  Its
/// parse_records / parse_record take no endianness: native order, as GlobalHeader::default
/// (src/global_header.rs:25-37).
pub struct CaptureParser;

impl CaptureParser {
    /// Parse a file with global header and packet records
    pub fn parse_file<'a>(data: &'a [u8]) -> Result<Vec<PcapRecord<'a>>, Error> {
        CaptureFile::parse(data).map(|(_, f)| f.records.into_inner())
    }

    /// Parse a sequence of one or more packet records
    pub fn parse_records<'a>(data: &'a [u8]) -> Result<Vec<PcapRecord<'a>>, Error> {
        PcapRecords::parse(data, global_header::NATIVE_ENDIAN).map(|(_, r)| r.into_inner())
    }

    /// Parse a single packet
    pub fn parse_record<'a>(data: &'a [u8]) -> Result<PcapRecord<'a>, Error> {
        PcapRecord::parse(data, global_header::NATIVE_ENDIAN).map(|(_, r)| r)
    }
}
