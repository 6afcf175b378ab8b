//! net-parser-rs-amd — a drop-in for net-parser-rs 0.3 whose hot path runs on an AMD MI355X.
//!
//! Switch a dependent crate over by renaming the dependency:
//!
//! ```toml
//! [dependencies]
//! net-parser-rs = { package = "net-parser-rs-amd", path = ".../rust/net-parser-rs-amd" }
//! ```
//!
//! and code written against the reference compiles unchanged:
//!
//! | reference (src file:line)                          | here                                         |
//! |----------------------------------------------------|----------------------------------------------|
//! | `net_parser_rs::parse` (src/lib.rs:44-46)          | [`parse`]: device record chain                |
//! | `CaptureFile::parse` (src/file.rs:14-35)           | [`CaptureFile::parse`]                        |
//! | `PcapRecords::parse` (src/record.rs:21-54)         | [`PcapRecords::parse`]: `npr_records_parse`   |
//! | `PcapRecord::parse` (src/record.rs:102-121)        | the reference's own (16 B, host side)         |
//! | `GlobalHeader::parse` (src/global_header.rs:40-70) | the reference's own (24 B, host side)         |
//! | `FlowExtraction::extract_flow` (src/flow/mod.rs:23)| [`flow::FlowExtraction`]: `npr_extract_flows` |
//! | `flow::convert_records` (src/flow/mod.rs:101-123)  | [`flow::convert_records`]                     |
//! | README `CaptureParser` facade (README.md:17-28)    | [`CaptureParser`]                             |
//!
//! Every type whose fields are public (`GlobalHeader`, `PcapRecord`, `Error`, `flow::Flow`,
//! `flow::device::Device`, `flow::info`, `flow::errors`, `common::MacAddress`, the layer id
//! enums) IS the reference crate's type, re-exported.  `CaptureFile` and `PcapRecords` are
//! redefined with the same public API because the reference's `PcapRecords` has a private field.
//!
//! Device errors (no GPU, a HIP failure) surface as `Error::Custom { msg }`: the reference's
//! error enum (src/errors.rs:3-11) has no variant for them.
#![allow(clippy::needless_lifetimes)]

pub mod ffi;
pub mod flow;

/// Path compatibility with `net_parser_rs::record::*` and `net_parser_rs::file::*`.
pub mod record {
    pub use crate::{PcapRecord, PcapRecords};
}
pub mod file {
    pub use crate::CaptureFile;
}

pub use net_parser_rs::{common, errors, global_header, layer2, layer3, layer4};
pub use net_parser_rs::{Error, GlobalHeader, PcapRecord};

use std::cell::RefCell;
use std::ffi::CStr;

// ---- one libnpr context per thread (npr_ctx is per thread; the reference is reentrant) -------
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

/// An npr_status as the reference's crate::errors::Error (codes 1..3 map 1:1, src/errors.rs:3-11).
pub(crate) fn check(ctx: *mut ffi::npr_ctx, st: ffi::npr_status) -> Result<(), Error> {
    match st {
        ffi::NPR_OK => Ok(()),
        ffi::NPR_INCOMPLETE => Err(Error::Incomplete { size: None }),
        ffi::NPR_FAILURE => Err(Error::Failure { msg: String::new() }),
        ffi::NPR_CUSTOM => Err(Error::Custom { msg: String::new() }),
        _ => {
            let m = unsafe { CStr::from_ptr(ffi::npr_ctx_last_error(ctx)) }.to_string_lossy().into_owned();
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

/// A device record row as the reference's PcapRecord borrowing `input` (src/record.rs:88-100).
pub(crate) fn to_record<'b>(input: &'b [u8], r: &ffi::npr_record) -> PcapRecord<'b> {
    let o = r.offset as usize + 16;
    PcapRecord::new(
        PcapRecord::convert_packet_time(r.ts_sec, r.ts_usec),
        r.actual_length,
        r.original_length,
        &input[o..o + r.actual_length as usize],
    )
}

// ---- PcapRecords (src/record.rs:7-54) ----------------------------------------------------------
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

    /// Records of `input` (no global header) in the given endianness, until the first
    /// incomplete record (src/record.rs:30-49); the remainder is returned like the reference's.
    /// The record chain is found and verified on the device (npr_records_parse).
    pub fn parse<'b>(input: &'b [u8], endianness: nom::Endianness) -> Result<(&'b [u8], PcapRecords<'b>), Error> {
        let (rows, consumed) = with_ctx(|ctx| {
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

// ---- CaptureFile (src/file.rs:4-35) -------------------------------------------------------------
#[derive(Clone, Debug)]
pub struct CaptureFile<'a> {
    pub global_header: GlobalHeader,
    pub records: PcapRecords<'a>,
}

impl<'a> CaptureFile<'a> {
    ///
    /// Parse a slice of bytes that start with libpcap file format header: the 24-byte header on
    /// the host (the reference's own GlobalHeader::parse), the record chain on the device.
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
