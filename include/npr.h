/*
 * npr.h — C-ABI of the MI355X-native pcap record parser + flow extractor.
 *
 * This is the drop-in boundary for the hot path of protectwise/net-parser-rs 0.3.0:
 * the nom parse paths of src/global_header.rs, src/record.rs, src/file.rs, src/layer2,
 * src/layer3, src/layer4 and src/flow.  The reference has no FFI of its own (it is a pure
 * Rust crate); every entry point below names the reference function it replaces, and
 * INTEGRATION.md shows the `extern "C"` block a Rust maintainer would add to bind it.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch / HIP types in any signature
 *     (streams are passed as `void*` = hipStream_t, NULL = the context's own stream).
 *   - Results carry BYTE OFFSETS into the caller's buffer, never pointers: the Rust API
 *     borrows the input slice (`&'a [u8]`), an offset is the FFI-safe equivalent.
 *   - Status codes 1..3 map 1:1 onto crate::errors::Error (src/errors.rs:3-11);
 *     negative codes are boundary errors the Rust API cannot produce.
 *   - A context is per host thread (the Rust functions are pure and reentrant; a context
 *     owns one device, one stream and its workspaces, so give each thread its own).  Any number
 *     of contexts may launch on one device at once: libnpr orders their parse launches (whose
 *     workgroups wait for one another) so that two never interleave on the CUs.  A stream passed
 *     to a call must stay valid until the next call on that device from another stream (or a
 *     device synchronisation): the order is recorded on it lazily.
 */
#ifndef NPR_H
#define NPR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NPR_ABI_VERSION 5

/* ---- status of an API call ------------------------------------------------------------ */
typedef enum npr_status {
  NPR_OK = 0,
  NPR_INCOMPLETE = 1,      /* crate::errors::Error::Incomplete  (src/errors.rs:5)  */
  NPR_FAILURE = 2,         /* crate::errors::Error::Failure     (src/errors.rs:7)  */
  NPR_CUSTOM = 3,          /* crate::errors::Error::Custom      (src/errors.rs:9)  */
  NPR_ERR_ARG = -1,        /* bad argument (null pointer, misaligned device buffer, ...) */
  NPR_ERR_DEVICE = -2,     /* HIP runtime error; see npr_ctx_last_error() */
  NPR_ERR_CAPACITY = -3,   /* an output array was too small; counts are still exact */
  NPR_ERR_TIMEOUT = -4,    /* tile hand-off did not complete (guard against a stalled grid) */
  NPR_ERR_NOMEM = -5
} npr_status;

/* nom::Endianness as chosen by GlobalHeader::parse (src/global_header.rs:43-53) */
typedef enum npr_endianness { NPR_LITTLE = 0, NPR_BIG = 1 } npr_endianness;

/* GlobalHeader (src/global_header.rs:13-23) */
typedef struct npr_global_header {
  int32_t endianness; /* npr_endianness */
  uint16_t version_major;
  uint16_t version_minor;
  int32_t zone;
  int32_t sig_figs;
  uint32_t snap_length;
  uint32_t network;
} npr_global_header;

/* PcapRecord (src/record.rs:59-65).  `payload` = input[offset+16 .. offset+16+actual_length];
 * timestamp = UNIX_EPOCH + ts_sec s + ts_usec us (convert_packet_time, src/record.rs:82-86). */
typedef struct npr_record {
  uint64_t offset;          /* byte offset of the 16-B record header in the input */
  uint32_t ts_sec;
  uint32_t ts_usec;
  uint32_t actual_length;   /* incl_len */
  uint32_t original_length; /* orig_len */
} npr_record;

/* Flow (src/flow/mod.rs:53-61) in a fixed 32-byte encoding.
 *   layer2 is always Ethernet (the only info::layer2::Id, src/flow/info.rs:8-10).
 *   kind bit0: layer3  0 = IPv4, 1 = IPv6      (info::layer3::Id; Arp never yields a flow)
 *   kind bit1: layer4  0 = Tcp,  1 = Udp       (info::layer4::Id; Vxlan is never produced)
 *   src_ip/dst_ip: the 4 address bytes in packet order for IPv4; 0 for IPv6, whose 16-byte
 *   addresses live in npr_flow_v6 at the same index.
 *   record_offset: 40-bit little-endian byte offset of the flow's record header (the
 *   `PcapRecord` half of convert_records' `(PcapRecord, Flow)` pair). */
typedef struct npr_flow {
  uint8_t src_ip[4];
  uint8_t dst_ip[4];
  uint16_t src_port;
  uint16_t dst_port;
  uint16_t vlan;
  uint8_t src_mac[6];
  uint8_t dst_mac[6];
  uint8_t kind;
  uint8_t record_offset[5];
} npr_flow;

typedef struct npr_flow_v6 {
  uint8_t src_ip[16];
  uint8_t dst_ip[16];
} npr_flow_v6;

#define NPR_FLOW_KIND_IPV6 0x1u
#define NPR_FLOW_KIND_UDP 0x2u

/* Per-record result of extract_flow: one code per leaf of the reference's error tree
 * flow::errors::Error (src/flow/errors.rs:5-19) and its per-layer `errors` modules. */
typedef enum npr_flow_status {
  NPR_FLOW_OK = 0,
  /* Error::NetParser(e): Ethernet::parse failed (src/flow/mod.rs:28-31) */
  NPR_FLOW_ETH_INCOMPLETE = 1, /* e = Incomplete: < 14 B, or a truncated 802.1Q/ad tag  */
  NPR_FLOW_ETH_FAILURE = 2,    /* e = Failure: unknown EtherType (src/layer2/ethernet.rs:57-73) */
  /* Error::L2(Ethernet(EthernetType{..})): LLDP or an 802.3 length (src/flow/layer2/ethernet.rs:125-130) */
  NPR_FLOW_L2_ETHERTYPE = 3,
  /* Error::L2(Ethernet(NetParser{l3, err})) */
  NPR_FLOW_L2_IPV4_INCOMPLETE = 4,
  NPR_FLOW_L2_IPV4_FAILURE = 5, /* unknown protocol id (src/layer3/mod.rs:54-72) */
  NPR_FLOW_L2_IPV4_CUSTOM = 6,  /* version != 4 (src/layer3/ipv4.rs:156) */
  NPR_FLOW_L2_IPV6_INCOMPLETE = 7,
  NPR_FLOW_L2_IPV6_FAILURE = 8,
  NPR_FLOW_L2_IPV6_CUSTOM = 9,
  NPR_FLOW_L2_ARP_INCOMPLETE = 10,
  /* Error::L2(Ethernet(Incomplete{l3, size})): bytes left after the L3 parse */
  NPR_FLOW_L2_IPV4_REMAINDER = 11,
  NPR_FLOW_L2_IPV6_REMAINDER = 12,
  NPR_FLOW_L2_ARP_REMAINDER = 13,
  /* Error::L3(Arp(Flow)) (src/flow/layer3/arp.rs:23-27) */
  NPR_FLOW_L3_ARP = 14,
  /* Error::L3(IPv4|IPv6(InternetProtocolId{id})): neither TCP nor UDP */
  NPR_FLOW_L3_IPV4_PROTOCOL = 15,
  NPR_FLOW_L3_IPV6_PROTOCOL = 16,
  /* Error::L3(IPv4|IPv6(NetParser{l4, err})) */
  NPR_FLOW_L3_IPV4_TCP_INCOMPLETE = 17,
  NPR_FLOW_L3_IPV4_TCP_FAILURE = 18, /* data offset outside [20, 60] (src/layer4/tcp.rs:68-82) */
  NPR_FLOW_L3_IPV4_UDP_INCOMPLETE = 19,
  NPR_FLOW_L3_IPV6_TCP_INCOMPLETE = 20,
  NPR_FLOW_L3_IPV6_TCP_FAILURE = 21,
  NPR_FLOW_L3_IPV6_UDP_INCOMPLETE = 22,
  /* Error::L3(IPv4|IPv6(Incomplete{l4: Udp, size})): UDP length != L3 payload length */
  NPR_FLOW_L3_IPV4_UDP_REMAINDER = 23,
  NPR_FLOW_L3_IPV6_UDP_REMAINDER = 24,
  NPR_FLOW_STATUS_COUNT = 25
} npr_flow_status;

/* The payload the reference's error variant carries for each per-record status (npr_flow_details):
 *   *_INCOMPLETE (nom level, crate::errors::Error::Incomplete{size}) -> the failing primitive's
 *       Needed::Size (nom 4.2: a be_u16 needs 2, take!(k) needs k; UDP lengths below 8 wrap as the
 *       reference's usize does, src/layer4/udp.rs:40);
 *   *_REMAINDER (flow-level Incomplete{size: rem.len()}, src/flow/layer2/ethernet.rs:67-76,
 *       src/flow/layer3/ipv4.rs:59-70) -> the bytes left after the layer's parse;
 *   *_FAILURE (map_opt! / map_res!, msg "Error: Code(<input>, MapOpt|MapRes)") -> start | end << 32:
 *       the frame offsets (from the payload start) of the failing primitive's input and of its
 *       parser's input end (the frame's end, or the IP payload's for TCP);
 *   *_CUSTOM ("Expected version 4, was {}") -> the version nibble;
 *   NPR_FLOW_L2_ETHERTYPE -> the EtherType (LLDP, or an 802.3 length);
 *   NPR_FLOW_L3_*_PROTOCOL -> the IP protocol id;  NPR_FLOW_OK, NPR_FLOW_L3_ARP -> 0. */

/* VXLAN inner flows (row f3; off the reference's flow path, which never produces a Vxlan flow,
 * quirk Q13): the outer frame's UDP payload parsed as Vxlan::parse (src/layer4/vxlan.rs:31-48),
 * then the inner Ethernet frame's flow as <Vxlan as FlowExtraction>::extract_flow
 * (src/flow/layer4/vxlan.rs:32-50).  Per-record status: an outer failure keeps its
 * flow status code, 1..24; then: */
enum {
  NPR_VXLAN_NOT_UDP = 32,    /* the outer flow is Ok but TCP */
  NPR_VXLAN_PORT = 33,       /* the outer UDP destination port is not the one asked for */
  NPR_VXLAN_INCOMPLETE = 34, /* the UDP payload is shorter than the 8-B VXLAN header (Incomplete) */
  NPR_VXLAN_INNER = 64       /* + the inner frame's flow status code, 1..24: the inner flow failed */
};

/* Totals written by the device at the end of a parse.  `consumed` is where the record
 * chain stopped: the Rust remainder slice is input[consumed..] (src/record.rs:51). */
typedef struct npr_summary {
  uint64_t n_records;
  uint64_t n_flows;
  uint64_t consumed;
  uint32_t flags; /* NPR_SUMMARY_* */
  uint32_t epoch;
  uint64_t entry; /* offset of the chain's first record (start, or the speculated one of a
                     speculative-start range; NPR_NO_ENTRY when none was found) */
} npr_summary;

#define NPR_NO_ENTRY 0xFFFFFFFFFFFFFFFFull

#define NPR_SUMMARY_RECORD_OVERFLOW 0x1u /* record_cap too small */
#define NPR_SUMMARY_FLOW_OVERFLOW 0x2u   /* flow_cap too small */

/* Device-resident outputs of npr_dev_parse_extract.  Any array may be NULL (not produced).
 *   record_offsets/records/record_status: dense, file order (PcapRecords::parse order);
 *   `records` is the full PcapRecord row, `record_offsets` just its offset.
 *   flows/flows_v6: convert_records order (reverse file order, Ok flows only,
 *   src/flow/mod.rs:101-123), RIGHT-ALIGNED: the valid range is
 *   [flow_cap - n_flows, flow_cap).  flows_v6[i] is written only when flows[i] is IPv6.
 *   summary: device pointer, always written. */
typedef struct npr_dev_outputs {
  uint64_t *record_offsets;
  npr_record *records;
  uint8_t *record_status;
  uint64_t record_cap;
  npr_flow *flows;
  npr_flow_v6 *flows_v6;
  uint64_t flow_cap;
  npr_summary *summary;
} npr_dev_outputs;

/* ---- library / context ---------------------------------------------------------------- */
typedef struct npr_ctx npr_ctx;

const char *npr_version(void);
int npr_abi_version(void);
/* Create a context on HIP device `device` (one stream, workspaces grown on demand). */
npr_status npr_ctx_create(int device, npr_ctx **out);
void npr_ctx_destroy(npr_ctx *ctx);
const char *npr_ctx_last_error(const npr_ctx *ctx);
/* Call before destroying a HIP stream that was passed to any npr_dev_* call (of any context on the
 * device).  libnpr orders the look-back launches of all contexts on a device; the order event of the
 * last launch is recorded lazily on that launch's stream (an eager record costs ~3 us of GPU time
 * per launch), so a destroyed stream must hand its pending record over first.  The context's own
 * stream needs no call (npr_ctx_destroy does it). */
npr_status npr_stream_release(npr_ctx *ctx, void *stream);
/* Diagnostics: per-launch speculation / hand-off counters (off by default; costs atomics).
 * Counters: [0] tiles pass 2 re-walked (pass 1's entry was not the exact one), [1] prefix folds
 * that waited for a mis-speculated tile's exact prefix, [3] sparse-walk scan rounds (resolving
 * contradicted lane groups), [4] sparse resolve passes whose shared re-walk queue was full (tasks
 * deferred to the next pass), [5] tiles with no plausible record start, [6] (stats mode 2 only)
 * resident look-back re-read rounds summed over workgroups; [7] is reserved (0).  In the sparse
 * walk [0] counts lane re-walks. */
npr_status npr_ctx_set_stats(npr_ctx *ctx, int enable);
npr_status npr_ctx_read_stats(npr_ctx *ctx, uint32_t *out, int n, int reset);
/* With npr_ctx_set_stats(ctx, 2): s_memrealtime (100 MHz) stamps of the last parse, 16 words
 * per row (the buffer holds one row per tile).
 * Resident pass (flows-only launches): row v = persistent wave v: [0] start [1] first tile landed
 *   [2] phase A done [3] range aggregate published + workgroup fold [4] prefix known [5] kept
 *   flows written [6] done; [8] tiles [9] kept rounds [10] deferred tiles [11] 1 = fast path;
 *   the first wave of each workgroup also [12] look-back start [13] lower aggregates all landed
 *   [14] workgroup prefix folded (scripts/res_stamps.py reads them).
 * Two-pass kernels: row t = tile t: pass 1 [0] tile start [1] entry known [2] walked [3] counted
 *   [4] published; pass 2 [5] tile start [6] record offsets known [7] written; on the first tile
 *   of a wave's chunk: [8] pass-2 entry [9] prologue issued [10] prefix known [11]/[12] pass-1
 *   group arrival start/end.
 * out may be NULL with cap 0 to query *n_tiles only. */
npr_status npr_ctx_read_stamps(npr_ctx *ctx, uint64_t *out, uint64_t cap, uint64_t *n_tiles);
/* Context options.
 * NPR_OPT_RESIDENT (default 1; env NPR_RESIDENT=0 sets 0 at create): a flows-only device parse
 *   (no record table / offsets / status requested) runs the resident single pass: one launch that
 *   reads the capture once and keeps each wave's decoded flows in registers until the exact
 *   convert_records rows are known.  0 (and every launch that asks for a record table, offsets or
 *   status) runs the two-pass kernels; N > 1 caps the resident pass at N waves (longer ranges per
 *   wave: a test knob).  Same results either way.
 * NPR_OPT_STREAM_CHUNK (KiB, default 0 = off): npr_parse_extract without a record table
 *   copies a capture of more than two chunks to the device in chunks on a second stream and
 *   launches each chunk's chained parse as soon as it (and the next chunk) has landed, so the
 *   H2D copy overlaps the parse.  Results are those of the unchunked parse: a record longer than
 *   a chunk ends a link early, which the call detects and answers by parsing the staged capture
 *   again in one go.  Off by default: from pageable host memory the chunked copies measured
 *   slower than one copy, and the copy is ~50x the parse, so overlap gains little.
 * NPR_OPT_PARK_FLOWS: accepted for ABI 2 callers, no effect.
 * NPR_OPT_PIPE: the pipelined resident pass was an experiment that measured slower
 *   and is not in this library: 0 is accepted, 1 returns NPR_ERR_ARG.
 * NPR_OPT_DEVICE_WINDOW (chunks, default 0 = auto): npr_parse_extract_pipelined keeps at most N
 *   chunks of the capture (a ring, plus a 260 KiB halo for records that straddle a chunk end) and
 *   3 links' flow rows on the device, so a host capture larger than device memory streams through
 *   it.  N >= 3 uses the window whenever the capture has more than N chunks; 0 uses a window of 8
 *   chunks only when staging the whole capture and its flow table would not fit in free device
 *   memory.  Same results as the staged call, except that a record longer than the halo cannot
 *   cross a chunk end in the window: the call then returns NPR_ERR_CAPACITY (a pcap snaplen is at
 *   most 262144 B, which the halo covers).  Windowed chunks are at least 512 KiB.
 * NPR_OPT_SPARSE (default 0 = auto): flows-only parses of captures of long records run the sparse
 *   record walk instead of the resident pass: lanes hop header to header and read
 *   one 112-B window per record instead of streaming every payload byte.  0 chooses it from the
 *   record density of the capture's first 256 KiB (at least 256 MiB past `start`, a known start, no
 *   shard); 1 never; 2 always (lane ranges sized from the density, else 16 KiB); N >= 64 always,
 *   with lane ranges of min(N, 256 KiB) bytes (a test knob).  Same results either way.
 * NPR_OPT_SPARSE_CAP (default 0 = 96): record slots per sparse lane; a lane with more records
 *   walks the rest again when its rows are written (a test knob; 1 .. 128).
 */
enum { NPR_OPT_PARK_FLOWS = 1, NPR_OPT_RESIDENT = 2, NPR_OPT_STREAM_CHUNK = 3, NPR_OPT_PIPE = 4,
       NPR_OPT_DEVICE_WINDOW = 5, NPR_OPT_SPARSE = 6, NPR_OPT_SPARSE_CAP = 7 };
npr_status npr_ctx_set_option(npr_ctx *ctx, int option, int value);
/* Which pass the context's last device parse launch ran (tests and diagnostics; no reference
 * counterpart): 0 none yet, 1 the two-pass kernels, 2 the resident single pass, 8 the sparse
 * record walk (4, a batched resident launch, is no longer produced). */
int npr_ctx_last_pass(const npr_ctx *ctx);
/* The flows-only device parse chooses its pass (and its link sizes) by the record density of the
 * capture's first 256 KiB, remembered per (device address, start, stop, byte order) so that a
 * capture parsed again costs no probe.  Call this when new bytes replace a capture at the same
 * address (NULL: forget every capture).  Without the call the choice still follows the bytes one
 * parse late: npr_dev_check corrects a remembered density that is more than 2x off the parse's own.
 * The host entry points forget their staging buffer's density whenever they stage new bytes.
 * The choice never changes a result, only the time. */
npr_status npr_ctx_forget_density(npr_ctx *ctx, const void *input);
/* Bytes of device workspace the next parse of `len` bytes needs (tile hand-off slots). */
uint64_t npr_workspace_bytes(uint64_t len);

/* ---- host-side, single objects (no device work: 24 B / 16 B) ----------------------------- */
/* GlobalHeader::parse (src/global_header.rs:40-70). *consumed = 24 on success. */
npr_status npr_global_header_parse(const uint8_t *input, size_t len, npr_global_header *out,
                                   size_t *consumed);
/* PcapRecord::parse (src/record.rs:102-121). *consumed = 16 + actual_length. */
npr_status npr_record_parse(const uint8_t *input, size_t len, npr_endianness endianness,
                            npr_record *out, size_t *consumed);

/* ---- host-side per-layer header objects (the reference's public layer parsers) ------------------
 * Each parses ONE header object from `input` as its reference function does (the nom chain step by
 * step, with the reference's release-build wrapping arithmetic).  No device work: these are the
 * object API for callers that inspect frames; the flows of whole captures come from the device.
 * Byte ranges of `input` (the reference's borrowed slices) are {offset, length} pairs.  Returns
 *   NPR_OK: `*out` filled, *consumed = the bytes the parser used (its remainder is input[*consumed..]);
 *   NPR_INCOMPLETE: *detail = nom's Needed::Size of the failing primitive (be_u16: 2, take!(k): k);
 *   NPR_FAILURE: a map_opt! / map_res! failed; *detail = start | end << 32, the offsets in `input`
 *     of the failing primitive's input and of its end (nom's Context::Code input slice);
 *   NPR_CUSTOM: the IP version check failed; *detail = the version nibble.
 * `consumed` and `detail` may be NULL. */
/* VlanTag (src/layer2/ethernet.rs:85-98): prio and dei are the reference's `(total & 0x7000) as u8`
 * and `(total & 0x8000) as u8`, i.e. always 0. */
typedef struct npr_vlan_tag {
  uint16_t vlan_type;  /* VlanTypeId::value(): 0x8100 or 0x88A8 */
  uint16_t vlan_value; /* the tag's 16 bits */
  uint8_t prio;
  uint8_t dei;
  uint16_t id;         /* vlan_value & 0x0FFF */
} npr_vlan_tag;
/* Ethernet (src/layer2/ethernet.rs:100-107) */
typedef struct npr_ethernet {
  uint8_t dst_mac[6];
  uint8_t src_mac[6];
  uint16_t ether_type; /* EthernetTypeId::value(): an 802.3 length (<= 1500) or 0x0800 / 0x86DD / 0x0806 / 0x88CC */
  uint16_t reserved;
  uint32_t n_vlans;    /* the frame's VLAN tags, outermost first; the first min(n_vlans, vlan_cap) go to `vlans` */
  uint64_t payload_offset, payload_length;
} npr_ethernet;
/* Ethernet::parse (src/layer2/ethernet.rs:204-216).  More tags than vlan_cap: NPR_ERR_CAPACITY with
 * the exact n_vlans (the other fields filled). */
npr_status npr_ethernet_parse(const uint8_t *input, size_t len, npr_ethernet *out, npr_vlan_tag *vlans,
                              size_t vlan_cap, size_t *consumed, uint64_t *detail);
/* IPv4 (src/layer3/ipv4.rs:14-29).  options / padding: length 0 = None (the reference's cond! takes
 * them only when they are non-empty). */
typedef struct npr_ipv4 {
  uint8_t version_and_length;
  uint8_t tos;
  uint16_t raw_length;
  uint16_t id;
  uint16_t flags;
  uint8_t ttl;
  uint8_t protocol;    /* InternetProtocolId::value() */
  uint16_t checksum;
  uint8_t src_ip[4];
  uint8_t dst_ip[4];
  uint64_t payload_offset, payload_length;
  uint64_t options_offset, options_length;
  uint64_t padding_offset, padding_length;
} npr_ipv4;
/* IPv4::parse (src/layer3/ipv4.rs:148-160) + parse_ipv4 (:76-146) */
npr_status npr_ipv4_parse(const uint8_t *input, size_t len, npr_ipv4 *out, size_t *consumed, uint64_t *detail);
/* IPv6 (src/layer3/ipv6.rs:10-16) */
typedef struct npr_ipv6 {
  uint8_t dst_ip[16];
  uint8_t src_ip[16];
  uint8_t protocol;    /* the first next header that has no next option (InternetProtocolId::value()) */
  uint8_t reserved[7];
  uint64_t payload_offset, payload_length;
} npr_ipv6;
/* IPv6::parse (src/layer3/ipv6.rs:87-99): one byte per "extension" header (quirk Q11). */
npr_status npr_ipv6_parse(const uint8_t *input, size_t len, npr_ipv6 *out, size_t *consumed, uint64_t *detail);
/* Arp (src/layer3/arp.rs:7-14) */
typedef struct npr_arp {
  uint8_t sender_ip[4];
  uint8_t sender_mac[6];
  uint8_t target_ip[4];
  uint8_t target_mac[6];
  uint16_t operation;
} npr_arp;
/* Arp::parse (src/layer3/arp.rs:54-76) */
npr_status npr_arp_parse(const uint8_t *input, size_t len, npr_arp *out, size_t *consumed, uint64_t *detail);
/* Tcp (src/layer4/tcp.rs:11-30) with its HeaderLengthAndFlags */
typedef struct npr_tcp {
  uint16_t src_port;
  uint16_t dst_port;
  uint32_t sequence_number;
  uint32_t acknowledgement_number;
  uint16_t header_length_and_flags; /* HeaderLengthAndFlags::inner */
  uint16_t flags;                   /* inner & 0x01FF */
  uint32_t header_length;           /* (inner >> 12) * 4, in [20, 60] */
  uint16_t window;
  uint16_t check;
  uint16_t urgent;
  uint16_t reserved;
  uint64_t options_offset, options_length;
  uint64_t payload_offset, payload_length;
} npr_tcp;
/* Tcp::parse (src/layer4/tcp.rs:59-101) */
npr_status npr_tcp_parse(const uint8_t *input, size_t len, npr_tcp *out, size_t *consumed, uint64_t *detail);
/* Udp (src/layer4/udp.rs:10-16) */
typedef struct npr_udp {
  uint16_t src_port;
  uint16_t dst_port;
  uint16_t checksum;
  uint16_t reserved;
  uint64_t payload_offset, payload_length;
} npr_udp;
/* Udp::parse (src/layer4/udp.rs:33-50): the payload is take!(length - 8) with the reference's usize
 * arithmetic, so a length field below 8 asks for ~2^64 bytes (NPR_INCOMPLETE, *detail = that size). */
npr_status npr_udp_parse(const uint8_t *input, size_t len, npr_udp *out, size_t *consumed, uint64_t *detail);
/* Vxlan (src/layer4/vxlan.rs:7-14) */
typedef struct npr_vxlan {
  uint16_t flags;
  uint16_t group_policy_id;
  uint32_t raw_network_identifier;
  uint32_t network_identifier;      /* raw >> 8 */
  uint32_t reserved;
  uint64_t payload_offset, payload_length;
} npr_vxlan;
/* Vxlan::parse (src/layer4/vxlan.rs:31-48): u16! u16! u32! in `endianness`, then the rest. */
npr_status npr_vxlan_parse(const uint8_t *input, size_t len, npr_endianness endianness, npr_vxlan *out,
                           size_t *consumed, uint64_t *detail);

/* ---- host-memory entry points (stage to HBM, run the device path, copy back) ------------- */
/* PcapRecords::parse (src/record.rs:21-54): records from byte 0, stop at the first Incomplete.
 * Writes up to `cap` records; *n_out = total found (> cap => NPR_ERR_CAPACITY). */
npr_status npr_records_parse(npr_ctx *ctx, const uint8_t *input, size_t len,
                             npr_endianness endianness, npr_record *out, size_t cap,
                             size_t *n_out, size_t *consumed);
/* CaptureFile::parse (src/file.rs:14-35) == net_parser_rs::parse (src/lib.rs:44-46). */
npr_status npr_capture_file_parse(npr_ctx *ctx, const uint8_t *input, size_t len,
                                  npr_global_header *header, npr_record *out, size_t cap,
                                  size_t *n_out, size_t *consumed);
/* FlowExtraction::extract_flow (src/flow/mod.rs:20-48) for a batch of records: dense
 * per-record status + flow (flow/flow_v6 rows of failed records are zero). `input` is the
 * buffer the records' offsets index into. flows_v6 may be NULL. */
npr_status npr_extract_flows(npr_ctx *ctx, const uint8_t *input, size_t len,
                             const npr_record *records, size_t n, npr_flow *flows,
                             npr_flow_v6 *flows_v6, uint8_t *status);
/* flow::convert_records (src/flow/mod.rs:101-123): Ok flows in reverse record order.
 * *n_out = number of flows (> cap => NPR_ERR_CAPACITY, nothing beyond cap written).
 * out_v6[i] (optional) is written only when out[i] is IPv6. */
npr_status npr_convert_records(npr_ctx *ctx, const uint8_t *input, size_t len,
                               const npr_record *records, size_t n, npr_flow *out,
                               npr_flow_v6 *out_v6, size_t cap, size_t *n_out);
/* The reference's `extract` bench step (benches/benches.rs:56-62) fused into one device
 * pass: CaptureFile::parse + convert_records.  `records` (optional, may be NULL) receives
 * the dense record table; `out`/`out_v6` the converted flows (left-aligned here). */
npr_status npr_parse_extract(npr_ctx *ctx, const uint8_t *input, size_t len,
                             npr_global_header *header, npr_record *records, size_t record_cap,
                             size_t *n_records, npr_flow *out, npr_flow_v6 *out_v6,
                             size_t flow_cap, size_t *n_flows, size_t *consumed);

/* The same `extract` step with the PCIe transfers pipelined (row f1; the north star's end-to-end
 * path): the capture goes to the device in chunks of `chunk_bytes` (0 = 32 MiB) by page-locked
 * DMA on one stream; each chunk's chained parse launches as soon as it (and the next chunk, for
 * records that straddle) has landed; each launch's flow rows go back on a third stream while
 * later chunks still upload (PCIe is full duplex).  Caller buffers that are not page-locked
 * (npr_host_alloc, or registered by the caller) are registered for the call.  The flows land
 * RIGHT-aligned, the device table's own layout: out[flow_cap - *n_flows .. flow_cap) in
 * convert_records order, so no pass moves them afterwards.  A record longer than a chunk ends a
 * link early; the call detects that and parses the staged capture again in one go.  Results
 * equal npr_parse_extract's.  A capture larger than free device memory (or than
 * NPR_OPT_DEVICE_WINDOW chunks) streams through a bounded device window instead of being staged
 * whole. */
npr_status npr_parse_extract_pipelined(npr_ctx *ctx, const uint8_t *input, size_t len,
                                       npr_global_header *header, npr_flow *out, npr_flow_v6 *out_v6,
                                       size_t flow_cap, size_t *n_flows, size_t *consumed,
                                       uint64_t chunk_bytes);
/* Page-locked host memory for captures and flow tables (hipHostMalloc): the DMA engines read and
 * write it at full PCIe rate, with no per-call registration. */
npr_status npr_host_alloc(npr_ctx *ctx, size_t bytes, void **out);
npr_status npr_host_free(npr_ctx *ctx, void *p);

/* ---- device-resident entry points ------------------------------------------------------- */
/* The hot path: one launch finds the record chain starting at `start` (24 for a capture
 * file, 0 for bare records), decodes every record and writes the outputs described in
 * npr_dev_outputs.  `input` is a 16-byte-aligned device pointer; `stream` a hipStream_t
 * (NULL = the context's stream).  Asynchronous: read `summary` after the stream syncs,
 * or call npr_dev_check() which also reports NPR_ERR_CAPACITY / NPR_ERR_TIMEOUT.
 * A flows-only parse of a capture larger than one resident launch holds (about 80 MB on MI355X)
 * runs as npr_dev_parse_extract_chunked. */
npr_status npr_dev_parse_extract(npr_ctx *ctx, const void *input, uint64_t len, uint64_t start,
                                 npr_endianness endianness, const npr_dev_outputs *out,
                                 void *stream);
/* Byte-range form for sharding one capture: only records that START in
 * [start, stop) are produced, while payloads may run past `stop` up to `len`.  With
 * speculative_start != 0, `start` is not known to be a record boundary: the first plausible
 * record start at or after it is speculated and reported in summary->entry.  The caller checks
 * it against the previous range's `consumed` and reruns with that exact start when they
 * differ.  `ref_record` is the offset of a known record header (the capture's first, 24)
 * whose ts_sec anchors the speculation, or NPR_NO_ENTRY.
 * npr_dev_parse_extract(start) == this with stop = len, speculative_start = 0, ref = start. */
npr_status npr_dev_parse_extract_range(npr_ctx *ctx, const void *input, uint64_t len, uint64_t start,
                                       uint64_t stop, npr_endianness endianness, int speculative_start,
                                       uint64_t ref_record, const npr_dev_outputs *out, void *stream);
/* Chained form (the resident single pass; flows-only outputs): continue the record chain, the
 * record count and the flow rows where the launch that wrote `prev` left them (`prev` a device
 * npr_summary of an earlier launch on this context; NULL = `start` is an exact record start).
 * Records that START in [start, stop) are produced; their Ok flows go to the convert_records rows
 * after prev's; *out->summary is cumulative.  A capture split at any byte boundaries and parsed
 * chunk after chunk this way equals one npr_dev_parse_extract of the whole. */
npr_status npr_dev_parse_extract_chain(npr_ctx *ctx, const void *input, uint64_t len, uint64_t start,
                                       uint64_t stop, npr_endianness endianness, const npr_summary *prev,
                                       uint64_t ref_record, const npr_dev_outputs *out, void *stream);
/* npr_dev_parse_extract in chunks of about `chunk_bytes` (0: what one launch keeps in registers,
 * about 80 MB on MI355X), chained on the device with no host synchronisation: captures of any size
 * at the single-launch rate.  Launches that need a record table / offsets / status run the
 * two-pass kernels in one launch instead. */
npr_status npr_dev_parse_extract_chunked(npr_ctx *ctx, const void *input, uint64_t len, uint64_t start,
                                         npr_endianness endianness, const npr_dev_outputs *out,
                                         uint64_t chunk_bytes, void *stream);
/* One shard of a capture held by this device (multi-GPU record-range sharding):
 * `input` holds FILE bytes [base, base + input_len).  Records that START in [start, stop) are
 * produced; every offset in the outputs (record offsets, summary->consumed / ->entry) is a file
 * offset.  The serial chain of PcapRecords::parse (src/record.rs:30-49) crosses shard boundaries:
 * rank r's exact first record is rank r-1's `consumed`, which the caller learns from one
 * exchange and checks against summary->entry (speculative_start != 0 lets this shard start
 * before it is known).  `input` must extend past `stop` to the end of the last record starting
 * before it (or to the end of the file): a chain that stops before `stop` in a buffer that ends
 * before the file does means the halo was too short, which the caller checks.
 * A shard's buffer does not hold the global header, so the speculation context comes from the
 * caller: usec_magic (the file's magic is 0xA1B2C3D4 in either byte order: ts_usec < 1e6) and
 * ts_ref (ts_sec of any record of the file, NPR_NO_ENTRY = none).  Flows-only outputs run as
 * chained resident launches of about chunk_bytes (0 = one launch's register capacity). */
typedef struct npr_shard {
  uint64_t base;
  uint64_t start;
  uint64_t stop;
  int32_t speculative_start;
  int32_t usec_magic;
  uint64_t ts_ref;
  uint64_t chunk_bytes;
} npr_shard;

npr_status npr_dev_parse_extract_shard(npr_ctx *ctx, const void *input, uint64_t input_len,
                                       npr_endianness endianness, const npr_shard *shard,
                                       const npr_dev_outputs *out, void *stream);
/* Several independent device-resident captures (e.g. consecutive capture batches of a stream) in one
 * call: each item is what npr_dev_parse_extract(ctx, input, len, start, endianness, &out, stream)
 * would parse, launched in order on the stream, with the same outputs and summary (check each with
 * npr_dev_check).  (ABI 2 ran flows-only items in one batched launch; it measured 0.96-1.09x of
 * separate launches and was removed) */
typedef struct npr_batch_item {
  const void *input;
  uint64_t len;
  uint64_t start;
  int32_t endianness; /* npr_endianness */
  int32_t reserved;
  npr_dev_outputs out;
} npr_batch_item;

npr_status npr_dev_parse_extract_batch(npr_ctx *ctx, const npr_batch_item *items, uint32_t n, void *stream);

/* Synchronise `stream`, copy the summary back and map its flags to a status. */
npr_status npr_dev_check(npr_ctx *ctx, const npr_dev_outputs *out, void *stream,
                         npr_summary *host_summary);
/* Host-memory form of npr_dev_vxlan_flows (synchronous). */
npr_status npr_vxlan_flows(npr_ctx *ctx, const uint8_t *input, size_t len, const npr_record *records, size_t n,
                           uint32_t dst_port, npr_endianness endianness, npr_flow *flows, npr_flow_v6 *flows_v6,
                           uint8_t *status, uint32_t *vni);
/* Per-record status and error payload (see above) of extract_flow over caller records, synchronous;
 * status / detail may be NULL.  The Rust crate calls it only for records whose flow failed. */
npr_status npr_flow_details(npr_ctx *ctx, const uint8_t *input, size_t len, const npr_record *records, size_t n,
                            uint8_t *status, uint64_t *detail);
/* Device form of npr_flow_details, asynchronous on `stream`. */
npr_status npr_dev_flow_details(npr_ctx *ctx, const void *input, uint64_t len, const npr_record *records,
                                uint64_t n, uint8_t *status, uint64_t *detail, void *stream);
/* Dense extract_flow over device-resident records (device npr_record array indexing into
 * `input`; payload = input[offset+16 .. offset+16+actual_length]).  flows[i] / status[i] for every
 * record (a failed record's flow row is zero); flows_v6[i] is written only when flows[i] is IPv6
 * (as in the convert_records tables; the host-memory npr_extract_flows returns zero side rows for
 * the others). */
npr_status npr_dev_extract_flows(npr_ctx *ctx, const void *input, uint64_t len,
                                 const npr_record *records, uint64_t n, npr_flow *flows,
                                 npr_flow_v6 *flows_v6, uint8_t *status, void *stream);
/* The distinct-flow table (row f4; new, not in the reference): one row per distinct
 * {family, protocol, src ip, dst ip, src port, dst port} of a device flow table (flows[0..n),
 * flows_v6 its IPv6 side rows or NULL for an IPv4-only table), in the order of the input rows that
 * first carry it.  out[k] = the flow of its first-seen record (lowest record offset, kept in the
 * row), out_v6[k] its side row, counts[k] = the sum of weights[] over its rows (1 per row when
 * weights is NULL; pass a previous call's counts to merge tables, e.g. one per GPU).  Rows past
 * cap are not written; *n_out (a device word) = the number of distinct flows.  Asynchronous on
 * `stream`; any of out_v6 / counts may be NULL.  Rows that tie on the first-seen offset (a record
 * listed twice, merged tables of several captures) resolve to the lowest input row.  At most 2^30
 * rows per call (NPR_ERR_ARG above). */
npr_status npr_dev_flow_aggregate(npr_ctx *ctx, const npr_flow *flows, const npr_flow_v6 *flows_v6,
                                  const uint64_t *weights, uint64_t n, npr_flow *out, npr_flow_v6 *out_v6,
                                  uint64_t *counts, uint64_t cap, uint64_t *n_out, void *stream);
/* VXLAN inner flows of device-resident records (row f3): dense outputs, row i for record i.
 * flows[i] = the INNER frame's flow with records[i]'s offset when status[i] == NPR_FLOW_OK
 * (zero row otherwise), flows_v6[i] its IPv6 addresses, vni[i] = the VXLAN network identifier
 * (raw u32 >> 8, src/layer4/vxlan.rs:44) when the header was read, else 0.  dst_port = 0 takes
 * every outer UDP flow, else only that destination port (4789 is the IANA VXLAN port).
 * `endianness` is Vxlan::parse's (the reference's tests pass NPR_BIG, src/layer4/vxlan.rs:91).
 * Any output array may be NULL. */
npr_status npr_dev_vxlan_flows(npr_ctx *ctx, const void *input, uint64_t len, const npr_record *records,
                               uint64_t n, uint32_t dst_port, npr_endianness endianness, npr_flow *flows,
                               npr_flow_v6 *flows_v6, uint8_t *status, uint32_t *vni, void *stream);
/* flow::convert_records (src/flow/mod.rs:101-123) over device-resident records, asynchronous on
 * `stream`: rows 0.. of out / out_v6 (device) = the Ok flows in REVERSE record order (rows past
 * cap are not written; out_v6[i] only when out[i] is IPv6), *n_out (a device word) = the number of
 * Ok flows, or UINT64_MAX when the launch's bounded look-back timed out.  One kernel pass
 * (DESIGN.md §3.4). */
npr_status npr_dev_convert_records(npr_ctx *ctx, const void *input, uint64_t len,
                                   const npr_record *records, uint64_t n, npr_flow *out,
                                   npr_flow_v6 *out_v6, uint64_t cap, uint64_t *n_out, void *stream);

/* ---- multi-GPU runtime (no reference counterpart) ------------------------------------------- */
/* The per-step summary exchange of the multi-GPU step on ONE node: `seg` is a
 * mapping, shared by the `world` rank processes, of world x depth slots of `rec` bytes each (slot
 * (r, d) at byte (r * depth + d) * rec: an 8-byte sequence word, the payload from byte 64).  Rank
 * `rank` publishes `mine` (n bytes) as exchange number `seq` (1, 2, ... in every rank's call
 * order) in its slot seq % depth, then waits until every rank's slot holds exchange `seq` and
 * copies the world payloads to out[world][n].  Spins, then yields; NPR_ERR_TIMEOUT after
 * timeout_ms.  depth >= 2: a slot is rewritten only after every rank has read it. */
npr_status npr_shm_all_gather(void *seg, int world, int rank, int depth, uint64_t rec, uint64_t seq,
                              const void *mine, uint64_t n, void *out, int timeout_ms);

#ifdef __cplusplus
}
#endif
#endif /* NPR_H */
