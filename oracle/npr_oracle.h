/*
 * npr_oracle.h — PARITY ORACLE, TEST INFRASTRUCTURE ONLY.
 *
 * A sequential CPU restatement of protectwise/net-parser-rs 0.3.0's parse paths, used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.  The
 * product (libnpr.so) never links, loads or calls anything in this directory.
 *
 * Pinning: the reference is Rust and no Rust toolchain exists in this image (no cargo/rustc,
 * no nom-4.x crate source), so oracle/_ref cannot be built.  The restatement is pinned by
 * every known-answer test the reference's own sources hold (tests/golden/kat.json, made by
 * tests/golden/make_golden.py).  Those KATs pin the success paths; the error-path codes and
 * the streaming Incomplete stop are restated from source and are "parity unpinned".
 *
 * Third-party arithmetic: the byte primitives come from nom "4" (Cargo.toml:16; Cargo.lock is
 * git-ignored, so it resolves to nom 4.2.3).  Semantics used here, all streaming-mode:
 * be_u8/be_u16/be_u32/u32!(e) and take!(n) return Err::Incomplete when fewer bytes remain;
 * map_opt!/map_res! return Err::Error (-> crate::errors::Error::Failure, src/errors.rs:43-47);
 * rest always succeeds; cond!(false, ..) consumes nothing.  Arithmetic follows the RELEASE
 * profile (wrapping u16/usize), which is what benches/benches.rs runs.
 */
#ifndef NPR_ORACLE_H
#define NPR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/npr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* nom result kinds of a single parser */
enum { OR_OK = 0, OR_INCOMPLETE = 1, OR_FAILURE = 2, OR_CUSTOM = 3 };

int or_global_header_parse(const uint8_t *in, size_t len, npr_global_header *out, size_t *consumed);
int or_record_parse(const uint8_t *in, size_t len, int endianness, npr_record *out, size_t *consumed);
/* PcapRecords::parse: returns the number of records (writes at most cap), *consumed = where the
 * chain stopped. Offsets are relative to `in`. */
size_t or_records_parse(const uint8_t *in, size_t len, int endianness, npr_record *out, size_t cap,
                        size_t *consumed);
/* CaptureFile::parse: returns OR_INCOMPLETE when len < 24. Offsets relative to `in`. */
int or_capture_file_parse(const uint8_t *in, size_t len, npr_global_header *hdr, npr_record *out,
                          size_t cap, size_t *n_out, size_t *consumed);
/* FlowExtraction::extract_flow on one record payload; fills flow (+ v6) on NPR_FLOW_OK.
 * record_offset is only stored into flow->record_offset. */
int or_extract_flow(const uint8_t *payload, size_t len, uint64_t record_offset, npr_flow *flow,
                    npr_flow_v6 *v6);
/* or_extract_flow + the payload its error variant carries (npr.h npr_flow_details) */
int or_extract_flow_detail(const uint8_t *payload, size_t len, uint64_t record_offset, npr_flow *flow,
                           npr_flow_v6 *v6, uint64_t *detail);
/* flow::convert_records: returns the number of flows (writes at most cap). */
size_t or_convert_records(const uint8_t *buf, size_t len, const npr_record *recs, size_t n,
                          npr_flow *out, npr_flow_v6 *out_v6, size_t cap);
/* Dense extract over a record list (status per record). */
void or_extract_flows(const uint8_t *buf, size_t len, const npr_record *recs, size_t n,
                      npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status);

/* Per-record status + the payload its error variant carries (include/npr.h npr_flow_details). */
void or_flow_details(const uint8_t *buf, size_t len, const npr_record *recs, size_t n, uint8_t *status,
                     uint64_t *detail);

/* row f3: Vxlan::parse (src/layer4/vxlan.rs:31-48) and the VXLAN inner flow */
typedef struct or_vxlan {
  uint16_t flags, group_policy_id;
  uint32_t raw_network_identifier, network_identifier;
  size_t payload_off;
} or_vxlan;
int or_vxlan_parse(const uint8_t *in, size_t n, int big, or_vxlan *v);
int or_vxlan_flow(const uint8_t *p, size_t n, uint64_t record_offset, uint32_t dst_port, int big, npr_flow *f,
                  npr_flow_v6 *v6, uint32_t *vni);
void or_vxlan_flows(const uint8_t *buf, size_t len, const npr_record *recs, size_t n, uint32_t dst_port, int big,
                    npr_flow *flows, npr_flow_v6 *flows_v6, uint8_t *status, uint32_t *vni);

/* ---- layer-level parsers (pinned individually by the reference's layer KATs) ---- */
typedef struct {
  const uint8_t *dst_mac, *src_mac;
  uint16_t ether_type; /* first non-VLAN EtherType */
  uint16_t vlan;       /* vlans_to_vlan: first (outermost) tag id, else 0 */
  uint32_t n_vlans;
  size_t payload_off;  /* payload = rest */
} or_eth;
typedef struct {
  const uint8_t *src, *dst; /* 4 (IPv4) or 16 (IPv6) bytes */
  uint8_t protocol;
  size_t payload_off, payload_len, rem;
} or_ip;
typedef struct {
  uint16_t operation;
  const uint8_t *sender_mac, *sender_ip, *target_mac, *target_ip;
  size_t rem;
} or_arp;
typedef struct {
  uint16_t src_port, dst_port;
  size_t header_length; /* TCP only */
  size_t payload_off, payload_len, rem;
} or_l4;
int or_eth_parse(const uint8_t *in, size_t n, or_eth *v);
int or_ipv4_parse(const uint8_t *in, size_t n, or_ip *v);
int or_ipv6_parse(const uint8_t *in, size_t n, or_ip *v);
int or_arp_parse(const uint8_t *in, size_t n, or_arp *v);
int or_tcp_parse(const uint8_t *in, size_t n, or_l4 *v);
int or_udp_parse(const uint8_t *in, size_t n, or_l4 *v);
size_t or_tcp_extract_length(uint16_t value);

/* Bench leg: CaptureFile::parse + convert_records on one buffer (benches/benches.rs:56-62).
 * Returns flows; *n_records = records parsed. Scratch arrays supplied by the caller. */
size_t or_bench_extract(const uint8_t *in, size_t len, npr_record *rec_scratch, size_t rec_cap,
                        npr_flow *flow_scratch, npr_flow_v6 *v6_scratch, size_t flow_cap,
                        size_t *n_records);

/* The same on `nthreads` host threads (serial chain walk, parallel extract_flow, reverse-order
 * rows from per-thread Ok counts).  dense / dense6 / status: n-record scratch. */
size_t or_bench_extract_mt(const uint8_t *in, size_t len, npr_record *rec_scratch, size_t rec_cap,
                           npr_flow *dense, npr_flow_v6 *dense6, uint8_t *status, npr_flow *out,
                           npr_flow_v6 *out6, size_t flow_cap, size_t *n_records, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
