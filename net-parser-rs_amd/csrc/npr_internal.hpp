// npr_internal.hpp — interface between the C-ABI layer (npr_capi.hip) and the kernels
// (npr_kernels.hip).  Not installed; the public boundary is include/npr.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/npr.h"

namespace npr {

// Tile geometry of the parse+extract kernels: ONE WAVE per tile.
constexpr int kBlock = 256;            // workgroup size of the auxiliary kernels (dense extract, compaction)
constexpr int kWave = 64;              // lanes per wave (the two-pass kernels: one-wave workgroups)
constexpr int kTile = 4096;            // bytes of the record stream owned by one tile (one wave; 8 KiB: DESIGN.md §5)
constexpr int kHalo = 128;             // bytes staged past the tile (headers + fast-decode window of straddlers)
constexpr int kStage = kTile + kHalo;  // bytes staged in LDS per tile
constexpr int kMaxRec = kTile / 16;    // every record is >= 16 B
constexpr int kRounds = kMaxRec / kWave;  // decode rounds of 64 records
static_assert(kTile % 1024 == 0 && kMaxRec % 128 == 0, "tile geometry");

// Hand-off words are 8-byte {tag:16 | value:48} granules, each written by ONE agent-scope store
// (self-validating: tag = the launch epoch).
//
// Per-tile slot.  a = the tile's speculative aggregate A (pass 1, by the tile's own wave);
// e = the tile's exclusive prefix inside its 64-tile group (pass 1, by the group's folder);
// p = the exact inclusive prefix P through the tile (pass 2, by the tile's own wave).
struct alignas(128) TileSlot {
  uint64_t a[3];  // {exit, entry + 1, n | okc << 24}
  uint64_t e[5];  // prefix words, see kPre*
  uint64_t p[3];  // {exit, cnt, ok}
  uint64_t pad[5];
};
// Aggregates of 64 tiles (level 1), 64 level-1 groups (level 2) and 64 level-2 blocks (level 3),
// each with its exclusive prefix inside its parent.
struct alignas(128) GroupSlot {
  uint64_t g[5];  // {exit, entry + 1, cnt, ok | valid << 32, mism + 1}
  uint64_t e[5];  // prefix words, see kPre*
  uint64_t pad[6];
};
// Resident single-pass kernel (k_parse_resident): one slot per wave (its contiguous tile range).
// a = the range's speculative aggregate {exit, entry + 1, cnt, ok} (phase A); p = the exact
// inclusive prefix through the range {exit, cnt, ok} (phase B).  Each workgroup folds its waves'
// aggregates into one GroupSlot (g) and looks back over the lower workgroups' G (decoupled
// look-back); e is unused by the resident pass.
struct alignas(128) RangeSlot {
  uint64_t a[4];
  uint64_t p[3];
  uint64_t e[5];  // unused by the resident pass (kept: RangeSlot and TileSlot share one layout)
  uint64_t pad[4];
};
static_assert(sizeof(RangeSlot) == sizeof(TileSlot), "range slots reuse the tile-slot allocation");
constexpr uint32_t kResMaxWaves = 4096;  // at most 4096 persistent waves
constexpr int kResSlots = 6;             // 64-record rounds of flows held in registers per wave
constexpr uint32_t kResWgMin = 16;       // waves per workgroup (npr_kernels.hip kResWg) is at least this

// exclusive-prefix words: {exit, cnt, ok | valid << 32 | empty << 33, mism + 1, entry + 1}
enum : int { kPreExit = 0, kPreCnt = 1, kPreOk = 2, kPreMism = 3, kPreEntry = 4 };
constexpr int kLevels = 3;  // group levels above the tiles

enum : uint32_t {
  kFlagMagicAtZero = 2u,  // buf[0..4) is the pcap magic (start >= 24): tighten ts_usec bound
  kFlagSpecStart = 8u,    // `start` is not a known record boundary: speculate tile 0's entry too
  kFlagHostSpec = 16u,    // a shard (buf does not hold bytes 0..3): frac_max / ts_ref come from the host
  kFlagHostRef = 32u,     //   ... and ts_ref is valid
};

// optional diagnostic counters (ParseParams::stats, NULL in production launches)
enum : uint32_t {
  kStatRewalk = 0,     // tiles pass 2 re-walked (pass 1's entry was not the exact one)
  kStatMismWait = 1,   // prefixes that waited for a mis-speculated tile's exact prefix
  kStatFoldSlow = 2,   // pass-1 group folds that took the serial (inconsistent-link) path
  kStatScanRounds = 3, // sparse scan: resolve rounds (0 when the fast path settles every link)
  kStatQueueFull = 4,  // sparse resolve passes whose shared re-walk queue overflowed (tasks deferred)
  kStatNoEntry = 5,    // tiles with no plausible record start
  kStatLbPolls = 6,    // resident look-back re-read rounds, summed over workgroups (DIAG kernels only)
  kStatCount = 8
};
constexpr int kStampWords = 16;  // diagnostic stamps per tile (npr_ctx_read_stamps)

struct ParseParams {
  // Every offset below is a FILE offset.  buf + o addresses file byte o; the caller's buffer holds
  // file bytes [base, len) (base = 0 except for a shard), so buf itself may point before it.
  const uint8_t *buf;  // caller pointer - base (caller pointer 16-B aligned)
  uint64_t len;
  uint64_t start;      // offset of the first record (or where to speculate it, kFlagSpecStart)
  uint64_t stop;       // only records starting before `stop` belong to this launch (<= len)
  uint64_t ref;        // a known record header (speculation's ts_sec reference) or ~0
  uint64_t org;        // start rounded down to kTile: tile t covers [org + t*kTile, ...)
  uint32_t big;        // file endianness
  uint32_t epoch;      // granule tag for this launch, 1..65535
  uint32_t ntiles;
  uint32_t frac_max;   // speculation bound on ts_usec (1e9 accepts ns captures)
  uint32_t flags;
  uint32_t timeout_ticks;  // s_memrealtime (100 MHz) ticks before a stalled hand-off aborts
  uint32_t ts_ref;         // kFlagHostRef: ts_sec of a known record of the capture (speculation anchor)
  uint64_t base;           // file offset of the caller's first byte (tiles start at org >= base)
  TileSlot *slots;
  GroupSlot *groups[kLevels + 1];  // [1..3]; [0] unused
  uint32_t ngroups[kLevels + 1];   // [0] = ntiles, [l] = ceil(ngroups[l-1] / 64)
  uint16_t *srec_g;        // pass-1 record offsets, kMaxRec per tile (pass 2 reuses them)
  uint32_t *abort_word;    // == epoch once any tile aborted
  uint64_t *rec_off;
  npr_record *recs;
  uint8_t *rec_status;
  uint64_t rec_cap;
  uint32_t *flows;         // npr_flow as 8 dwords
  uint32_t *flows_v6;      // npr_flow_v6 as 8 dwords
  uint64_t flow_cap;
  npr_summary *summary;
  uint32_t *stats;         // kStatCount counters or NULL
  uint64_t *stamps;        // diagnostic per-tile s_memrealtime stamps [ntiles][kStampWords] or NULL
  // resident single pass (flows-only launches): 0 = use the two-pass kernels
  uint32_t nwaves;         // persistent waves, each owning a contiguous tile range (<= kResMaxWaves, <= ntiles)
  // whole workgroups (nwaves a multiple of 16): tiles dealt per workgroup first (wg_q each, one more
  // for the first wg_r), then over its 16 waves (the oldest take the extra tiles); wg_q == 0: per wave
  uint32_t wg_q, wg_r;
  RangeSlot *rslots;       // [nwaves]
  GroupSlot *rgroups;      // workgroup aggregates G(b), [ceil(nwaves / kResWg)]
  uint32_t *rcnt;          // pacing counter word (res_arrive; never read)
  uint32_t pack;           // resident pass: sparse tiles share kept rounds (k_parse_resident<.., true>)
  const npr_summary *prev; // chained launch (resident pass only): continue the chain and the counts
  uint32_t prev_epoch;     //   of the launch that wrote *prev (its epoch, 0 = unchecked); NULL = none
};

// k_count_tiles then k_emit_tiles, one one-wave workgroup per tile each; or (p.nwaves != 0)
// k_parse_resident, one launch of p.nwaves persistent waves in 16-wave workgroups.
hipError_t launch_parse_extract(const ParseParams &p, hipStream_t s);
// resident waves per CU the hardware admits for k_parse_resident (occupancy query)
int resident_waves_per_cu();
hipError_t launch_extract_dense(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n,
                                uint32_t *flows, uint32_t *flows_v6, uint8_t *status,
                                hipStream_t s);
// the payload of each record's extract_flow error (status and detail may each be NULL)
hipError_t launch_flow_detail(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n, uint8_t *status,
                              uint64_t *detail, hipStream_t s);
// row f3: VXLAN inner flows (dense, row i for record i; any output may be NULL)
hipError_t launch_vxlan_flows(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n, uint32_t dst_port,
                              bool big, uint32_t *flows, uint32_t *flows_v6, uint8_t *status, uint32_t *vni,
                              hipStream_t s);
// row f4: the distinct-flow table (npr_flowtable.hip).  work: flow_table_bytes(n) bytes (any
// content); out / out_v6 / counts: up to cap rows; *total = the number of distinct flows.
hipError_t launch_flow_aggregate(const uint32_t *flows, const uint32_t *flows_v6, const uint64_t *weights, uint64_t n,
                                 void *work, uint32_t *out, uint32_t *out_v6, uint64_t *counts, uint64_t cap,
                                 uint64_t *total, hipStream_t s);
uint64_t flow_table_bytes(uint64_t n);
constexpr uint64_t kMaxAggRows = 1ull << 30;  // rows per call: S = 2^31 slots, 32-bit slot indices
// convert_records in one pass (k_convert_records): rows 0.. = Ok flows in reverse record order,
// *total = all Ok flows (rows past cap are not written; ~0 when a bounded wait timed out).
// look: convert_look_words(n, cus) granules whose tags are not `epoch` at launch; cus = the
// device's CU count (it sets the records per lane).
hipError_t launch_convert_records(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n,
                                  uint32_t *out, uint32_t *out_v6, uint64_t cap, uint64_t *look, uint32_t epoch,
                                  uint64_t *total, uint64_t timeout_ticks, int cus, hipStream_t s);
uint64_t convert_look_words(uint64_t n, int cus);

// ---- the sparse record walk (npr_sparse.hip): flows-only parses of captures of
// long records.  The range [start, stop) is cut into lane ranges of `span` bytes; each lane
// speculates its first record, hops header to header with direct loads (never streaming the
// payloads), decodes each record from one window, and keeps its Ok flows in `cap` slots.  A scan
// kernel makes the lanes' chains exact (re-walking mis-speculated lanes) and a row kernel moves
// the slots to their convert_records rows.
struct SparseLane {  // one lane range's walk (k_sparse_walk; rewritten exact by a k_sparse_scan fix-up)
  uint64_t entry;    // first record (speculated, or exact), ~0 = none found
  uint64_t exit;     // chain position after the range, or the incomplete record (chain END)
  uint32_t cnt, ok;  // records / Ok flows
  uint64_t ovf;      // the first record without a slot (record `cap`; ~0: every record has one)
  uint64_t okmask;   // bit k: record k (slot k) is an Ok flow, k < 64
  uint64_t okmask2;  // ... bit k - 64 for 64 <= k < 128
};
struct SparsePre {   // exact chain state before a 64-lane group (k_sparse_scan -> k_sparse_rows)
  uint64_t exit, cnt, ok, pad;
};
constexpr uint32_t kSparseAggWords = 8;  // a 64-lane group's aggregate (npr::Seg, 64 B)
struct SparseParams {
  ParseParams kp;         // buf, len, start, stop, ref, big, epoch, frac_max, flags, ts_ref, flows,
                          // flows_v6, flow_cap, summary, prev, prev_epoch, stats (the rest unused)
  uint64_t span;          // bytes per lane range (lane i: [start + i span, min(+span, stop)))
  uint64_t nlanes;
  uint32_t ngroups;       // ceil(nlanes / 64): one wave of k_sparse_walk each
  uint32_t cap;           // Ok-flow slots per lane
  SparseLane *lanes;      // [nlanes]
  uint64_t *aggs;         // [ngroups][kSparseAggWords]
  uint64_t *first_entry;  // [ngroups]: the group's first lane entry found (speculative starts)
  SparsePre *pre;         // [ngroups]
  uint64_t *ctl;          // [0] = {epoch, 1} once the scan finished exact (the row kernel checks it)
  uint32_t *area;         // slots, record k of lane l of group g at slot r = (g cap + k) 64 + l, in two
                          // arrays (28 B per record): area[16 B x r] = {ip_s (IPv6: the address
  uint32_t *area_b;       // block's payload offset), ip_d, ports, smac01 | dmac45 << 16} and
                          // area_b[12 B x r] = {smac2..5, dmac0..3, vlan:12 | kind:2 | offset - lane start:18}
  uint64_t *scan;         // k_sparse_scan's scratch: sparse_scan_words(ngroups) words
  uint64_t *lite;         // the aggregates' link fields as arrays: entry [ngroups], exit [ngroups],
                          // cnt | ok << 32 | valid << 63 [ngroups] (the scan's fast path loads these)
};
constexpr uint64_t sparse_scan_words(uint64_t ngroups) { return 7 * ngroups + 2; }
hipError_t launch_sparse(const SparseParams &sp, hipStream_t s);
constexpr uint32_t kSparseCapDefault = 96;  // slots per lane (<= kSparseCapMax: two mask words)
constexpr uint32_t kSparseRelBits = 18;      // a slot's record offset, relative to its lane's start
constexpr uint64_t kSparseSpanMax = 1ull << kSparseRelBits;  // lane ranges are at most this long
constexpr uint32_t kSparseCapMax = 128;

}  // namespace npr
