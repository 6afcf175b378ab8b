// npr_internal.hpp — interface between the C-ABI layer (npr_capi.hip) and the kernels
// (npr_kernels.hip).  Not installed; the public boundary is include/npr.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/npr.h"

namespace npr {

// Tile geometry of the parse+extract kernels: ONE WAVE per tile.
constexpr int kBlock = 256;            // workgroup size of the auxiliary kernels (dense extract, compaction)
constexpr int kWave = 64;              // the parse kernels: one-wave workgroups
#ifndef NPR_TILE_BYTES
#define NPR_TILE_BYTES 4096
#endif
constexpr int kTile = NPR_TILE_BYTES;  // bytes of the record stream owned by one tile (one wave)
constexpr int kHalo = 128;             // bytes staged past the tile (headers + fast-decode window of straddlers)
constexpr int kStage = kTile + kHalo;  // bytes staged in LDS per tile
constexpr int kMaxRec = kTile / 16;    // every record is >= 16 B
constexpr int kRounds = kMaxRec / kWave;  // decode rounds of 64 records
// An Ok record spans >= 16 + 42 bytes (header + Ethernet/IPv4/UDP), so at most this many Ok
// records start in one tile: the per-tile capacity of the parked-flow scratch.
constexpr int kMaxOk = (kTile + 57) / 58 + 1;

// Per-tile hand-off slot: A = speculative aggregate (k_scan_tiles), P = exact inclusive prefix
// (k_emit_tiles).  Each word is an 8-byte {tag:16 | value:48} granule written by ONE
// agent-scope store (self-validating: tag = the launch epoch).
struct alignas(64) TileSlot {
  uint64_t a[4];
  uint64_t p[4];
};

// Aggregates of 64 tiles (G1) and of 64 G1s = 4096 tiles (G2), folded by the last arriver.
constexpr int kGroup = 64;
struct alignas(32) GroupSlot {
  uint64_t g[4];
};

enum : uint32_t {
  kFlagMagicAtZero = 2u,  // buf[0..4) is the pcap magic (start >= 24): tighten ts_usec bound
  kFlagLight = 4u,        // flows only (no record table / status): pass 1 parks the flows, pass 2 copies
  kFlagSpecStart = 8u,    // `start` is not a known record boundary: speculate tile 0's entry too
};

// optional diagnostic counters (ParseParams::stats, NULL in production launches)
enum : uint32_t {
  kStatRewalk = 0,     // tiles pass 2 re-walked (pass 1's entry was not the exact one)
  kStatMismWait = 1,   // prefix folds that waited for a mis-speculated tile's exact prefix
  kStatWeakEntry = 4,  // tiles that used a weak speculation
  kStatNoEntry = 5,    // tiles with no plausible record start
  kStatCount = 8
};
constexpr int kStampWords = 16;  // diagnostic stamps per tile (npr_ctx_read_stamps)

struct ParseParams {
  const uint8_t *buf;  // 16-B aligned device pointer
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
  TileSlot *slots;
  GroupSlot *groups1;      // ngroups1 = ceil(ntiles / 64)
  GroupSlot *groups2;      // ceil(ngroups1 / 64)
  uint32_t *cnt1, *cnt2;   // arrival counters (zero between launches)
  uint32_t ngroups1, ngroups2;
  uint16_t *srec_g;        // pass-1 record offsets, kMaxRec per tile (pass 2 reuses them)
  uint32_t *park;          // light mode: pass-1 Ok flows, kMaxOk 32-B rows per tile
  uint32_t *park_v6;       // light mode: their IPv6 addresses (when flows_v6)
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
  uint64_t *stamps;        // diagnostic per-tile s_memrealtime stamps [ntiles][8] or NULL
};

// Persistent grids (capped at ntiles) whose workgroups each own a contiguous run of tiles:
// grid_emit == 0 -> one fused launch (k_parse_fused, grid_scan workgroups); else k_scan_tiles
// then k_emit_tiles.
hipError_t launch_parse_extract(const ParseParams &p, uint32_t grid_scan, uint32_t grid_emit, hipStream_t s);
int scan_blocks_per_cu();  // resident workgroups per CU (occupancy API)
int emit_blocks_per_cu();
int fused_blocks_per_cu();
hipError_t launch_extract_dense(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n,
                                uint32_t *flows, uint32_t *flows_v6, uint8_t *status,
                                hipStream_t s);
// convert_records over a dense extract: Ok rows of (flows, flows_v6, status) in reverse order.
hipError_t launch_compact_reverse(const uint32_t *flows, const uint32_t *flows_v6,
                                  const uint8_t *status, uint64_t n, uint32_t *out,
                                  uint32_t *out_v6, uint64_t cap, uint32_t *block_counts,
                                  uint64_t *total, hipStream_t s);
uint64_t compact_workspace_words(uint64_t n);

}  // namespace npr
