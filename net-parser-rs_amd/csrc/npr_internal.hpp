// npr_internal.hpp — interface between the C-ABI layer (npr_capi.hip) and the kernels
// (npr_kernels.hip).  Not installed; the public boundary is include/npr.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/npr.h"

namespace npr {

// Tile geometry of the fused parse+extract kernel.
constexpr int kBlock = 256;            // 4 waves
constexpr int kTile = 16384;           // bytes of the record stream owned by one workgroup
constexpr int kHalo = 256;             // bytes staged past the tile (headers of straddling records)
constexpr int kStage = kTile + kHalo;  // bytes staged in LDS per workgroup
constexpr int kMaxRec = kTile / 16;    // every record is >= 16 B
constexpr int kSlots = kMaxRec / kBlock;

// Per-tile hand-off slot: A = speculative aggregate, P = exact inclusive prefix.  Each word is
// an 8-byte {tag:16 | value:48} granule written by ONE agent-scope store (self-validating).
struct alignas(64) TileSlot {
  uint64_t a[4];
  uint64_t p[4];
};

// Two-level look-back: the last tile of every kGroup-tile group publishes a group aggregate.
constexpr int kGroup = 64;
struct alignas(32) GroupSlot {
  uint64_t g[4];
};

enum : uint32_t {
  kFlagSpecFirst = 1u,    // tile 0's entry is speculative too (shard that starts mid-stream)
  kFlagMagicAtZero = 2u,  // buf[0..4) is the pcap magic (start >= 24): tighten ts_usec bound
};

// optional diagnostic counters (ParseParams::stats, NULL in production launches)
enum : uint32_t {
  kStatRewalk = 0,     // tiles whose speculated entry was wrong (re-walked)
  kStatMismWait = 1,   // look-back waits for a mismatching tile's exact prefix
  kStatSpin = 2,       // look-back polls that found an unpublished predecessor
  kStatSlide = 3,      // look-back windows with no exact prefix (slid 64 tiles further)
  kStatWeakEntry = 4,  // tiles that used a weak speculation
  kStatNoEntry = 5,    // tiles with no plausible record start
  kStatCount = 8
};

struct ParseParams {
  const uint8_t *buf;  // 16-B aligned device pointer
  uint64_t len;
  uint64_t start;      // offset of the first record
  uint64_t org;        // start rounded down to kTile: tile t covers [org + t*kTile, ...)
  uint32_t big;        // file endianness
  uint32_t epoch;      // granule tag for this launch, 1..65535
  uint32_t ntiles;
  uint32_t frac_max;   // speculation bound on ts_usec (1e9 accepts ns captures)
  uint32_t flags;
  uint32_t timeout_ticks;  // s_memrealtime (100 MHz) ticks before a stalled hand-off aborts
  TileSlot *slots;
  GroupSlot *groups;       // ntiles / kGroup
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
  uint64_t pcnt_slow;      // kernel-internal: record index base during a slow-path re-decode
};

hipError_t launch_parse_extract(const ParseParams &p, hipStream_t s);
// persistent pipelined variant: `grid` resident workgroups loop over the tiles
hipError_t launch_parse_pipe(const ParseParams &p, uint32_t grid, hipStream_t s);
int pipe_blocks_per_cu();
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
