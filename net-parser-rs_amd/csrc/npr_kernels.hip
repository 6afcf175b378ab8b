// npr_kernels.hip — CDNA4 (gfx950) kernels for the pcap record chain + flow extraction.
//
// Replaces, on the device, the nom parse paths of protectwise/net-parser-rs 0.3.0:
//   PcapRecords::parse loop           src/record.rs:21-54     -> walk_tile() + speculation + prefix folds
//   PcapRecord::parse                 src/record.rs:102-121   -> hdr() / walk_tile()
//   FlowExtraction::extract_flow      src/flow/mod.rs:20-48   -> decode<>() / decode_fast<>()
//     Ethernet::parse + vlan loop     src/layer2/ethernet.rs:143-216
//     IPv4::parse / parse_ipv4        src/layer3/ipv4.rs:76-160
//     IPv6::parse / parse_next_header src/layer3/ipv6.rs:29-99
//     Arp::parse                      src/layer3/arp.rs:54-76
//     Tcp::parse / Udp::parse         src/layer4/tcp.rs:59-101, src/layer4/udp.rs:33-50
//     per-layer flow dispatch         src/flow/layer2/ethernet.rs:39-133, src/flow/layer3/*.rs
//   flow::convert_records             src/flow/mod.rs:101-123 -> reverse-order rows, ranked by ballot
//
// Design.  A 4 KiB TILE of the record stream is the unit of work; every tile is
// staged into LDS by DMA and its entry (first record start) is SPECULATED from header plausibility
// (tile 0 starts at `start`); a wave walks the chain from it, decodes every record's flow status
// and summarises the tile as A = {entry, exit, records, Ok flows}.  Tiles combine under a
// chain-consistency monoid (an aggregate is exact when each entry continues its predecessor's
// exit).  Three launch shapes use these pieces:
//   k_count_tiles + k_emit_tiles (record-table launches): two streaming passes of one-wave
//     workgroups, one per tile; pass 1 publishes A and folds 64-tile groups, pass 2 rebuilds the
//     exact state before each tile from the folds and writes every record row and flow;
//   k_parse_resident (flows-only launches, the default): persistent waves, each owning a
//     contiguous tile range, flows kept in registers; one pass with a decoupled look-back over
//     16-wave workgroup aggregates (chained launches for captures past what registers hold).
// A wrong speculation costs a wait or a re-walk, never a wrong result.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "npr_decode.hpp"  // decode<>: the general per-record decode tree (host + device)
#include "npr_device.hpp"   // shared device helpers (fast decode, granules, segments, speculation context)
#include "npr_internal.hpp"

namespace npr {



// one record (header at LDS offset rel) -> status (+ flow words); fast shape first
template <bool FIELDS>
__device__ __forceinline__ uint32_t decode_rec(const ParseParams &kp, const uint32_t *w, uint64_t tile_lo,
                                               uint32_t rel, FlowWords &f, bool valid = true) {
  // lanes whose result is unused read what the first used lane reads: LDS broadcasts identical
  // addresses, so they add no bank conflicts (a sparse tile has ~5 used lanes of 64; their stale
  // offsets were random addresses: C3 46 % of LDS-active cycles conflicted)
  const uint64_t vb = __ballot(valid);
  const uint32_t rel0 = vb ? (uint32_t)__builtin_amdgcn_readlane((int)rel, (int)__builtin_ctzll(vb)) : 0u;
  const uint32_t rr = valid ? rel : rel0;
  const uint32_t incl = hdr(w, rr, 2, kp.big);
  uint32_t st = decode_fast<FIELDS, true>(w, rr + 16u, incl, f, valid);
  if (__ballot(valid && st == 0xffu)) {  // uniform test: most tiles never take the general path
    if (valid && st == 0xffu) {
      const uint64_t p = tile_lo + rel;
      // (saturated: a record the walk found lies inside the capture, but a position past it must read
      // zeros, never wrap to a huge reach -- round 4's faulting timing-only build)
      TileReader r{w, (const uint8_t *)w, rel + 16u, kp.buf + p + 16, p + 16 <= kp.len ? kp.len - p - 16 : 0ull};
      st = decode<FIELDS>(r, incl, f);
    }
  }
  return st;
}

__device__ __forceinline__ uint64_t tile_end(const ParseParams &kp, int64_t k) {
  const uint64_t e = kp.org + (uint64_t)(k + 1) * kTile;
  return e < kp.stop ? e : kp.stop;
}

// Chain-consistency monoid: X then Y (Y's tiles follow X's).  Y's counts are trusted only when
// Y's speculated entry is exactly where X's chain continues.
__device__ __forceinline__ Seg combine(const ParseParams &kp, const Seg &X, const Seg &Y) {
  Seg r = X;
  r.last = Y.last;
  if (!X.valid) return r;                       // keep the lowest mismatch
  if (X.exit < tile_end(kp, X.last)) return r;  // chain ended inside X (Q3): Y is moot
  if (X.exit >= tile_end(kp, Y.last)) return r; // one record spans all of Y: no record starts there
  if (X.exit != Y.entry) {                      // Y's speculated start is wrong
    r.valid = false;
    r.mism = Y.first;
    return r;
  }
  r.exit = Y.exit;
  r.cnt = X.cnt + Y.cnt;
  r.ok = X.ok + Y.ok;
  r.valid = Y.valid;
  r.mism = Y.mism;
  return r;
}

// Bounded wait: false once the grid aborted or this wait exceeded the time budget.
__device__ __forceinline__ bool spin_ok(const ParseParams &kp, uint64_t t0) {
  __builtin_amdgcn_s_sleep(2);
  if (__hip_atomic_load(kp.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kp.epoch) return false;
  if (__builtin_amdgcn_s_memrealtime() - t0 > kp.timeout_ticks) {
    __hip_atomic_store(kp.abort_word, kp.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}

// Elements of level l: tiles (l = 0) and groups of 64^l tiles (l = 1..kLevels).
__device__ __forceinline__ int64_t elem_first(int lvl, int64_t idx) { return idx << (6 * lvl); }
__device__ __forceinline__ int64_t elem_last(const ParseParams &kp, int lvl, int64_t idx) {
  const int64_t l = ((idx + 1) << (6 * lvl)) - 1;
  return l < (int64_t)kp.ntiles - 1 ? l : (int64_t)kp.ntiles - 1;
}
__device__ __forceinline__ uint64_t *prefix_words(const ParseParams &kp, int lvl, int64_t idx) {
  return lvl == 0 ? kp.slots[idx].e : kp.groups[lvl][idx].e;
}

// One lane's element of a 64-wide window of aggregates.
struct LaneSeg {
  uint64_t entry, exit, cnt, ok;
  int64_t first, last, mism;
  uint32_t valid, present;  // (32-bit: no padding bytes)
};

// level 0: A = {exit, entry + 1, n | okc << 24};  levels 1..3: G = {exit, entry + 1, cnt, ok | valid << 32, mism + 1}
__device__ __forceinline__ LaneSeg load_agg(const ParseParams &kp, int lvl, int64_t idx, bool inr) {
  LaneSeg L{};
  L.mism = -1;
  L.valid = true;
  L.first = elem_first(lvl, idx);
  L.last = elem_last(kp, lvl, idx);
  if (!inr) return L;
  const uint32_t ep = kp.epoch;
  const uint64_t *w = lvl == 0 ? kp.slots[idx].a : kp.groups[lvl][idx].g;
  const uint64_t w0 = ld_agent(w + 0), w1 = ld_agent(w + 1), w2 = ld_agent(w + 2);
  const uint64_t w3 = lvl == 0 ? w0 : ld_agent(w + 3), w4 = lvl == 0 ? w0 : ld_agent(w + 4);
  L.present = tagged(w0, ep) && tagged(w1, ep) && tagged(w2, ep) && tagged(w3, ep) && tagged(w4, ep);
  const uint64_t e1 = w1 & kMask48;
  L.entry = e1 ? e1 - 1 : kNone;
  L.exit = w0 & kMask48;
  if (lvl == 0) {
    L.cnt = w2 & 0xffffffull;
    L.ok = (w2 >> 24) & 0xffffffull;
  } else {
    const uint64_t v3 = w3 & kMask48, m = w4 & kMask48;
    L.cnt = w2 & kMask48;
    L.ok = v3 & 0xffffffffull;
    L.valid = (v3 >> 32) & 1ull;
    L.mism = L.valid ? -1 : (int64_t)m - 1;
  }
  return L;
}

__device__ __forceinline__ void put_agg(const ParseParams &kp, GroupSlot *G, const Seg &c) {
  const uint32_t ep = kp.epoch;
  st_agent(&G->g[0], gran(ep, c.exit));
  st_agent(&G->g[1], gran(ep, c.entry == kNone ? 0ull : c.entry + 1));
  st_agent(&G->g[2], gran(ep, c.cnt));
  st_agent(&G->g[3], gran(ep, (c.ok & 0xffffffffull) | ((uint64_t)c.valid << 32)));
  st_agent(&G->g[4], gran(ep, c.valid ? 0ull : (uint64_t)c.mism + 1));
}

// exclusive prefix of an element inside its parent: {exit, cnt, ok | valid << 32 | empty << 33,
// mism + 1, entry + 1} (a parent's first child has the empty prefix)
__device__ __forceinline__ void put_prefix(const ParseParams &kp, uint64_t *e, const Seg &p, bool empty) {
  const uint32_t ep = kp.epoch;
  st_agent(e + kPreExit, gran(ep, empty ? 0ull : p.exit));
  st_agent(e + kPreCnt, gran(ep, empty ? 0ull : p.cnt));
  st_agent(e + kPreOk, gran(ep, empty ? (1ull << 32) | (1ull << 33) : (p.ok & 0xffffffffull) | ((uint64_t)p.valid << 32)));
  st_agent(e + kPreMism, gran(ep, (empty || p.valid) ? 0ull : (uint64_t)p.mism + 1));
  st_agent(e + kPreEntry, gran(ep, (empty || p.entry == kNone) ? 0ull : p.entry + 1));
}

// the prefix words of element idx of level lvl (already loaded) as a segment of tiles
// [first tile of the parent, first tile of the element - 1]
__device__ __forceinline__ Seg prefix_seg(uint64_t e0, uint64_t e1, uint64_t e2, uint64_t e3, uint64_t e4, int lvl,
                                          int64_t idx, bool &empty) {
  Seg s;
  const uint64_t v = e2 & kMask48, m = e3 & kMask48, en = e4 & kMask48;
  s.exit = e0 & kMask48;
  s.cnt = e1 & kMask48;
  s.ok = v & 0xffffffffull;
  s.valid = (v >> 32) & 1ull;
  empty = (v >> 33) & 1ull;
  s.mism = s.valid ? -1 : (int64_t)m - 1;
  s.entry = en ? en - 1 : kNone;
  s.first = elem_first(lvl, idx & ~63ll);
  s.last = elem_first(lvl, idx) - 1;
  return s;
}


// Fold lanes [lo .. 0] (ascending tile order = descending lane) into one segment.  Fast path:
// every link consistent, no END, no pass-through, all valid -> two wave sums; otherwise the
// serial monoid (wave-uniform, readlane).
__device__ __forceinline__ Seg fold_window(const ParseParams &kp, const LaneSeg &L, int lo) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint64_t prev_exit = shfl_down64(L.exit);  // exit of the preceding segment (lane + 1)
  const bool inr = lane <= lo;
  const bool bad = lane < lo && (!L.valid || L.entry != prev_exit);
  const bool endc = inr && L.exit < tile_end(kp, L.last);
  const bool lo_bad = lane == lo && !L.valid;
  Seg r;
  if (__ballot(bad || endc || lo_bad) == 0ull) {
    // a window of <= 64 aggregates never counts 2^32 records (<= 64 blocks x 1M records)
    r.cnt = __ockl_wfred_add_u32(inr ? (uint32_t)L.cnt : 0u);
    r.ok = __ockl_wfred_add_u32(inr ? (uint32_t)L.ok : 0u);
    r.entry = rl64(L.entry, lo);
    r.exit = rl64(L.exit, 0);
    r.first = (int64_t)rl64((uint64_t)L.first, lo);
    r.last = (int64_t)rl64((uint64_t)L.last, 0);
    r.mism = -1;
    r.valid = true;
    return r;
  }
  const uint64_t bval = __ballot(L.valid);
  auto lane_seg = [&](int j) {
    Seg y;
    y.entry = rl64(L.entry, j);
    y.exit = rl64(L.exit, j);
    y.cnt = rl64(L.cnt, j);
    y.ok = rl64(L.ok, j);
    y.first = (int64_t)rl64((uint64_t)L.first, j);
    y.last = (int64_t)rl64((uint64_t)L.last, j);
    y.mism = (int64_t)rl64((uint64_t)L.mism, j);
    y.valid = (bval >> j) & 1ull;
    return y;
  };
  r = lane_seg(lo);
  for (int j = lo - 1; j >= 0; --j) r = combine(kp, r, lane_seg(j));
  return r;
}

// Load + fold `cnt` (1..64) consecutive level-`lvl` aggregates starting at element `base`
// (wave-uniform).  Waits (bounded) until all are published.
__device__ bool fold_range(const ParseParams &kp, int lvl, int64_t base, int cnt, Seg &out, uint64_t t0) {
  const int lane = (int)(threadIdx.x & 63u);
  const bool inr = lane < cnt;
  for (;;) {
    const LaneSeg L = load_agg(kp, lvl, base + cnt - 1 - lane, inr);
    if (__ballot(inr && !L.present) == 0ull) {
      out = fold_window(kp, L, cnt - 1);
      return true;
    }
    if (!spin_ok(kp, t0)) return false;
  }
}

// Exact prefix through tile m: its P granules (published by k_emit_tiles), bounded wait.
__device__ bool wait_exact(const ParseParams &kp, int64_t m, Seg &X, uint64_t t0) {
  const TileSlot *s = kp.slots + m;
  for (;;) {
    const uint64_t p0 = ld_agent(&s->p[0]), p1 = ld_agent(&s->p[1]), p2 = ld_agent(&s->p[2]);
    if (tagged(p0, kp.epoch) && tagged(p1, kp.epoch) && tagged(p2, kp.epoch)) {
      X.exit = p0 & kMask48;
      X.cnt = p1 & kMask48;
      X.ok = p2 & kMask48;
      X.first = 0;
      X.last = m;
      X.mism = -1;
      X.valid = true;
      return true;
    }
    if (!spin_ok(kp, t0)) return false;
  }
}

// Generic exact prefix of tiles [a, t) continuing X: ascending, largest aligned aggregates
// first; every contradiction is settled by the exact prefix of the offending tile (published by
// its own wave in k_emit_tiles; that wave was dispatched earlier, so it is resident or done).
template <bool DIAG>
__device__ bool prefix_generic(const ParseParams &kp, Seg X, int64_t a, int64_t t, Seg &out, uint64_t t0) {
  for (;;) {
    if (!X.valid) {
      const int64_t m = X.mism;
      if (!wait_exact(kp, m, X, t0)) return false;
      if (DIAG && kp.stats && (threadIdx.x & 63u) == 0) atomicAdd(kp.stats + kStatMismWait, 1u);
      a = m + 1;
    }
    if (a >= t) break;
    int lvl = 0;
    for (int l = kLevels; l >= 1; --l) {
      const int64_t span = 1ll << (6 * l);
      if ((a & (span - 1)) == 0 && t - a >= span) {
        lvl = l;
        break;
      }
    }
    const int64_t unit = 1ll << (6 * lvl);
    int64_t cnt = (t - a) >> (6 * lvl);
    const int64_t to_parent = lvl == kLevels ? 64 : ((unit << 6) - (a & ((unit << 6) - 1))) >> (6 * lvl);
    cnt = cnt < to_parent ? cnt : to_parent;
    cnt = cnt < 64 ? cnt : 64;
    Seg Y;
    if (!fold_range(kp, lvl, a >> (6 * lvl), (int)cnt, Y, t0)) return false;
    X = combine(kp, X, Y);
    a += cnt << (6 * lvl);
  }
  out = X;
  return true;
}

__device__ __forceinline__ Seg start_seg(const ParseParams &kp) {
  Seg X;
  X.entry = X.exit = kp.start;
  X.cnt = X.ok = 0;
  X.first = X.last = -1;
  X.mism = -1;
  X.valid = true;
  return X;
}

// Fold element `idx` of level `lvl` (1..kLevels) from its (up to 64) children of level lvl-1:
// publish the element's aggregate G and every child's exclusive prefix inside the element.  Run
// by the wave that produced the element's LAST child; the other children come from waves
// dispatched before it.  False if a wait timed out (the launch then reports NPR_ERR_TIMEOUT).
template <bool DIAG>
__device__ bool fold_children(const ParseParams &kp, int lvl, int64_t idx, uint64_t t0) {
  const int lane = (int)(threadIdx.x & 63u);
  const int64_t c0 = idx << 6;
  const int64_t nch = (int64_t)kp.ngroups[lvl - 1];
  const int size = (int)(nch - c0 < 64 ? nch - c0 : 64);
  const bool inr = lane < size;
  LaneSeg L;
  for (;;) {
    L = load_agg(kp, lvl - 1, c0 + lane, inr);
    if (__ballot(inr && !L.present) == 0ull) break;
    if (!spin_ok(kp, t0)) return false;
  }
  const uint64_t prev_exit = shfl_up64(L.exit);  // lane j <- lane j-1
  const bool link_bad = inr && (!L.valid || (lane > 0 && L.entry != prev_exit));
  const bool end_mid = lane < size - 1 && L.exit < tile_end(kp, L.last);
  Seg ep{}, agg;
  if (__ballot(link_bad || end_mid) == 0ull) {
    // consistent chain through every child: exclusive prefixes are plain prefix sums
    const uint32_t c = inr ? (uint32_t)L.cnt : 0u, o = inr ? (uint32_t)L.ok : 0u;
    const uint32_t cx = excl_scan_u32(c), ox = excl_scan_u32(o);
    ep.entry = rl64(L.entry, 0);
    ep.exit = prev_exit;
    ep.cnt = cx;
    ep.ok = ox;
    ep.valid = true;
    ep.mism = -1;
    agg.entry = ep.entry;
    agg.exit = rl64(L.exit, size - 1);
    agg.cnt = (uint32_t)__builtin_amdgcn_readlane((int)(cx + c), size - 1);
    agg.ok = (uint32_t)__builtin_amdgcn_readlane((int)(ox + o), size - 1);
    agg.valid = true;
    agg.mism = -1;
  } else {
    // the serial monoid (wave-uniform): an END, a pass-through or a mis-speculated child
    if (DIAG && kp.stats && lane == 0) atomicAdd(kp.stats + kStatFoldSlow, 1u);
    const uint64_t bval = __ballot(L.valid);
    Seg r{};
    for (int j = 0; j < size; ++j) {
      Seg y;
      y.entry = rl64(L.entry, j);
      y.exit = rl64(L.exit, j);
      y.cnt = rl64(L.cnt, j);
      y.ok = rl64(L.ok, j);
      y.first = (int64_t)rl64((uint64_t)L.first, j);
      y.last = (int64_t)rl64((uint64_t)L.last, j);
      y.mism = (int64_t)rl64((uint64_t)L.mism, j);
      y.valid = (bval >> j) & 1ull;
      if (j == 0) {
        r = y;
      } else {
        if (lane == j) ep = r;
        r = combine(kp, r, y);
      }
    }
    agg = r;
  }
  if (inr) put_prefix(kp, prefix_words(kp, lvl - 1, c0 + lane), ep, lane == 0);
  if (lane == 0) put_agg(kp, kp.groups[lvl] + idx, agg);
  return true;
}

// ---------------------------------------------------------------------------------------------
// speculation (tile-relative 32-bit arithmetic) + chain walk
// ---------------------------------------------------------------------------------------------

// The 16-B header at LDS offset r, in the capture's endianness: five aligned dword reads +
// four v_alignbyte (every lane its own r).
__device__ __forceinline__ void hdr4(const uint32_t *w, uint32_t r, bool big, uint32_t (&h)[4]) {
  const uint32_t *p = w + (r >> 2);
  const uint32_t sh = r & 3u;
  uint32_t x[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) x[k] = p[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t v = __builtin_amdgcn_alignbyte(x[k + 1], x[k], sh);
    h[k] = big ? __builtin_bswap32(v) : v;
  }
}

// Is LDS offset r a plausible record start on its own header (and does its payload fit)?
__device__ __forceinline__ bool head_ok(const SpecCtx &c, const uint32_t (&h)[4], uint32_t r) {
  return c.avail - r >= 16 && plaus(c, h[0], h[1], h[2], h[3]) && c.avail - r - 16 >= h[2];
}

// How plausible is a start at r whose own header passed head_ok?  1 = weak (fewer than two
// chained headers could be checked inside the staged window); 2 = strong; 0 = a chained header
// fails.  Wave-uniform.  A heuristic only: k_emit_tiles verifies every guess; a wrong one costs
// a wait or a re-walk, never a result.
__device__ __forceinline__ int chain_grade(const SpecCtx &c, const uint32_t *w, uint32_t r, uint32_t ts, uint32_t incl) {
  uint32_t q = r + 16 + incl;
  int ver = 0;
  for (int hop = 0; hop < 3; ++hop) {
    if (q == c.avail && c.exact_end) return 2;
    if (q + 16 > (uint32_t)kStage) return ver >= 2 ? 2 : 1;
    if (c.avail - q < 16) return ver >= 1 ? 2 : 1;
    const uint32_t ts2 = hdr(w, q, 0, c.big), incl2 = hdr(w, q, 2, c.big);
    if (!plaus(c, ts2, hdr(w, q, 1, c.big), incl2, hdr(w, q, 3, c.big))) return 0;
    if (ts2 - ts + kTsWindow > 2u * kTsWindow) return 0;
    ++ver;
    if (c.avail - q - 16 < incl2) return ver >= 2 ? 2 : 1;
    ts = ts2;
    q += 16 + incl2;
  }
  return 2;
}

// chain_grade() in ONE parallel LDS read: lanes 1..3 read the headers of hops 1..3 at the
// positions they have if the candidate's record length repeats.  Returns chain_grade()'s answer
// when every hop it needs sits where assumed, else -1 (the caller then hops serially).
__device__ __forceinline__ int stride_grade(const SpecCtx &c, const uint32_t *w, uint32_t r, uint32_t ts, uint32_t incl) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k = lane >= 1u && lane <= 3u ? lane : 0u;
  const uint32_t q = r + k * (16u + incl);
  const bool in_stage = k != 0u && q + 16u <= (uint32_t)kStage;
  uint32_t h[4];
  hdr4(w, in_stage ? q : 0u, c.big, h);
  const uint32_t myts = lane == 0u ? ts : h[0];
  const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)myts, 0x111, 0xf, 0xf, false);  // row_shr:1
  const uint64_t eof = __ballot(k && q == c.avail && c.exact_end);
  const uint64_t stage = __ballot(k && !in_stage);
  const uint64_t shrt = __ballot(k && c.avail - q < 16u);
  const uint64_t pass = __ballot(k && plaus(c, h[0], h[1], h[2], h[3]) && h[0] - prev + kTsWindow <= 2u * kTsWindow);
  const uint64_t cut = __ballot(k && c.avail - q - 16u < h[2]);
  const uint64_t same = __ballot(k && h[2] == incl);
  int ver = 0;
  for (int i = 1; i <= 3; ++i) {
    const uint64_t b = 1ull << i;
    if (i >= 2 && !(same & (b >> 1))) return -1;  // hop i is not where the stride puts it
    if (eof & b) return 2;
    if (stage & b) return ver >= 2 ? 2 : 1;
    if (shrt & b) return ver >= 1 ? 2 : 1;
    if (!(pass & b)) return 0;
    ++ver;
    if (cut & b) return ver >= 2 ? 2 : 1;
  }
  return 2;
}

// PcapRecords::parse loop (src/record.rs:30-49) over one tile, from `entry`, by one wave.
// Records whose header starts before tile_hi belong to this tile.  Returns the exit: the first
// chain offset >= tile_hi, or (chain END, Q3) the offset of the first incomplete record.
// Stride speculation: while the record length repeats, lane j confirms records j, j+64, j+128,
// j+192 ahead in one LDS round trip (up to 256 records per step); one record per step otherwise.
constexpr int kWalkUnroll = 4;
// last_io: the incl_len of the record before `entry` (in), of the last record walked (out), so a
// wave walking consecutive tiles keeps hopping through variable-length traffic; NULL: unknown
// (the first record tries a stride)
constexpr uint32_t kAnyLen = ~0u;  // walk_tile: no previous record length known
// incl_len of the record header at LDS byte r (wave-uniform) in the capture's byte order
template <bool BIG>
__device__ __forceinline__ uint32_t incl_at(const uint32_t *w, uint32_t r) {
  const uint32_t i = (r >> 2) + 2u;
  const uint32_t v = __builtin_amdgcn_alignbyte(w[i + 1], w[i], r & 3u);
  return __builtin_amdgcn_readfirstlane(BIG ? __builtin_bswap32(v) : v);
}

// A run of hops through variable-length records, from the record at r (length incl, already
// checked): each record's offset goes to srec[n] (every lane stores the one address: a broadcast,
// no exec-mask switch); the run stops at hop_span or at a record that is not a plain hop (same
// length as the previous one, or longer than a tile).  hop_span is 0 unless every record starting
// inside the tile with incl <= kTile ends inside the capture, so no Incomplete test is needed
// here.  Returns the next position.
__device__ __forceinline__ uint32_t lds_addr(const void *p) {  // byte address in LDS of an LDS pointer
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void *)p);
}
template <bool BIG>
__device__ __forceinline__ uint32_t hop_run(const uint32_t *w, uint16_t *srec, uint32_t r, uint32_t incl,
                                            uint32_t hop_span, uint32_t &n, uint32_t &last) {
  // The loop by hand (the compiled one spent ~17 SALU per hop on flow blocks and copies): per hop
  // one broadcast ds_write_b16 of the offset, two ds_read_b32 of the next header's incl_len word
  // pair, v_alignbyte + readfirstlane, and three compare-and-branch exits; the srec address walks
  // in a VGPR.  Both LDS pointers come from __shared__ arrays (every walk_tile caller's).
  uint32_t va, vd, vlo, vhi, t;
  // every operand wave-uniform by construction; readfirstlane makes that visible where the
  // compiler's uniformity analysis loses track (the asm takes them in scalar registers)
  const uint32_t sa = __builtin_amdgcn_readfirstlane(lds_addr(srec) + 2u * n);
  const uint32_t wb = __builtin_amdgcn_readfirstlane(lds_addr(w));
  r = __builtin_amdgcn_readfirstlane(r);
  n = __builtin_amdgcn_readfirstlane(n);
  incl = __builtin_amdgcn_readfirstlane(incl);
  hop_span = __builtin_amdgcn_readfirstlane(hop_span);
#define NPR_HOP_ASM(PERM)                                                                              \
  asm volatile(                                                                                        \
      "v_mov_b32 %[va], %[sa]\n"                                                                       \
      "1:\n\t"                                                                        \
      "v_mov_b32 %[vd], %[r]\n\t"                                                                      \
      "ds_write_b16 %[va], %[vd]\n\t"                                                                  \
      "v_add_u32 %[va], 2, %[va]\n\t"                                                                  \
      "s_add_u32 %[n], %[n], 1\n\t"                                                                    \
      "s_add_u32 %[r], %[r], %[incl]\n\t"                                                              \
      "s_add_u32 %[r], %[r], 16\n\t"                                                                   \
      "s_mov_b32 %[last], %[incl]\n\t"                                                                 \
      "s_cmp_ge_u32 %[r], %[span]\n\t"                                                                 \
      "s_cbranch_scc1 2f\n\t"                                                          \
      "s_and_b32 %[t], %[r], -4\n\t"                                                                   \
      "s_add_u32 %[t], %[t], %[wb]\n\t"                                                                \
      "v_mov_b32 %[vlo], %[t]\n\t"                                                                     \
      "ds_read_b32 %[vhi], %[vlo] offset:12\n\t"                                                       \
      "ds_read_b32 %[vlo], %[vlo] offset:8\n\t"                                                        \
      "s_and_b32 %[t], %[r], 3\n\t"                                                                    \
      "s_waitcnt lgkmcnt(0)\n\t"                                                                       \
      "v_alignbyte_b32 %[vlo], %[vhi], %[vlo], %[t]\n\t" PERM                                          \
      "s_nop 0\n\t"                                                                                    \
      "v_readfirstlane_b32 %[incl], %[vlo]\n\t"                                                        \
      "s_cmp_eq_u32 %[incl], %[last]\n\t"                                                              \
      "s_cbranch_scc1 2f\n\t"                                                          \
      "s_cmpk_le_u32 %[incl], %[tile]\n\t"                                                             \
      "s_cbranch_scc1 1b\n"                                                             \
      "2:"                                                                             \
      : [r] "+s"(r), [n] "+s"(n), [incl] "+s"(incl), [last] "=&s"(last), [t] "=&s"(t), [va] "=&v"(va),  \
        [vd] "=&v"(vd), [vlo] "=&v"(vlo), [vhi] "=&v"(vhi)                                             \
      : [sa] "s"(sa), [wb] "s"(wb), [span] "s"(hop_span), [perm] "s"(0x00010203u), [tile] "i"(kTile)  \
      : "scc", "memory")
  if constexpr (BIG) NPR_HOP_ASM("v_perm_b32 %[vlo], 0, %[vlo], %[perm]\n\t");
  else NPR_HOP_ASM("");
#undef NPR_HOP_ASM
  return r;
}

__device__ __forceinline__ uint64_t walk_tile_inl(const ParseParams &kp, const uint32_t *w, uint16_t *srec, uint64_t tile_lo,
                              uint64_t tile_hi, uint64_t entry, uint32_t &n_out, uint32_t *last_io = nullptr) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool big = kp.big;
  const uint32_t span = (uint32_t)(tile_hi - tile_lo);
  const uint64_t av = kp.len - tile_lo;
  const uint32_t avail = av > 0xffffffffull ? 0xffffffffu : (uint32_t)av;  // bytes from tile_lo
  const uint32_t hop_span = avail - span >= (uint32_t)kTile + 16u ? span : 0u;
  uint32_t r = (uint32_t)(uni64(entry) - tile_lo);  // relative chain position (entry < tile_hi)
  uint32_t n = 0;                                   // record offsets stored in srec
  uint32_t last = last_io ? *last_io : kAnyLen;     // the previous record's incl_len
  uint64_t exit_far = kNone;  // a record longer than a tile: the chain leaves at this offset
  while (r < span) {
    const uint32_t incl = big ? incl_at<true>(w, r) : incl_at<false>(w, r);
    if (last == kAnyLen) last = incl;
    const uint32_t e = incl + 16u;
    if (e < 16u || e > avail - r) {  // (32-bit test; exact below when avail was clamped)
      const uint64_t room = av - r;
      if (room < 16 || room - 16 < incl) break;  // Err(Incomplete) -> stop (:37-45)
    }
    // a record longer than a tile (no stride to speculate on), or one whose length differs from
    // the previous record's (variable-length traffic: a stride guess would confirm only itself):
    // hops, one header read each
    if (incl > (uint32_t)kTile) {  // the chain leaves the tile with this record
      srec[n] = (uint16_t)r;
      ++n;
      last = incl;
      exit_far = tile_lo + r + 16ull + incl;
      break;
    }
    if (incl != last) {
      r = big ? hop_run<true>(w, srec, r, incl, hop_span, n, last) : hop_run<false>(w, srec, r, incl, hop_span, n, last);
      continue;
    }
    const uint32_t stride = e;
    if (span - r <= 64u * stride) {  // one header per lane reaches the tile's end: a single read
      const uint32_t q0 = r + lane * stride;
      uint32_t h0 = hdr(w, q0 < span ? q0 : 0u, 2, big);
      asm volatile("" : "+v"(h0));
      const uint64_t b0 = __ballot((lane == 0) | ((q0 < span) & (h0 == incl) & (avail - q0 >= stride)));
      const uint32_t m = (~b0 == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~b0);
      srec[n + lane] = (uint16_t)q0;
      n += m;
      r += m * stride;
      continue;
    }
    uint64_t b[kWalkUnroll];
    uint32_t qr[kWalkUnroll];
    uint32_t h[kWalkUnroll];
#pragma unroll
    for (int u = 0; u < kWalkUnroll; ++u) {  // all header reads issued together, unconditionally
      qr[u] = r + (lane + 64u * (uint32_t)u) * stride;  // < 2^24: k < 256, stride <= 16 + kTile
      h[u] = hdr(w, qr[u] < span ? qr[u] : 0u, 2, big);
    }
#pragma unroll
    for (int u = 0; u < kWalkUnroll; ++u) asm volatile("" : "+v"(h[u]));  // no load sinking
#pragma unroll
    for (int u = 0; u < kWalkUnroll; ++u)  // bitwise, not short-circuit: no branches
      b[u] = __ballot(((lane == 0) & (u == 0)) | ((qr[u] < span) & (h[u] == incl) & (avail - qr[u] >= stride)));
    uint32_t m = 0;
#pragma unroll
    for (int u = 0; u < kWalkUnroll; ++u) {
      if (m != 64u * (uint32_t)u) break;
      m += (~b[u] == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~b[u]);
    }
    // unconditional stores: lanes past m write beyond the chain's records, into slots the next
    // step (or nothing) overwrites; srec holds 2 * kMaxRec entries so no index overflows
#pragma unroll
    for (int u = 0; u < kWalkUnroll; ++u) srec[n + lane + 64u * (uint32_t)u] = (uint16_t)qr[u];
    n += m;
    r += m * stride;
  }
  n_out = n;
  if (last_io) *last_io = last;
  return exit_far != kNone ? exit_far : tile_lo + r;
}
// (the resident pass inlines walk_tile_inl: a call there keeps its length state in scratch
// memory; the two-pass kernels call this out-of-line copy, which keeps their registers free)
__device__ uint64_t walk_tile(const ParseParams &kp, const uint32_t *w, uint16_t *srec, uint64_t tile_lo,
                              uint64_t tile_hi, uint64_t entry, uint32_t &n_out, uint32_t *last_io = nullptr) {
  return walk_tile_inl(kp, w, srec, tile_lo, tile_hi, entry, n_out, last_io);
}

// diagnostics (DIAG kernel variants only: the production kernels carry none of this)
struct Stamps {  // kept in registers, written once at the end (a store per stamp would make
  uint64_t v[kStampWords];  // later vmcnt waits wait for it and skew what is measured)
};
__device__ __forceinline__ void stamp_at(Stamps &st, int k) { st.v[k] = __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ void stamp_flush(const ParseParams &kp, const Stamps &st, uint32_t t, uint32_t mask) {
  if (kp.stamps && (threadIdx.x & 63u) == 0)
    for (int k = 0; k < kStampWords; ++k)
      if (mask & (1u << k)) kp.stamps[(uint64_t)t * kStampWords + k] = st.v[k];
}



// First strong (else first weak) record start in [lo, span) of the staged tile; kNone if
// neither (wave-uniform).  64 candidates per round are screened on their own header (one
// 16-B read per lane); only the survivors, in offset order, have their chain graded.
// (the capture's length by value, not the ParseParams: a by-reference kernel argument reaching a
// call the compiler does not inline is copied to scratch memory first)
__device__ __forceinline__ uint64_t speculate(SpecCtx sc, uint64_t len, const uint32_t *w, uint64_t tile_lo, uint32_t lo,
                              uint32_t span) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t avail = len - tile_lo;
  sc.avail = avail > 0xffffffffull ? 0xffffffffu : (uint32_t)avail;
  sc.exact_end = avail <= 0xffffffffull;
  uint32_t weak = 0xffffffffu;
  for (uint32_t base = lo; base < span; base += 64) {
    const uint32_t r = base + lane;
    uint32_t h[4];
    hdr4(w, r < span ? r : 0u, sc.big, h);
    uint64_t m = __ballot(r < span && head_ok(sc, h, r));
    while (m) {
      const int j = __builtin_ctzll(m);
      m &= m - 1;
      const uint32_t c = base + (uint32_t)j;
      const uint32_t ts = (uint32_t)__builtin_amdgcn_readlane((int)h[0], j);
      const uint32_t incl = (uint32_t)__builtin_amdgcn_readlane((int)h[2], j);
      int g = stride_grade(sc, w, c, ts, incl);
      if (g < 0) g = chain_grade(sc, w, c, ts, incl);  // record lengths differ: hop by hop
      if (g == 2) return tile_lo + base + (uint32_t)j;
      if (g == 1 && weak == 0xffffffffu) weak = base + (uint32_t)j;
    }
  }
  return weak == 0xffffffffu ? kNone : tile_lo + weak;
}

// one npr_flow row (8 words) / its IPv6 side row, 16-B stores
__device__ __forceinline__ void put_flow(uint32_t *row, const FlowWords &f, uint64_t p) {
  u32x4 *d = reinterpret_cast<u32x4 *>(row);
  d[0] = u32x4{f.d[0], f.d[1], f.d[2], f.d[3]};
  d[1] = u32x4{f.d[4], f.d[5], f.d[6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8)};
}
__device__ __forceinline__ void put_v6(uint32_t *row, const FlowWords &f) {
  u32x4 *d = reinterpret_cast<u32x4 *>(row);
  d[0] = u32x4{f.v6[0], f.v6[1], f.v6[2], f.v6[3]};
  d[1] = u32x4{f.v6[4], f.v6[5], f.v6[6], f.v6[7]};
}


// ---- LDS-DMA staging --------------------------------------------------------------------------
// A tile lands in LDS straight from HBM (`buffer_load_dwordx4 ... lds`, 1 KiB per instruction,
// range-checked: bytes past the input read 0) with no registers held in flight: kTile/1024 rows
// of 16 B per lane, then one 256-B halo row of 4 B per lane.
constexpr int kRows = kTile / 1024;
constexpr int kSlotWords = kTile / 4 + 64;  // tile + 256-B halo row (>= kStage + the decoder's 72-B over-read)
static_assert(kHalo <= 256 - 80, "halo row must hold the halo + the decode over-read");
typedef __attribute__((address_space(3))) void *lds_ptr_t;

// aux = cache policy: the resident pass reads the capture exactly once (nt: 33.1 vs 33.8 us per
// launch at C2); the two-pass kernels re-read it from the Infinity Cache in pass 2 (default policy)
template <int AUX = 0>
__device__ __forceinline__ void dma_tile(const ParseParams &kp, uint64_t tile_lo, uint32_t *dst) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t avail = kp.len > tile_lo ? kp.len - tile_lo : 0;
  const uint32_t nbytes = avail < (uint64_t)kStage ? (uint32_t)avail : (uint32_t)kStage;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(kp.buf + tile_lo), 0, (int)((nbytes + 15u) & ~15u), 0x00020000);
  // each row's voffset is formed right at its load (volatile: never hoisted), so only lane * 16
  // stays live across the parse: five loop-invariant offsets kept in VGPRs were spilled to scratch
  // under the resident passes' register budget, and every reload drained the ring (vmcnt(0))
  const uint32_t l16 = lane * 16u;
#pragma unroll
  for (int i = 0; i < kRows; ++i) {
    uint32_t vo;
    asm volatile("v_or_b32 %0, %1, %2" : "=v"(vo) : "n"(1024 * i), "v"(l16));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + i * 256), 16, vo, 0, 0, AUX);
  }
  uint32_t vh;
  asm volatile("v_lshrrev_b32 %0, 2, %1\n\tv_or_b32 %0, %2, %0" : "=&v"(vh) : "v"(l16), "n"(kTile));
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + kRows * 256), 4, vh, 0, 0, AUX);
}
// pass 1's record offsets of tile t (kMaxRec u16) -> LDS
__device__ __forceinline__ void dma_offsets(const ParseParams &kp, uint32_t t, uint16_t *dst) {
  const uint32_t lane = threadIdx.x & 63u;
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc((void *)(kp.srec_g + (uint64_t)t * kMaxRec), 0, kMaxRec * 2, 0x00020000);
#pragma unroll
  for (int i = 0; i < kMaxRec / 128; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, (lds_ptr_t)(reinterpret_cast<uint32_t *>(dst) + i * 64), 4,
                                             lane * 4u + 256u * (uint32_t)i, 0, 0, 0);
}
__device__ __forceinline__ void wait_all_vmem() {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  wave_sync();                         // LDS reads of the landed bytes stay below the wait
}

struct TileShared {  // one wave's LDS
  uint32_t data[kSlotWords];   // the staged tile + halo
  uint16_t srec[2 * kMaxRec];  // record offsets (+ room for the walk's unconditional stores)
};

// ---------------------------------------------------------------------------------------------
// pass 1: k_count_tiles — ONE WAVE per tile, no waits on other tiles (bar the folds below).
//   stage the tile | entry: `start` for tile 0, else a speculated record start | walk ->
//   record offsets (kept in the scratch for pass 2) | status-only decode -> Ok count |
//   publish A = {entry, exit, n, Ok count}.  The wave that produced the LAST child of a group
//   (64 tiles), block (64 groups) or super-block (64 blocks) then folds it: the group's
//   aggregate and each child's exclusive prefix inside it (chain-consistency monoid).
// ---------------------------------------------------------------------------------------------
template <bool DIAG>
__global__ __launch_bounds__(kWave) void k_count_tiles(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) TileShared sh;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t t = blockIdx.x;
  Stamps st;
  const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
  const uint64_t tile_hi = tile_lo + kTile < kp.stop ? tile_lo + kTile : kp.stop;
  if (DIAG) stamp_at(st, 0);
  dma_tile(kp, tile_lo, sh.data);
  const bool spec0 = (kp.flags & kFlagSpecStart) != 0;
  const bool known = t == 0 && !spec0;  // tile 0 of a capture starts at `start`
  const uint32_t scb = known ? 0u : spec_ctx_load(kp);
  wait_all_vmem();
  if (DIAG) stamp_at(st, 1);
  const uint32_t *w = sh.data;

  uint64_t entry = kp.start;
  if (!known) {
    const SpecCtx sc = spec_ctx(kp, scb);
    const uint32_t lo = t == 0 ? (uint32_t)(kp.start - tile_lo) : 0u;  // a range starts at `start`
    entry = tile_hi > tile_lo + lo ? speculate(sc, kp.len, w, tile_lo, lo, (uint32_t)(tile_hi - tile_lo)) : kNone;
    if (DIAG && kp.stats && lane == 0 && entry == kNone) atomicAdd(kp.stats + kStatNoEntry, 1u);
  }
  entry = uni64(entry);
  if (DIAG) stamp_at(st, 8);
  uint32_t n = 0;
  uint64_t ex = entry == kNone ? 0ull : entry;
  if (entry != kNone && entry >= tile_lo && entry < tile_hi) ex = walk_tile(kp, w, sh.srec, tile_lo, tile_hi, entry, n);
  ex = uni64(ex);
  wave_sync();
  if (DIAG) stamp_at(st, 9);

  // record offsets -> scratch ((n + 1) / 2 u16 pairs; the descriptor's range drops the rest)
  if (kp.srec_g && n) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(sh.srec);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(kp.srec_g + (uint64_t)t * kMaxRec), 0, (int)(((n + 1) / 2) * 4u), 0x00020000);
#pragma unroll
    for (int i = 0; i < kMaxRec / 128; ++i)
      __builtin_amdgcn_raw_buffer_store_b32(src[lane + 64u * (uint32_t)i], rs, (int)(lane * 4u + 256u * (uint32_t)i), 0, 0);
  }
  if (DIAG) stamp_at(st, 10);
  // Ok count: status-only decode of every record
  uint32_t okc = 0;
  for (int s = 0; s < kRounds; ++s) {
    if ((uint32_t)s * 64u >= n) break;
    const uint32_t i = lane + (uint32_t)s * 64u;
    const bool valid = i < n;  // every lane decodes (stale offsets are in-bounds), masked after
    FlowWords f;
    const bool ok = decode_rec<false>(kp, w, tile_lo, sh.srec[i], f, valid) == NPR_FLOW_OK && valid;
    okc += (uint32_t)__builtin_popcountll(__ballot(ok));
  }
  if (DIAG) stamp_at(st, 11);
  if (lane == 0) {
    TileSlot *slot_t = kp.slots + t;
    const uint32_t ep = kp.epoch;
    st_agent(&slot_t->a[0], gran(ep, ex));
    st_agent(&slot_t->a[1], gran(ep, entry == kNone ? 0ull : entry + 1));
    st_agent(&slot_t->a[2], gran(ep, (uint64_t)n | ((uint64_t)okc << 24)));
  }
  if (DIAG) stamp_at(st, 2);
  // Fold the group this tile is the folder of, then (when that group is the last of its block)
  // the block, then the super-block.  A group's folder is one of its last 8 tiles, rotating with
  // the group index: consecutive tiles are dealt round-robin over the 8 XCDs, so a fixed member
  // (say the last) would put every fold wait on one XCD and leave it trailing the others.  The
  // folder waits (bounded) for its group's tiles, all dispatched at most 7 tiles after it.
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t grp = t >> 6;
  const int64_t glast = (grp << 6) + 63 < (int64_t)kp.ntiles - 1 ? (grp << 6) + 63 : (int64_t)kp.ntiles - 1;
  const int64_t folder = (grp << 6) + 56 + (grp & 7) < glast ? (grp << 6) + 56 + (grp & 7) : glast;
  if ((int64_t)t == folder) {
    int64_t idx = grp;
    for (int lvl = 1; lvl <= kLevels; ++lvl) {
      if (!fold_children<DIAG>(kp, lvl, idx, t0)) break;
      const int64_t nself = (int64_t)kp.ngroups[lvl];  // elements of this level
      const int64_t par = idx >> 6;
      const int64_t plast = (par << 6) + 63 < nself - 1 ? (par << 6) + 63 : nself - 1;
      if (idx != plast || lvl == kLevels) break;  // the parent is folded by its last child's folder
      idx = par;
    }
  }
  if (DIAG) stamp_at(st, 3);
  if (DIAG) stamp_flush(kp, st, t, 0xF0Fu);
}

// ---------------------------------------------------------------------------------------------
// pass 2: k_emit_tiles — ONE WAVE per tile.  The exact chain state before tile t is
//   anchor ⊕ G3(super-blocks before) ⊕ E(block) ⊕ E(group) ⊕ E(tile)
// where E(x) is x's exclusive prefix inside its parent, folded by pass 1: four point loads
// (plus a window of level-3 aggregates past 1 GiB), issued together with the tile's DMA.  A
// contradiction (a mis-speculated tile m < t) is settled by m's exact prefix P(m), published
// below by m's own wave.  Then: the record offsets (pass 1's when its entry was the exact
// position, else a walk) | decode every record | record table / status | Ok flows straight to
// their convert_records (reverse-order) rows, ranked by ballot | publish P(t).
// ---------------------------------------------------------------------------------------------
template <bool DIAG>
__global__ __launch_bounds__(kWave) void k_emit_tiles(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) TileShared sh;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t t = blockIdx.x;
  Stamps st;
  const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
  const uint64_t tile_hi = tile_lo + kTile < kp.stop ? tile_lo + kTile : kp.stop;
  if (DIAG) stamp_at(st, 5);
  dma_tile(kp, tile_lo, sh.data);
  if (kp.srec_g) dma_offsets(kp, t, sh.srec);
  // context words, one per lane, from the slot allocation (tile slots, then the level-1/2/3
  // group slots): A(t) [0,3), E(t) [3,8) (a and e are adjacent), E(group) [8,13), E(block)
  // [13,18), A(0).entry [18] (the anchor of a speculative start)
  const uint32_t g = t >> 6, h = t >> 12, sup = t >> 18;
  const uint32_t og1 = (uint32_t)((const char *)kp.groups[1] - (const char *)kp.slots);
  const uint32_t og2 = (uint32_t)((const char *)kp.groups[2] - (const char *)kp.slots);
  const uint32_t off = lane < 8u    ? t * 128u + lane * 8u
                       : lane < 13u ? og1 + g * 128u + 40u + (lane - 8u) * 8u
                       : lane < 18u ? og2 + h * 128u + 40u + (lane - 13u) * 8u
                       : lane == 18u ? 8u : 0x7ffffff8u;  // past the range: 0
  const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)kp.slots, 0, 0x7ffffff8, 0x00020000);
  const uint32_t vlo = __builtin_amdgcn_raw_buffer_load_b32(rc, (int)off, 0, 0);
  const uint32_t vhi = __builtin_amdgcn_raw_buffer_load_b32(rc, (int)off + 4, 0, 0);
  wait_all_vmem();
  const uint64_t v = ((uint64_t)vhi << 32) | vlo;
  const bool spec0 = (kp.flags & kFlagSpecStart) != 0;
  if (__ballot(lane < 18u + (spec0 ? 1u : 0u) && !tagged(v, kp.epoch))) return;  // pass 1 aborted
  if (DIAG) stamp_at(st, 12);
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();

  // ---- exact prefix before t: anchor, then E(block), E(group), E(tile).  Fast path: each prefix
  // is empty, or valid with its entry exactly where the chain stands (then it is a plain sum).
  uint64_t entry0 = kp.start, xe = kp.start, xc = 0, xo = 0;
  if (spec0) {
    const uint64_t e1 = rl64(v, 18) & kMask48;
    entry0 = e1 ? e1 - 1 : kNone;
    xe = e1 ? e1 - 1 : kp.stop;
  }
  bool fast = sup == 0;
#pragma unroll
  for (int k = 2; k >= 0; --k) {
    const int b = k == 2 ? 13 : (k == 1 ? 8 : 3);
    const uint64_t pok = rl64(v, b + kPreOk);
    const bool empty = (pok >> 33) & 1ull, valid = (pok >> 32) & 1ull;
    if (!empty) {
      const uint64_t en = rl64(v, b + kPreEntry) & kMask48;
      fast = fast && valid && en == xe + 1;
      xe = rl64(v, b + kPreExit) & kMask48;
      xc += rl64(v, b + kPreCnt) & kMask48;
      xo += pok & 0xffffffffull;
    }
  }
  Seg X;
  if (fast) {
    X.exit = xe;
    X.cnt = xc;
    X.ok = xo;
  } else {  // the general monoid: ends, pass-throughs, mis-speculations, > 1 GiB before t
    X = start_seg(kp);
    if (spec0) X.entry = X.exit = entry0 == kNone ? kp.stop : entry0;
    for (int64_t b = 0; b < sup; b += 64) {  // level-3 aggregates before this super-block
      Seg Y;
      const int64_t cnt = sup - b < 64 ? sup - b : 64;
      if (!fold_range(kp, kLevels, b, (int)cnt, Y, t0)) return;
      X = combine(kp, X, Y);
    }
    bool empty;
    Seg E = prefix_seg(rl64(v, 13), rl64(v, 14), rl64(v, 15), rl64(v, 16), rl64(v, 17), 2, h, empty);
    if (!empty) X = combine(kp, X, E);
    E = prefix_seg(rl64(v, 8), rl64(v, 9), rl64(v, 10), rl64(v, 11), rl64(v, 12), 1, g, empty);
    if (!empty) X = combine(kp, X, E);
    E = prefix_seg(rl64(v, 3), rl64(v, 4), rl64(v, 5), rl64(v, 6), rl64(v, 7), 0, t, empty);
    if (!empty) X = combine(kp, X, E);
    if (!X.valid && !prefix_generic<DIAG>(kp, X, t, t, X, t0)) return;
  }
  if (DIAG) stamp_at(st, 6);

  // ---- this tile's records, from the exact chain position
  const uint64_t pos = uni64(X.exit), pcnt = uni64(X.cnt), pok = uni64(X.ok);
  const uint64_t a0 = rl64(v, 0) & kMask48, a1 = rl64(v, 1) & kMask48, a2 = rl64(v, 2) & kMask48;
  uint32_t n = 0;
  uint64_t ex = pos;
  if (pos >= tile_lo && pos < tile_hi) {
    if (kp.srec_g && a1 == pos + 1) {  // pass 1 walked from the exact entry: reuse its offsets
      n = (uint32_t)(a2 & 0xffffffull);
      ex = a0;
    } else {
      ex = uni64(walk_tile(kp, sh.data, sh.srec, tile_lo, tile_hi, pos, n));
      wave_sync();
      if (DIAG && kp.stats && lane == 0) atomicAdd(kp.stats + kStatRewalk, 1u);
    }
  }
  if (DIAG) stamp_at(st, 13);
  const uint32_t *w = sh.data;
  uint32_t okbase = 0;
  for (int s = 0; s < kRounds; ++s) {
    if ((uint32_t)s * 64u >= n) break;
    const uint32_t i = lane + (uint32_t)s * 64u;
    const bool valid = i < n;  // every lane decodes (stale offsets are in-bounds), masked after
    FlowWords f;
    const uint32_t rel = sh.srec[i];
    const uint32_t st = decode_rec<true>(kp, w, tile_lo, rel, f, valid);
    const bool ok = st == NPR_FLOW_OK && valid;
    if (valid && (kp.rec_status || kp.rec_off || kp.recs)) {
      const uint64_t p = tile_lo + rel;
      const uint64_t idx = pcnt + i;
      if (idx < kp.rec_cap) {
        if (kp.rec_status) kp.rec_status[idx] = (uint8_t)st;
        if (kp.rec_off) kp.rec_off[idx] = p;
        if (kp.recs) {
          const bool big = kp.big;
          uint64_t *row = reinterpret_cast<uint64_t *>(kp.recs + idx);
          row[0] = p;
          row[1] = (uint64_t)hdr(w, rel, 0, big) | ((uint64_t)hdr(w, rel, 1, big) << 32);
          row[2] = (uint64_t)hdr(w, rel, 2, big) | ((uint64_t)hdr(w, rel, 3, big) << 32);
        }
      }
    }
    const uint64_t bal = __ballot(ok);
    if (ok && kp.flows) {
      const uint64_t fi = pok + okbase + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      if (fi < kp.flow_cap) {
        const uint64_t o = kp.flow_cap - 1 - fi;  // convert_records pops from the end
        put_flow(kp.flows + o * 8, f, tile_lo + rel);
        if (kp.flows_v6 && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16))) put_v6(kp.flows_v6 + o * 8, f);
      }
    }
    okbase += (uint32_t)__builtin_popcountll(bal);
  }
  if (DIAG) stamp_at(st, 14);
  const uint64_t ncnt = pcnt + n, nok = pok + okbase;
  if (lane == 0) {
    const uint32_t ep = kp.epoch;
    TileSlot *slot_t = kp.slots + t;
    st_agent(&slot_t->p[0], gran(ep, ex));
    st_agent(&slot_t->p[1], gran(ep, ncnt));
    st_agent(&slot_t->p[2], gran(ep, nok));
    if (t == kp.ntiles - 1) {
      uint32_t fl = 0;
      if ((kp.rec_off || kp.recs || kp.rec_status) && ncnt > kp.rec_cap) fl |= NPR_SUMMARY_RECORD_OVERFLOW;
      if (kp.flows && nok > kp.flow_cap) fl |= NPR_SUMMARY_FLOW_OVERFLOW;
      kp.summary->n_records = ncnt;
      kp.summary->n_flows = nok;
      kp.summary->consumed = ex;
      kp.summary->flags = fl;
      kp.summary->entry = entry0;
      kp.summary->epoch = kp.epoch;
    }
  }
  if (DIAG) stamp_at(st, 7);
  if (DIAG) stamp_flush(kp, st, t, 0x70E0u);
}

// =============================================================================================
// RESIDENT SINGLE PASS — k_parse_resident (flows-only launches: the `extract` bench's output)
//
// ONE launch of W persistent waves in workgroups of kResWg (16: one workgroup per CU, 4 waves per
// SIMD); wave v = b * kResWg + wid owns the contiguous tile range [c0(v), c1(v)).  Every byte of
// the capture is read once:
//   phase A: the range streams through a two-slot LDS ring per wave (LDS-DMA, the next tile in
//     flight while the current one is parsed); the chain is speculated ONCE, at the range's first
//     tile (wave 0: `start`), then walked tile to tile (stride speculation for repeating lengths,
//     hop_run for variable ones); every record is decoded with its fields and the Ok flows of each
//     64-record round are KEPT IN REGISTERS (kResSlots rounds; PACK: sparse tiles share the last
//     round; later rounds are deferred to phase B).  The wave's range aggregate A(v) = {exit,
//     entry, records, Ok flows} goes to LDS (and to its RangeSlot for the rare generic prefix).
//   the prefix: wave 0 folds the workgroup's 16 A's in LDS (chain-consistency monoid), publishes
//     the workgroup aggregate G(b) and looks back over G(0..b-1) of the LOWER workgroups (all
//     windows loaded at once, only unpublished lanes re-read by returning atomics with backed-off
//     naps): E(b) = anchor (or the previous link's summary) ⊕ G(0) ⊕ ... ⊕ G(b-1), then each
//     wave's prefix X(v) = E(b) ⊕ A(waves before v in b) in LDS.  All workgroups are co-resident
//     (the host sizes the grid by the occupancy query) and every wait is bounded.
//   phase B: when X(v).exit is v's speculated entry (the common case), the register-held flows go
//     straight to their convert_records rows flow_cap - 1 - (X.ok + rank) and only deferred tiles
//     are re-read; otherwise the range is re-walked from the exact position.  A contradiction below
//     v waits for the offending wave's exact prefix P(m), published at the end of its own phase B.
// =============================================================================================
constexpr int kResRing = 2;               // LDS tile slots per wave (1 processed + kResRing-1 in flight)
constexpr int kDmaPer = kRows + 1;        // DMA instructions per staged tile
constexpr uint32_t kResWg = 16;           // waves per workgroup (one workgroup per CU): folded in LDS
static_assert(kResWg >= kResWgMin, "workgroup aggregate slots (npr_capi.hip group_slots) are sized for kResWgMin");
static_assert(kResWg == kResWgMin, "the host's per-workgroup tile split (ParseParams::wg_q) counts kResWgMin waves");
static_assert(kResRing >= 2 && (kResRing - 1) * kDmaPer < 64, "vmcnt field is 6 bits");

struct ResShared {  // one wave's LDS
  uint32_t data[kResRing][kSlotWords];
  uint16_t srec[2 * kMaxRec];
};

// wave v's tiles: q = ntiles / nwaves each, one more for the first ntiles % nwaves waves (the
// last-dispatched waves start latest, so they get the shorter ranges)
// Whole workgroups (kp.wg_q != 0): workgroup b holds wg_q tiles, one more for b < wg_r, so every CU
// parses the same number (C2: 76-77 tiles, where the per-wave split gave 80 or 64); its waves split
// them in order, the extra tiles going to the lowest waves -- the oldest on each SIMD, which the
// arbiter favours (per-wave phase A ended 1.7 us later for waves 12-15 than for waves 0-3 of a
// workgroup, profiles/r06_stamps_rereads.txt).  Otherwise q = ntiles / nwaves per wave.
__device__ __forceinline__ void res_wg_range(const ParseParams &kp, uint32_t b, uint32_t &g0, uint32_t &gs) {
  g0 = b * kp.wg_q + (b < kp.wg_r ? b : kp.wg_r);
  gs = kp.wg_q + (b < kp.wg_r ? 1u : 0u);
}
__device__ __forceinline__ void res_range(const ParseParams &kp, uint32_t v, uint32_t &c0, uint32_t &c1) {
  if (kp.wg_q) {
    uint32_t g0, gs;
    res_wg_range(kp, v / kResWg, g0, gs);
    const uint32_t w = v % kResWg, q = gs / kResWg, r = gs % kResWg;
    c0 = g0 + w * q + (w < r ? w : r);
    c1 = c0 + q + (w < r ? 1u : 0u);
    return;
  }
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves;
  c0 = v * q + (v < r ? v : r);
  c1 = c0 + q + (v < r ? 1u : 0u);
}
// the wave whose range holds tile m
__device__ __forceinline__ uint32_t res_wave_of(const ParseParams &kp, int64_t m) {
  if (kp.wg_q) {
    const uint32_t t = (uint32_t)m, big = kp.wg_r * (kp.wg_q + 1u);
    const uint32_t b = t < big ? t / (kp.wg_q + 1u) : kp.wg_r + (t - big) / kp.wg_q;
    uint32_t g0, gs;
    res_wg_range(kp, b, g0, gs);
    const uint32_t q = gs / kResWg, r = gs % kResWg, u = t - g0, big2 = r * (q + 1u);
    return b * kResWg + (u < big2 ? u / (q + 1u) : r + (u - big2) / q);
  }
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves;
  const uint64_t big = (uint64_t)r * (q + 1);
  return (uint64_t)m < big ? (uint32_t)((uint64_t)m / (q + 1)) : (uint32_t)(r + ((uint64_t)m - big) / q);
}
constexpr uint32_t kStepPrioTiles = 8;  // wave ranges up to this many tiles use stepped priorities
// wait until at most `ahead` tiles' DMAs are outstanding (the youngest vector-memory
// instructions are the DMAs of the tiles ahead and at least PF prefetches, so this retires the
// current tile)
template <int PF>
__device__ __forceinline__ void res_wait(uint32_t ahead) {
  constexpr int w0 = PF, w1 = kDmaPer + PF, w2 = 2 * kDmaPer + PF;
  if (ahead == 0) __builtin_amdgcn_s_waitcnt(0x0F70 | (w0 & 15) | ((w0 >> 4) << 14));
  else if (ahead == 1 || kResRing <= 2) __builtin_amdgcn_s_waitcnt(0x0F70 | (w1 & 15) | ((w1 >> 4) << 14));
  else __builtin_amdgcn_s_waitcnt(0x0F70 | (w2 & 15) | ((w2 >> 4) << 14));
  wave_sync();
}

// Waiting waves must not steal issue slots and memory requests from the waves still in phase A
// (a window poll is 64 lanes x 5 granules): wait on ONE sentinel granule with a backed-off
// s_sleep first, load whole windows only once it is there.
__device__ __forceinline__ bool res_nap(const ParseParams &kp, uint64_t t0, uint32_t &nap) {
  // (shorter naps, or the abort word read every 16th nap only, measured 3.5-4.5 us slower at C2)
  for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(8);  // ~512 clocks each
  nap = nap < 2u ? nap * 2u : 2u;
  if (__hip_atomic_load(kp.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kp.epoch) return false;
  if (__builtin_amdgcn_s_memrealtime() - t0 > kp.timeout_ticks) {
    __hip_atomic_store(kp.abort_word, kp.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}
__device__ __forceinline__ uint64_t ld_res(uint64_t *p);
__device__ __forceinline__ bool res_sentinel(const ParseParams &kp, uint64_t *p, uint64_t t0) {
  uint32_t nap = 1;
  while (!tagged(uni64(ld_res(p)), kp.epoch))
    if (!res_nap(kp, t0, nap)) return false;
  return true;
}

// hand-off granule read: a returning atomic (the coherent value even when this XCD's L2 holds a
// line from an earlier poll)
__device__ __forceinline__ uint64_t ld_res(uint64_t *p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane's element of a window: lvl 0 = wave v's A, lvl 1 = workgroup b's aggregate G(b)
// the tiles [first, last] of element idx (lvl 0: wave idx; lvl 1: workgroup idx)
__device__ __forceinline__ void res_tiles(const ParseParams &kp, int lvl, int64_t idx, LaneSeg &L) {
  uint32_t c0, c1, d0, d1;
  const uint32_t v0 = lvl == 0 ? (uint32_t)idx : (uint32_t)idx * kResWg;
  const uint32_t v1 = lvl == 0 ? (uint32_t)idx : v0 + kResWg - 1u < kp.nwaves - 1 ? v0 + kResWg - 1u : kp.nwaves - 1;
  res_range(kp, v0, c0, c1);
  res_range(kp, v1, d0, d1);
  L.first = c0;
  L.last = (int64_t)d1 - 1;
}
// (tiles = false: first / last left for the caller -- the look-back sets them once its windows
// are in, so they are not live across its polls)
__device__ __forceinline__ LaneSeg load_res(const ParseParams &kp, int lvl, int64_t idx, bool inr, bool sc1 = false,
                                            bool tiles = true) {
  LaneSeg L{};
  L.mism = -1;
  L.valid = true;
  if (!inr) return L;
  if (tiles) res_tiles(kp, lvl, idx, L);
  const uint32_t ep = kp.epoch;
  uint64_t *w = lvl == 0 ? kp.rslots[idx].a : kp.rgroups[idx].g;
  uint64_t w0, w1, w2, w3, w4;
  if (sc1) {  // sc1 loads: fast, but may hit a stale line (the tags tell; callers re-read those)
    w0 = ld_agent(w + 0), w1 = ld_agent(w + 1), w2 = ld_agent(w + 2), w3 = ld_agent(w + 3);
    w4 = lvl == 0 ? w0 : ld_agent(w + 4);
  } else {
    w0 = ld_res(w + 0), w1 = ld_res(w + 1), w2 = ld_res(w + 2), w3 = ld_res(w + 3);
    w4 = lvl == 0 ? w0 : ld_res(w + 4);
  }
  L.present = tagged(w0, ep) && tagged(w1, ep) && tagged(w2, ep) && tagged(w3, ep) && tagged(w4, ep);
  const uint64_t e1 = w1 & kMask48;
  L.entry = e1 ? e1 - 1 : kNone;
  L.exit = w0 & kMask48;
  L.cnt = w2 & kMask48;
  if (lvl == 0) {
    L.ok = w3 & kMask48;
  } else {
    const uint64_t v3 = w3 & kMask48, m = w4 & kMask48;
    L.ok = v3 & 0xffffffffull;
    L.valid = (v3 >> 32) & 1ull;
    L.mism = L.valid ? -1 : (int64_t)m - 1;
  }
  return L;
}

// fold `cnt` (1..64) consecutive level-`lvl` elements from `base` (bounded wait for all)
__device__ __forceinline__ bool res_fold(const ParseParams &kp, int lvl, int64_t base, int cnt, Seg &out, uint64_t t0) {
  const int lane = (int)(threadIdx.x & 63u);
  const bool inr = lane < cnt;
  const int64_t last = base + cnt - 1;
  if (!res_sentinel(kp, lvl == 0 ? &kp.rslots[last].a[3] : &kp.rgroups[last].g[4], t0)) return false;
  uint32_t nap = 1;
  for (;;) {
    const LaneSeg L = load_res(kp, lvl, last - lane, inr);
    if (__ballot(inr && !L.present) == 0ull) {
      out = fold_window(kp, L, cnt - 1);
      return true;
    }
    if (!res_nap(kp, t0, nap)) return false;
  }
}

// Pacing arrival on the launch's one counter word: a returning atomic whose round trip delays
// the caller's first look-back read.  Nothing reads the count (it wraps freely).
__device__ __forceinline__ uint32_t res_arrive(uint32_t *ctr) {
  return __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// Fold a window of `size` children held one per lane (ascending lane = ascending order): each
// lane's exclusive prefix inside the window (lane 0: none) and the window's aggregate (the chain-
// consistency monoid; fast path: every link consistent -> two exclusive scans).
__device__ __forceinline__ void res_fold_lanes(const ParseParams &kp, const LaneSeg &L, int size, Seg &ep, Seg &agg) {
  const int lane = (int)(threadIdx.x & 63u);
  const bool inr = lane < size;
  const uint64_t prev_exit = shfl_up64(L.exit);
  const bool link_bad = inr && (!L.valid || (lane > 0 && L.entry != prev_exit));
  const bool end_mid = lane < size - 1 && L.exit < tile_end(kp, L.last);
  ep = Seg{};
  if (__ballot(link_bad || end_mid) == 0ull) {
    const uint32_t c = inr ? (uint32_t)L.cnt : 0u, o = inr ? (uint32_t)L.ok : 0u;
    const uint32_t cx = excl_scan_u32(c), ox = excl_scan_u32(o);
    ep.entry = rl64(L.entry, 0);
    ep.exit = prev_exit;
    ep.cnt = cx;
    ep.ok = ox;
    ep.first = (int64_t)rl64((uint64_t)L.first, 0);
    ep.last = (int64_t)shfl_up64((uint64_t)L.last);
    ep.valid = true;
    ep.mism = -1;
    agg.entry = ep.entry;
    agg.exit = rl64(L.exit, size - 1);
    agg.cnt = (uint32_t)__builtin_amdgcn_readlane((int)(cx + c), size - 1);
    agg.ok = (uint32_t)__builtin_amdgcn_readlane((int)(ox + o), size - 1);
    agg.first = ep.first;
    agg.last = (int64_t)rl64((uint64_t)L.last, size - 1);
    agg.valid = true;
    agg.mism = -1;
  } else {
    const uint64_t bval = __ballot(L.valid);
    Seg r{};
    for (int j = 0; j < size; ++j) {
      Seg y;
      y.entry = rl64(L.entry, j);
      y.exit = rl64(L.exit, j);
      y.cnt = rl64(L.cnt, j);
      y.ok = rl64(L.ok, j);
      y.first = (int64_t)rl64((uint64_t)L.first, j);
      y.last = (int64_t)rl64((uint64_t)L.last, j);
      y.mism = (int64_t)rl64((uint64_t)L.mism, j);
      y.valid = (bval >> j) & 1ull;
      if (j == 0) {
        r = y;
      } else {
        if (lane == j) ep = r;
        r = combine(kp, r, y);
      }
    }
    agg = r;
  }
}

constexpr int kTopWin = (int)((kResMaxWaves / kResWg + 63) / 64);  // windows of workgroup aggregates

// an exclusive prefix (kPre* words) as the segment of tiles [first, last]
__device__ __forceinline__ Seg res_prefix_seg(const ParseParams &kp, uint64_t *e, int64_t first, int64_t last,
                                              bool &empty) {
  const uint64_t e0 = ld_res(e + kPreExit), e1 = ld_res(e + kPreCnt), e2 = ld_res(e + kPreOk);
  const uint64_t e3 = ld_res(e + kPreMism), e4 = ld_res(e + kPreEntry);
  Seg s;
  const uint64_t v = e2 & kMask48, m = e3 & kMask48, en = e4 & kMask48;
  s.exit = e0 & kMask48;
  s.cnt = e1 & kMask48;
  s.ok = v & 0xffffffffull;
  s.valid = (v >> 32) & 1ull;
  empty = (v >> 33) & 1ull;
  s.mism = s.valid ? -1 : (int64_t)m - 1;
  s.entry = en ? en - 1 : kNone;
  s.first = first;
  s.last = last;
  return s;
}

// exact chain state before wave v, from X = E(b) ⊕ (prefix inside the workgroup) when that is
// flagged: contradictions settled by exact prefixes P(m), then aggregates (G(b) where aligned)
__device__ __forceinline__ bool res_prefix(const ParseParams &kp, uint32_t v, Seg &X, uint64_t t0, const Seg *own_a) {
  const uint32_t lane = threadIdx.x & 63u;
  if (X.valid) return true;
  // a mis-speculated range m < v: from its exact prefix on, aggregates (G1 where aligned)
  if (kp.stats && lane == 0) atomicAdd(kp.stats + kStatMismWait, 1u);
  for (;;) {
    uint32_t a;
    if (!X.valid) {
      const uint32_t m = res_wave_of(kp, X.mism);
      RangeSlot *s = kp.rslots + m;
      uint32_t nap = 1;
      for (;;) {
        const uint64_t p0 = ld_res(&s->p[0]), p1 = ld_res(&s->p[1]), p2 = ld_res(&s->p[2]);
        if (tagged(p0, kp.epoch) && tagged(p1, kp.epoch) && tagged(p2, kp.epoch)) {
          uint32_t c0, c1;
          res_range(kp, m, c0, c1);
          X.exit = p0 & kMask48;
          X.cnt = p1 & kMask48;
          X.ok = p2 & kMask48;
          X.first = 0;
          X.last = (int64_t)c1 - 1;
          X.mism = -1;
          X.valid = true;
          break;
        }
        if (!res_nap(kp, t0, nap)) return false;
      }
      a = m + 1;
    } else {
      return true;
    }
    while (a < v && X.valid) {
      Seg Y;
      if (a % kResWg == 0 && v - a >= kResWg) {
        const uint32_t ng = (v - a) / kResWg, take = ng < 64 ? ng : 64;
        if (!res_fold(kp, 1, a / kResWg, (int)take, Y, t0)) return false;
        a += take * kResWg;
      } else {
        const uint32_t to_grp = kResWg - a % kResWg, cnt = v - a < to_grp ? v - a : to_grp;
        if (a / kResWg == v / kResWg) {  // this workgroup's waves: their A's are in its LDS
          const uint32_t idx = a + cnt - 1u - lane;  // (descending, as res_fold)
          LaneSeg L{};
          L.mism = -1;
          L.valid = true;
          if (lane < cnt) {
            const Seg &A = own_a[idx % kResWg];
            L.entry = A.entry;
            L.exit = A.exit;
            L.cnt = A.cnt;
            L.ok = A.ok;
            L.first = A.first;
            L.last = A.last;
            L.present = true;
          }
          Y = fold_window(kp, L, (int)cnt - 1);
        } else if (!res_fold(kp, 0, a, (int)cnt, Y, t0)) {  // (a workgroup that published its A's)
          return false;
        }
        a += cnt;
      }
      X = combine(kp, X, Y);
    }
    if (X.valid) return true;
  }
}

// Row-block staging in LDS: 16-B chunk c of a block of N chunks (two per 32-B row) sits at slot
// stg_slot<N>(c): the rows' first halves (even c) in order, a 128-B pad, then their second halves.
// A row's two ds_write_b128 (one row per lane, 32-B stride) and the whole-line reads (chunk c by
// lane c) are then both bank-conflict-free; with chunk c at slot c the row stores were 2-way
// conflicted (round 2: 0.87 M of 2.46 M LDS cycles per C2 launch were conflict cycles).
template <uint32_t N>
__device__ __forceinline__ uint32_t stg_slot(uint32_t c) { return (c & 1u) ? N / 2u + 8u + (c >> 1) : c >> 1; }

constexpr int kPolSc1 = 16;  // buffer-store cache policy: sc1 (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16)
// 16-B flow-row store, one row per lane (IPv6 side rows, res_emit's re-read rows).  Plain (write-back):
// measured 33.9 us per launch against 38.1 us with write-through (sc1) stores in round 1's kernel,
// which stored every row this way (phase B's row blocks are written through since round 3).
__device__ __forceinline__ void st_wt16(uint32_t *p, u32x4 v) { *reinterpret_cast<u32x4 *>(p) = v; }

// one Ok flow row (+ its IPv6 side row, re-read from the capture at the decoded offset)
__device__ __forceinline__ void res_put_v6(const ParseParams &kp, uint64_t o, const uint32_t (&s)[8], uint64_t p);
__device__ __forceinline__ void res_put(const ParseParams &kp, uint64_t o, const uint32_t (&s)[8], uint64_t p) {
  const bool v6 = (s[6] & (NPR_FLOW_KIND_IPV6 << 16)) != 0;
  uint32_t *d = kp.flows + o * 8;
  st_wt16(d, u32x4{v6 ? 0u : s[0], v6 ? 0u : s[1], s[2], s[3]});
  st_wt16(d + 4, u32x4{s[4], s[5], s[6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8)});
  if (v6) res_put_v6(kp, o, s, p);
}
// the IPv6 side row of an IPv6 flow (its 32-B address block re-read from the capture)
__device__ __forceinline__ void res_put_v6(const ParseParams &kp, uint64_t o, const uint32_t (&s)[8], uint64_t p) {
  if (kp.flows_v6) {
    const uint64_t a = p + 16 + s[0];  // the 32-B address block: 9 aligned dwords + alignbyte
    const uint64_t al = a & ~3ull;
    const uint64_t room = kp.len - al;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(kp.buf + al), 0, (int)(room < 36 ? room : 36), 0x00020000);
    uint32_t x[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) x[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * k, 0, 0);
    const uint32_t sh = (uint32_t)(a & 3u);
    uint32_t *d6 = kp.flows_v6 + o * 8;
    st_wt16(d6, u32x4{__builtin_amdgcn_alignbyte(x[1], x[0], sh), __builtin_amdgcn_alignbyte(x[2], x[1], sh),
                      __builtin_amdgcn_alignbyte(x[3], x[2], sh), __builtin_amdgcn_alignbyte(x[4], x[3], sh)});
    st_wt16(d6 + 4, u32x4{__builtin_amdgcn_alignbyte(x[5], x[4], sh), __builtin_amdgcn_alignbyte(x[6], x[5], sh),
                          __builtin_amdgcn_alignbyte(x[7], x[6], sh), __builtin_amdgcn_alignbyte(x[8], x[7], sh)});
  }
}

// Re-read tiles [t0, c1) of the range from the exact chain position `pos` (counts pcnt / pok
// before it): walk, decode, write every Ok flow.  Returns the exit; updates the counts.
__device__ __forceinline__ uint64_t res_emit(const ParseParams &kp, ResShared &sh, uint32_t t_from, uint32_t c1, uint64_t pos,
                             uint64_t &cnt, uint64_t &ok) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int k = 0; k < kResRing - 1; ++k)
    if (t_from + k < c1) dma_tile<2>(kp, kp.org + (uint64_t)(t_from + k) * kTile, sh.data[k]);
  bool ended = false;
  uint32_t wlast = kAnyLen;
  for (uint32_t t = t_from; t < c1; ++t) {
    const uint32_t slot = (t - t_from) % kResRing;
    const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
    const uint64_t tile_hi = tile_lo + kTile < kp.stop ? tile_lo + kTile : kp.stop;
    if (t + kResRing - 1 < c1)
      dma_tile<2>(kp, tile_lo + (uint64_t)(kResRing - 1) * kTile, sh.data[(slot + kResRing - 1) % kResRing]);
    res_wait<0>(c1 - 1 - t < (uint32_t)(kResRing - 1) ? c1 - 1 - t : (uint32_t)(kResRing - 1));
    const uint32_t *w = sh.data[slot];
    if (!ended && pos >= tile_lo && pos < tile_hi) {
      uint32_t n = 0;
      const uint64_t ex = uni64(walk_tile_inl(kp, w, sh.srec, tile_lo, tile_hi, pos, n, &wlast));
      wave_sync();
      uint32_t okbase = 0;
      for (int s = 0; s < kRounds; ++s) {
        if ((uint32_t)s * 64u >= n) break;
        const uint32_t i = lane + (uint32_t)s * 64u;
        const bool valid = i < n;
        FlowWords f;
        const uint32_t rel = sh.srec[i];
        const bool okr = decode_rec<true>(kp, w, tile_lo, rel, f, valid) == NPR_FLOW_OK && valid;
        const uint64_t bal = __ballot(okr);
        if (okr && kp.flows) {
          const uint64_t fi = ok + okbase + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
          if (fi < kp.flow_cap) {
            const uint64_t o = kp.flow_cap - 1 - fi;
            const uint32_t sw[8] = {(f.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) ? f.v6off : f.d[0], f.d[1], f.d[2], f.d[3],
                                    f.d[4], f.d[5], f.d[6], 0u};
            res_put(kp, o, sw, tile_lo + rel);
          }
        }
        okbase += (uint32_t)__builtin_popcountll(bal);
      }
      cnt += n;
      ok += okbase;
      ended = ex < tile_hi;  // Err(Incomplete): the chain stops here (Q3)
      pos = ex;
    }
    wave_sync();  // done with this slot before it is refilled
  }
  return pos;
}

// The kept rounds' Ok flows to rows flow_cap - 1 - (x0 + Ok rank), x0 = the exact Ok flows before
// the wave (phase B).  Each round's Ok rows are one contiguous
// block: staged in the wave's idle ring slot in address order, then stored as contiguous 16-B chunks
// (lane i: chunks i and 64 + i), so each store instruction writes whole lines, written through (sc1)
// through a buffer resource over exactly the block (its range check drops the chunks past 2 nok).
// A write-only microbenchmark (scripts/microbench/store_pattern.hip) writes one-row-per-lane rounds
// (two stores at a 32-B stride) at 1.5-1.8 TB/s and contiguous ones at 2.4-3.3 TB/s; write-through
// measured 28.1-28.5 us per C2 launch against 30.3-30.7 us non-temporal (round 3,
// scripts/gpu_variants.sh), C3 1.443 against 1.478 ms.  Rounds past flow_cap go row by row (res_put).
template <int NS>
__device__ __forceinline__ void res_write_kept(const ParseParams &kp, uint32_t *stg_words, const uint32_t (&fl)[NS][8],
                                               uint32_t ns, uint32_t m_ok, uint32_t m_lo, uint32_t m_hi, uint64_t x0,
                                               uint64_t base) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    if ((uint32_t)q < ns) {
      const uint32_t okb = __builtin_amdgcn_readlane(m_ok, q);
      const uint64_t bal = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(m_hi, q) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane(m_lo, q);
      const uint32_t nok = (uint32_t)__builtin_popcountll(bal);
      const uint64_t f0 = x0 + okb;
      if (nok && f0 + nok <= kp.flow_cap) {
        const bool mine = (bal >> lane) & 1ull;
        const uint32_t rank = (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
        const uint64_t p = base + fl[q][7];
        const bool v6 = (fl[q][6] & (NPR_FLOW_KIND_IPV6 << 16)) != 0;
        u32x4 *stg = reinterpret_cast<u32x4 *>(stg_words);
        if (mine) {
          const uint32_t k = nok - 1u - rank;  // rank r lands at row flow_cap - 1 - (f0 + r)
          stg[stg_slot<128>(2 * k)] = u32x4{v6 ? 0u : fl[q][0], v6 ? 0u : fl[q][1], fl[q][2], fl[q][3]};
          stg[stg_slot<128>(2 * k + 1)] =
              u32x4{fl[q][4], fl[q][5], fl[q][6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8)};
        }
        wave_sync();
        u32x4 *dst = reinterpret_cast<u32x4 *>(kp.flows + (kp.flow_cap - f0 - nok) * 8);
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc((void *)dst, 0, (int)(2u * nok * 16u), 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(stg[stg_slot<128>(lane)], rr, (int)(lane * 16u), 0, kPolSc1);
        __builtin_amdgcn_raw_buffer_store_b128(stg[stg_slot<128>(lane + 64)], rr, (int)((lane + 64u) * 16u), 0, kPolSc1);
        if (mine && v6) res_put_v6(kp, kp.flow_cap - 1 - (f0 + rank), fl[q], p);
        wave_sync();  // the slot is rewritten by the next round
      } else if ((bal >> lane) & 1ull) {
        const uint64_t fi = x0 + okb + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
        if (fi < kp.flow_cap) res_put(kp, kp.flow_cap - 1 - fi, fl[q], base + fl[q][7]);
      }
    }
  }
}

struct ResWgShared {  // one workgroup's LDS: the waves' rings, then the in-LDS fold
  ResShared w[kResWg];
  uint32_t prog[kResWg];  // tiles each wave has parsed in phase A (~0: done or inactive), for fair priorities
  Seg a[kResWg];   // each wave's range aggregate A
  Seg x[kResWg];   // each wave's prefix: anchor ⊕ G(0..b-1) ⊕ A(waves before it here)
  uint32_t fail;   // a bounded wait of wave 0 timed out: every wave leaves
};

// One capture of the resident pass (the kernel comment above).  Run by every wave of the workgroup.
// Returns false when the workgroup must leave the kernel (a bounded wait timed out).
// (Round 3's k_parse_batch ran several captures through this body in one launch, staging capture
// k+1's first tiles during capture k's look-back: 1.01-1.09x on 8 captures of 16 K-1 M records,
// profiles/r04_batch_small.jsonl, under the 1.3x that would have paid for a second instantiation.)
template <bool DIAG, bool PACK>
__device__ __forceinline__ bool res_capture(const ParseParams &kp, ResWgShared &sh) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar LDS bases
  const uint32_t b = blockIdx.x, v = b * kResWg + wid;
  const uint32_t nb = (kp.nwaves + kResWg - 1) / kResWg;
  const uint32_t nw = kp.nwaves - b * kResWg < kResWg ? kp.nwaves - b * kResWg : kResWg;  // waves of this workgroup
  const bool active = wid < nw;
  Stamps st;
  if (DIAG) stamp_at(st, 0);
  uint32_t c0 = 0, c1 = 0;
  if (active) res_range(kp, v, c0, c1);
  const uint64_t base = kp.org + (uint64_t)c0 * kTile;  // kept record offsets are relative to this
  const bool spec0 = (kp.flags & kFlagSpecStart) != 0 || kp.prev != nullptr;  // chained: tile 0 speculates too
  if (lane == 0) sh.prog[wid] = active && c0 < c1 ? 0u : ~0u;
  const uint32_t scb = spec_ctx_load(kp);  // older than the ring's DMAs: landed with the first tile
#pragma unroll
  for (int k = 0; k < kResRing - 1; ++k)
    if (c0 + k < c1) dma_tile<2>(kp, base + (uint64_t)k * kTile, sh.w[wid].data[k]);
  __builtin_amdgcn_s_setprio(3);  // lowered by one per tile parsed (below)

  // ---- phase A ------------------------------------------------------------------------------
  uint32_t fl[kResSlots][8];                   // kept rounds: d[0..6] (IPv6: d[0] = address offset), record offset - base
  uint32_t m_ok = 0, m_lo = 0, m_hi = 0;       // lane k: Ok flows before kept round k, its Ok ballot
  uint32_t ns = 0;                             // kept rounds
  uint32_t fill = 64;                          // lanes used in kept round ns - 1
  uint64_t entry = kNone, pos = kNone;         // speculated entry; chain position
  bool ended = false;
  uint32_t cnt = 0, okc = 0;                   // records / Ok flows of the range (speculative chain)
  uint32_t tdef = c1;                          // first deferred tile (its flows are re-read in phase B)
  uint64_t pdef = 0;
  uint32_t cdef = 0, odef = 0;
  SpecCtx sc{};
  uint32_t wlast = kAnyLen;  // incl_len of the last record walked (walk_tile)
  uint64_t wait_ticks = 0;  // DIAG: phase A time spent waiting for tiles to land
  uint64_t walk_ticks = 0;  // DIAG: ... walking the record chain
  // ---- phase A, the one-length prefix (dense captures: C2, any capture of one record size) --------
  // The range's first tiles while every record starting in a tile has the length of the tile's
  // first record, at most 64 of them, and the capture runs on for a tile past it (so no record of
  // the tile is incomplete): one header read per lane confirms the tile's records, lane l decodes
  // record l, and the flows land in kept round k = the tile's index in the range (a compile-time
  // register block: no per-round dynamic select).  The chain walk, the round bookkeeping and the
  // loop control of the general loop below cost ~300 SALU + ~270 VALU per C2 tile beside the
  // decode (PMC); this path issues a fraction of that.  The first tile that does not
  // qualify goes to the general loop, which continues from the same state (same results).
  uint32_t t_gen = c0;       // first tile of the general loop
  bool succ_issued = false;  // the fast prefix already issued that tile's successor's DMA
  if constexpr (!PACK) {
    // 32-bit positions relative to the range base (the prefix covers at most kResSlots tiles), one
    // buffer resource over the range (bytes past the capture read 0, as dma_tile's do), the
    // header's byte order as a v_perm selector
    const uint64_t stop64 = kp.stop - base, len64 = kp.len - base;  // base <= stop <= len
    const uint32_t stop_r = stop64 < 0xffffffffull ? (uint32_t)stop64 : 0xffffffffu;
    const uint32_t len_r = len64 < 0x7fff0000ull ? (uint32_t)len64 : 0x7fff0000u;
    const __amdgpu_buffer_rsrc_t rsr =
        __builtin_amdgcn_make_buffer_rsrc((void *)(kp.buf + base), 0, (int)((len_r + 15u) & ~15u), 0x00020000);
    const uint32_t hsel = kp.big ? 0x00010203u : 0x03020100u;
    const uint32_t l16 = lane * 16u;
    uint32_t pr = 0;  // the chain position - base, once an entry is known
    bool go = active && c0 < c1;
#pragma unroll
    for (uint32_t Q = 0; Q < (uint32_t)kResSlots; ++Q) {  // (unrolled: kept round Q is a register block)
      const uint32_t t = c0 + Q;
      if (!go || t >= c1) break;
      const uint32_t slot = Q % kResRing;
      const uint32_t lo_r = Q * (uint32_t)kTile;
      const uint32_t hi_r = lo_r + (uint32_t)kTile < stop_r ? lo_r + (uint32_t)kTile : stop_r;
      if (t + 1 < c1) {  // the successor tile's DMA (dma_tile's rows, offsets into the range)
        uint32_t *dst = sh.w[wid].data[(slot + 1) % kResRing];
#pragma unroll
        for (int i = 0; i < kRows; ++i) {
          uint32_t vo;
          asm volatile("v_add_u32 %0, %1, %2" : "=v"(vo) : "n"(1024 * i + (int)kTile), "v"(l16 + lo_r));
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsr, (lds_ptr_t)(dst + i * 256), 16, vo, 0, 0, 2);
        }
        uint32_t vh;
        asm volatile("v_lshrrev_b32 %0, 2, %1\n\tv_add_u32 %0, %2, %0" : "=&v"(vh) : "v"(l16), "v"(lo_r + 2u * (uint32_t)kTile));
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsr, (lds_ptr_t)(dst + kRows * 256), 4, vh, 0, 0, 2);
      }
      const uint64_t tw0 = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
      res_wait<0>(t + 1 < c1 ? 1u : 0u);
      if (DIAG) wait_ticks += __builtin_amdgcn_s_memrealtime() - tw0;
      const uint32_t *w = sh.w[wid].data[slot];
      if (Q == 0) {
        const uint64_t tile_lo = base, tile_hi = base + hi_r;
        sc = spec_ctx(kp, scb);
        if (DIAG) stamp_at(st, 1);
        uint64_t e;
        if (t == 0 && !spec0) {
          e = kp.start;
        } else {
          const uint32_t lo = t == 0 ? (uint32_t)(kp.start - tile_lo) : 0u;
          e = tile_hi > tile_lo + lo ? speculate(sc, kp.len, w, tile_lo, lo, (uint32_t)(tile_hi - tile_lo)) : kNone;
        }
        e = uni64(e);
        if (e != kNone) {
          entry = pos = e;
          pr = (uint32_t)(e - base);
        }
      }
      const uint32_t span = hi_r - lo_r;
      // every record starting in the tile ends inside the capture (no Incomplete test needed)
      bool fast = pos != kNone && pr >= lo_r && pr < hi_r && len_r - hi_r >= (uint32_t)kTile + 16u;
      uint32_t r = 0, incl = 0, stride = 16, q = 0, n = 0;
      bool inb = false;
      if (fast) {
        r = pr - lo_r;
        incl = (uint32_t)__builtin_amdgcn_readfirstlane(__builtin_amdgcn_perm(0u, lds_le32(w, r + 8u), hsel));
        stride = incl + 16u;
        fast = incl <= (uint32_t)kTile && span - r <= 64u * stride;
      }
      if (fast) {
        q = r + lane * stride;  // < 2^24: lane < 64, stride <= 16 + kTile
        inb = q < span;
        const uint32_t h = __builtin_amdgcn_perm(0u, lds_le32(w, (inb ? q : r) + 8u), hsel);
        // every record of the tile: the same length (readfirstlane: visibly uniform control flow)
        fast = __builtin_amdgcn_readfirstlane((int)(__ballot(inb && h != incl) == 0ull)) != 0;
        n = (uint32_t)__builtin_amdgcn_readfirstlane((int)__builtin_popcountll(__ballot(inb)));
      }
      if (!fast) {  // the general loop takes this tile (its successor's DMA is in flight)
        go = false;
        t_gen = t;
        succ_issued = t + 1 < c1;
        break;
      }
      // lane l decodes record l (lanes past the tile's records read record 0: LDS broadcast)
      const uint32_t rr = inb ? q : r;
      FlowWords f;
      const uint32_t stc = decode_fast<true, true>(w, rr + 16u, incl, f, inb);
      if (__builtin_amdgcn_readfirstlane((int)(__ballot(inb && stc == 0xffu) != 0ull))) {
        // a frame only the general decode<> handles: the general loop takes the tile
        go = false;
        t_gen = t;
        succ_issued = t + 1 < c1;
        break;
      }
      const uint64_t bal = __ballot(inb && stc == NPR_FLOW_OK);
      fl[Q][0] = (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) ? f.v6off : f.d[0];
#pragma unroll
      for (int j = 1; j < 7; ++j) fl[Q][j] = f.d[j];
      fl[Q][7] = lo_r + rr;  // record offset - base
      m_ok = lane == Q ? okc : m_ok;
      m_lo = lane == Q ? (uint32_t)bal : m_lo;
      m_hi = lane == Q ? (uint32_t)(bal >> 32) : m_hi;
      // (loop-carried state made visibly wave-uniform: the general loop's hand-written hop walk
      // takes it in scalar registers)
      okc = (uint32_t)__builtin_amdgcn_readfirstlane(okc + (uint32_t)__builtin_popcountll(bal));
      cnt = (uint32_t)__builtin_amdgcn_readfirstlane(cnt + n);
      ns = Q + 1;
      fill = n;
      wlast = (uint32_t)__builtin_amdgcn_readfirstlane(incl);
      pr = (uint32_t)__builtin_amdgcn_readfirstlane(lo_r + r + n * stride);  // >= hi_r: the n-th record was the tile's last
      wave_sync();  // done with this slot before it is refilled
      if (c1 - c0 <= kStepPrioTiles) {  // (the general loop's priority steps, below)
        if (Q == 0) __builtin_amdgcn_s_setprio(2);
        else if (Q == 1) __builtin_amdgcn_s_setprio(1);
        else if (Q == 2) __builtin_amdgcn_s_setprio(0);
      } else if ((Q & 3u) == 3u) {
        if (lane == 0) sh.prog[wid] = Q + 1;
        uint32_t mn = lane < kResWg ? sh.prog[lane] : ~0u;
#pragma unroll
        for (int o = 1; o < (int)kResWg; o <<= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
        const uint32_t d = Q + 1 - __builtin_amdgcn_readfirstlane(mn);
        if (d == 0) __builtin_amdgcn_s_setprio(3);
        else if (d == 1) __builtin_amdgcn_s_setprio(2);
        else if (d == 2) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
      t_gen = t + 1;
      succ_issued = false;
    }
    if (pos != kNone) pos = uni64(base + pr);
    static_assert(kResSlots == 6, "one fast tile per kept round");
  }
  for (uint32_t t = t_gen; t < c1; ++t) {
    const uint32_t k = t - c0, slot = k % kResRing;
    const uint64_t tile_lo = base + (uint64_t)k * kTile;
    const uint64_t tile_hi = tile_lo + kTile < kp.stop ? tile_lo + kTile : kp.stop;
    if (t + kResRing - 1 < c1 && !(succ_issued && t == t_gen))
      dma_tile<2>(kp, tile_lo + (uint64_t)(kResRing - 1) * kTile, sh.w[wid].data[(slot + kResRing - 1) % kResRing]);
    const uint64_t tw0 = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    res_wait<0>(c1 - 1 - t < (uint32_t)(kResRing - 1) ? c1 - 1 - t : (uint32_t)(kResRing - 1));
    if (DIAG) wait_ticks += __builtin_amdgcn_s_memrealtime() - tw0;
    if (t == c0) {
      sc = spec_ctx(kp, scb);
      if (DIAG) stamp_at(st, 1);
    }
    const uint32_t *w = sh.w[wid].data[slot];
    if (!ended) {
      if (pos == kNone) {
        uint64_t e;
        if (t == 0 && !spec0) {
          e = kp.start;
        } else {
          const uint32_t lo = t == 0 ? (uint32_t)(kp.start - tile_lo) : 0u;
          e = tile_hi > tile_lo + lo ? speculate(sc, kp.len, w, tile_lo, lo, (uint32_t)(tile_hi - tile_lo)) : kNone;
        }
        e = uni64(e);
        if (e != kNone) entry = pos = e;
      }
      if (pos != kNone && pos < tile_hi) {
        uint32_t n = 0;
        const uint64_t tw1 = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
        const uint64_t ex = uni64(walk_tile_inl(kp, w, sh.w[wid].srec, tile_lo, tile_hi, pos, n, &wlast));
        wave_sync();
        if (DIAG) walk_ticks += __builtin_amdgcn_s_memrealtime() - tw1;
        const uint32_t rounds = (n + 63u) >> 6;
        // a tile of few records (sparse captures) shares the last kept round when it fits there
        const bool pack = PACK && ns > 0 && fill + n <= 64u && n > 0;
        if (tdef == c1 && ns + (pack ? 0u : rounds) > (uint32_t)kResSlots) {  // out of registers: defer the rest
          tdef = t;
          pdef = pos;
          cdef = cnt;
          odef = okc;
        }
        if (tdef == c1) {
          // fresh rounds: lane l of round s decodes record 64 s + l; packed (one round): lane
          // fill + i decodes record i, so its flow lands in its lane of round ns - 1 directly
          const uint32_t nr = pack ? 1u : rounds;
          const uint32_t fu = pack ? __builtin_amdgcn_readfirstlane(fill) : 0u;
          for (uint32_t s = 0; s < nr; ++s) {
            const uint32_t qu = __builtin_amdgcn_readfirstlane(pack ? ns - 1u : ns);  // uniform: one scalar branch per slot
            const uint32_t i = pack ? ((lane - fu) & 63u) : lane + s * 64u;
            const bool valid = pack ? (lane >= fu && lane < fu + n) : i < n;
            FlowWords f;
            const uint32_t rel = sh.w[wid].srec[i];
            const bool okr = decode_rec<true>(kp, w, tile_lo, rel, f, valid) == NPR_FLOW_OK && valid;
            const uint64_t bal = __ballot(okr);
            const uint32_t sw[8] = {(f.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) ? f.v6off : f.d[0], f.d[1], f.d[2], f.d[3],
                                    f.d[4], f.d[5], f.d[6], (uint32_t)(tile_lo + rel - base)};
            const bool keep = pack && !valid;  // packed: the round's earlier lanes stay
#pragma unroll
            for (int q = 0; q < kResSlots; ++q)
              if ((uint32_t)q == qu) {
#pragma unroll
                for (int j = 0; j < 8; ++j) fl[q][j] = keep ? fl[q][j] : sw[j];
              }
            m_ok = lane == qu && !pack ? okc : m_ok;
            m_lo = lane == qu ? (pack ? m_lo : 0u) | (uint32_t)bal : m_lo;
            m_hi = lane == qu ? (pack ? m_hi : 0u) | (uint32_t)(bal >> 32) : m_hi;
            if (!pack) ++ns;
            okc += (uint32_t)__builtin_popcountll(bal);
          }
          if (pack) fill = fu + n;
          else if (rounds) fill = n - 64u * (rounds - 1u);  // lanes used in the last kept round
        } else {  // deferred: status only (the Ok count), flows re-read in phase B
          for (uint32_t s = 0; s < rounds; ++s) {
            const uint32_t i = lane + s * 64u;
            const bool valid = i < n;
            FlowWords f;
            const bool okr = decode_rec<false>(kp, w, tile_lo, sh.w[wid].srec[i], f, valid) == NPR_FLOW_OK && valid;
            okc += (uint32_t)__builtin_popcountll(__ballot(okr));
          }
        }
        cnt += n;
        ended = ex < tile_hi;  // Err(Incomplete): the chain stops here (Q3)
        pos = ex;
      }
    }
    wave_sync();  // done with this slot before it is refilled
    // keep the CU's waves in step: the SIMD arbiter favours older waves, which would finish their
    // ranges long before the younger ones (C3: the four age ranks of a SIMD finished phase A at
    // 125 / 139 / 157 / 179 us), and the workgroup waits for its last.  Long ranges: each tile, a
    // wave d tiles ahead of the workgroup's slowest runs at priority 3 - min(d, 3) (C3 link
    // 258 -> 222 us); short ones (C2: 4-5 tiles) step down per tile, which costs less there
    // (33.2 vs 34.1 us).
    if (c1 - c0 <= kStepPrioTiles) {  // short ranges: step down after each of the first three tiles
      if (k == 0) __builtin_amdgcn_s_setprio(2);
      else if (k == 1) __builtin_amdgcn_s_setprio(1);
      else if (k == 2) __builtin_amdgcn_s_setprio(0);
    } else if ((k & 3u) == 3u) {  // (every 4th tile: the update costs issue slots)
      if (lane == 0) sh.prog[wid] = k + 1;
      uint32_t mn = lane < kResWg ? sh.prog[lane] : ~0u;
#pragma unroll
      for (int o = 1; o < (int)kResWg; o <<= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o));
      const uint32_t d = k + 1 - __builtin_amdgcn_readfirstlane(mn);
      if (d == 0) __builtin_amdgcn_s_setprio(3);
      else if (d == 1) __builtin_amdgcn_s_setprio(2);
      else if (d == 2) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
  }
  if (lane == 0) sh.prog[wid] = ~0u;  // done: no longer the slowest
  if (DIAG) stamp_at(st, 2);
  const uint32_t ep = kp.epoch;
  if (active && lane == 0) {  // A: in LDS for the workgroup fold (in HBM after the barrier, below)
    Seg A;
    A.entry = entry;
    A.exit = pos == kNone ? 0ull : pos;
    A.cnt = cnt;
    A.ok = okc;
    A.first = c0;
    A.last = (int64_t)c1 - 1;
    A.mism = -1;
    A.valid = true;
    sh.a[wid] = A;
  }
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (wid == 0) {
    // Wave 0 folds for the whole workgroup.  The rings are idle until the barrier below: its kept
    // flows wait there (stashed right after the publication, which does not wait for it), so the
    // windows get the registers.  16-B chunks, lane-contiguous: ds_write_b128 / ds_read_b128.
    static_assert(kResSlots * 8 * 64 * 4 <= 2 * sizeof(ResShared), "stash fits two rings");
    u32x4 *stash = reinterpret_cast<u32x4 *>(&sh.w[0].data[0][0]);
    // (1) the workgroup's waves, one per lane, from LDS: prefixes inside the workgroup + G(b)
    LaneSeg L{};
    if ((uint32_t)lane < nw) {
      const Seg &A = sh.a[lane];
      L.entry = A.entry;
      L.exit = A.exit;
      L.cnt = A.cnt;
      L.ok = A.ok;
      L.first = A.first;
      L.last = A.last;
      L.mism = -1;
      L.valid = true;
      L.present = true;
    }
    Seg e, agg;
    res_fold_lanes(kp, L, (int)nw, e, agg);
    // G(b), then the arrival.  No store drain in between: readers check the granules' tags and
    // re-read (returning atomics) until they are this launch's.  Nothing waits for the count: the
    // arrival's round trip only paces the first window read below (measured 0.3 us better than
    // reading at once, which re-reads more aggregates that are not published yet)
    if (lane == 0) put_agg(kp, kp.rgroups + b, agg);
    if (lane == 0) (void)res_arrive(kp.rcnt);
    if (DIAG) stamp_at(st, 3);
#pragma unroll
    for (int q = 0; q < kResSlots; ++q) {
      stash[(2 * q) * 64 + lane] = u32x4{fl[q][0], fl[q][1], fl[q][2], fl[q][3]};
      stash[(2 * q + 1) * 64 + lane] = u32x4{fl[q][4], fl[q][5], fl[q][6], fl[q][7]};
    }
    // (2) E(b) = anchor ⊕ G(0) ⊕ ... ⊕ G(b-1), looking back: every window read at once, then
    //     only the aggregates that are not this launch's yet re-read, until all are (a workgroup
    //     proceeds as soon as the ones below it are published, not when the whole grid is)
    bool okw = true;
    if (DIAG) stamp_at(st, 12);
    Seg E = start_seg(kp);
    uint64_t entry0 = kp.start;
    LaneSeg G[kTopWin];
#pragma unroll
    for (int w = 0; w < kTopWin; ++w) {  // descending inside a window (fold_window's order)
      const uint32_t w0 = 64u * (uint32_t)w, sz = b > w0 ? (b - w0 < 64u ? b - w0 : 64u) : 0u;
      G[w] = load_res(kp, 1, (int64_t)w0 + sz - 1 - lane, (uint32_t)lane < sz, true, false);
    }
    // every window at once: re-read (returning atomics) only the aggregates not yet this
    // launch's -- not published yet, or a line an earlier launch left in this XCD's L2
    uint32_t nap = 1;
    int tries = 0;
    for (;; ++tries) {
      bool miss = false;
#pragma unroll
      for (int w = 0; w < kTopWin; ++w) {
        const uint32_t w0 = 64u * (uint32_t)w, sz = b > w0 ? (b - w0 < 64u ? b - w0 : 64u) : 0u;
        miss = miss || __ballot((uint32_t)lane < sz && !G[w].present) != 0ull;
      }
      if (!miss) break;
      if (tries && !res_nap(kp, t0, nap)) {
        okw = false;
        break;
      }
#pragma unroll
      for (int w = 0; w < kTopWin; ++w) {
        const uint32_t w0 = 64u * (uint32_t)w, sz = b > w0 ? (b - w0 < 64u ? b - w0 : 64u) : 0u;
        const bool need = (uint32_t)lane < sz && !G[w].present;
        if (__ballot(need)) {
          const LaneSeg N = load_res(kp, 1, (int64_t)w0 + sz - 1 - lane, need, false, false);
          if (need) G[w] = N;
        }
      }
    }
#pragma unroll
    for (int w = 0; w < kTopWin; ++w) {  // the windows' tiles
      const uint32_t w0 = 64u * (uint32_t)w, sz = b > w0 ? (b - w0 < 64u ? b - w0 : 64u) : 0u;
      if ((uint32_t)lane < sz) res_tiles(kp, 1, (int64_t)w0 + sz - 1 - lane, G[w]);
    }
    if (DIAG) stamp_at(st, 13);
    if (DIAG && kp.stats && lane == 0 && tries) atomicAdd(kp.stats + kStatLbPolls, (uint32_t)tries);
    if (kp.prev) {  // a chained launch: the chain continues where the previous one left it
      const uint64_t pc = kp.prev->consumed, pr = kp.prev->n_records, pf = kp.prev->n_flows;
      okw = okw && (kp.prev_epoch == 0 || kp.prev->epoch == kp.prev_epoch);  // it completed
      entry0 = kp.prev->entry;  // the chain's first record, as the first link reported it
      E.entry = E.exit = pc;
      E.cnt = pr;
      E.ok = pf;
    } else if (kp.flags & kFlagSpecStart) {  // anchor: the entry wave 0 speculated
      entry0 = b == 0 ? sh.a[0].entry : rl64(G[0].entry, (int)(b < 64u ? b : 64u) - 1);
      E.entry = E.exit = entry0 == kNone ? kp.stop : entry0;
    }
#pragma unroll
    for (int w = 0; w < kTopWin; ++w) {
      const uint32_t w0 = 64u * (uint32_t)w;
      if (w0 >= b || !okw) break;
      E = combine(kp, E, fold_window(kp, G[w], (int)(b - w0 < 64u ? b - w0 : 64u) - 1));
    }
    if (DIAG) stamp_at(st, 14);
    // (3) each wave's prefix.  A workgroup with a wave whose chain is not the exact one (or whose
    // prefix is not settled) publishes its waves' A's, for the generic prefixes of the waves above
    // it (res_prefix: from the mis-speculated wave's exact prefix P(m) on, folding A's of m's
    // workgroup); with every chain exact nothing reads them, and no wave stores them.
    const Seg Xl = lane == 0 ? E : combine(kp, E, e);
    if ((uint32_t)lane < nw) sh.x[lane] = Xl;
    if (__ballot((uint32_t)lane < nw && (!Xl.valid || Xl.exit != sh.a[lane].entry)) && (uint32_t)lane < nw) {
      const Seg &A = sh.a[lane];
      RangeSlot *rs = kp.rslots + b * kResWg + lane;
      st_agent(&rs->a[0], gran(ep, A.exit));
      st_agent(&rs->a[1], gran(ep, A.entry == kNone ? 0ull : A.entry + 1));
      st_agent(&rs->a[2], gran(ep, A.cnt));
      st_agent(&rs->a[3], gran(ep, A.ok));
    }
    if (lane == 0) {
      sh.fail = okw ? 0u : 1u;
      if (b == nb - 1) kp.summary->entry = entry0;
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < kResSlots; ++q) {
      const u32x4 x = stash[(2 * q) * 64 + lane], y = stash[(2 * q + 1) * 64 + lane];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fl[q][j] = x[j];
        fl[q][4 + j] = y[j];
      }
    }
  }
  __syncthreads();
  if (sh.fail) return false;
  if (!active) return true;

  // ---- phase B ------------------------------------------------------------------------------
  Seg X = sh.x[wid];
  // (a wave whose prefix is settled and continues its chain exactly is nobody's P(m))
  const bool publish_p = !X.valid || X.exit != entry;
  if (!X.valid && !res_prefix(kp, v, X, t0, sh.a)) return false;
  if (DIAG) stamp_at(st, 4);
  const uint64_t range_lo = base, range_hi = tile_end(kp, (int64_t)c1 - 1);
  uint64_t xe = uni64(X.exit), xc = uni64(X.cnt), xo = uni64(X.ok);
  const bool before_end = X.exit < tile_end(kp, X.last);  // the chain ended before this range
  if (!before_end && xe < range_hi && xe >= range_lo) {
    if (entry != kNone && xe == entry) {  // the speculated chain is the exact one: flows from registers
      if (kp.flows) res_write_kept<kResSlots>(kp, sh.w[wid].data[0], fl, ns, m_ok, m_lo, m_hi, xo, base);
      if (DIAG) stamp_at(st, 5);
      if (tdef < c1) {
        uint64_t dc = xc + cdef, dok = xo + odef;
        (void)res_emit(kp, sh.w[wid], tdef, c1, pdef, dc, dok);
        if (kp.stats && lane == 0) atomicAdd(kp.stats + kStatRewalk, c1 - tdef);
      }
      xe = pos;
      xc += cnt;
      xo += okc;
    } else {  // mis-speculated: re-read the whole range from the exact position
      xe = uni64(res_emit(kp, sh.w[wid], c0, c1, xe, xc, xo));
      if (kp.stats && lane == 0) atomicAdd(kp.stats + kStatRewalk, c1 - c0);
    }
  }
  if (lane == 0) {
    if (publish_p) {
      RangeSlot *rs = kp.rslots + v;
      st_agent(&rs->p[0], gran(ep, xe));
      st_agent(&rs->p[1], gran(ep, xc));
      st_agent(&rs->p[2], gran(ep, xo));
    }
    if (v == kp.nwaves - 1) {
      uint32_t fl2 = 0;
      if (kp.flows && xo > kp.flow_cap) fl2 |= NPR_SUMMARY_FLOW_OVERFLOW;
      kp.summary->n_records = xc;
      kp.summary->n_flows = xo;
      kp.summary->consumed = xe;
      kp.summary->flags = fl2;
      kp.summary->epoch = ep;
    }
  }
  if (DIAG) {
    stamp_at(st, 6);
    st.v[8] = c1 - c0;
    st.v[9] = ns;
    st.v[10] = c1 - tdef;
    st.v[11] = (entry != kNone && xe == pos) ? 1 : 0;
    st.v[15] = wait_ticks;
    st.v[7] = walk_ticks;
    stamp_flush(kp, st, v, wid == 0 ? 0xFFFFu : 0x8FFFu);
  }
  return true;
}

// PACK: sparse tiles share kept rounds (links sized past one round per tile; the host sets it from
// the capture's density).  A separate instantiation: the merge costs dense captures registers.
template <bool DIAG, bool PACK>
__global__ __launch_bounds__(kResWg * kWave) void k_parse_resident(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) ResWgShared sh;
  (void)res_capture<DIAG, PACK>(kp, sh);
}

int resident_waves_per_cu() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void *>(&k_parse_resident<false, false>), kResWg * kWave, 0) !=
      hipSuccess)
    return 0;
  return nb * (int)kResWg;
}

template <bool DIAG>
static hipError_t launch(const ParseParams &p, hipStream_t s) {
  hipLaunchKernelGGL((k_count_tiles<DIAG>), dim3(p.ntiles), dim3(kWave), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_emit_tiles<DIAG>), dim3(p.ntiles), dim3(kWave), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_parse_extract(const ParseParams &p, hipStream_t s) {
  if (p.nwaves) {
    const uint32_t nb = (p.nwaves + kResWg - 1) / kResWg;
    const bool diag = p.stats || p.stamps;
    auto k = diag ? (p.pack ? k_parse_resident<true, true> : k_parse_resident<true, false>)
                  : (p.pack ? k_parse_resident<false, true> : k_parse_resident<false, false>);
    hipLaunchKernelGGL(k, dim3(nb), dim3(kResWg * kWave), 0, s, p);
    return hipGetLastError();
  }
  return (p.stats || p.stamps) ? launch<true>(p, s) : launch<false>(p, s);
}

// ---------------------------------------------------------------------------------------------
// per-record extract over caller-supplied records (FlowExtraction::extract_flow per PcapRecord,
// src/flow/mod.rs:20-48; flow::convert_records, src/flow/mod.rs:101-123)
//
// Each lane owns one record: its 24-B row is three dwordx2 loads, and the first kRowWin
// bytes around its payload (16-B aligned, so six dwordx4 loads issued back to back: ONE memory
// latency) land in the lane's own LDS row, where decode_fast / decode<> read them like a staged
// tile (the general decode falls back to global bytes past the window).  The per-byte global
// walk this replaces paid one dependent round trip per header field.
// ---------------------------------------------------------------------------------------------
constexpr int kRowWin = 96;                 // staged bytes: [payload & ~15, +96) holds decode_fast's 72 + misalignment
constexpr int kRowWords = kRowWin / 4 + 1;  // + 1 pad dword: odd stride, per-lane rows are bank-conflict-free
static_assert(15 + 18 * 4 <= kRowWin, "decode_fast's 18-word window fits the staged row at any misalignment");

struct RowReader {
  const uint32_t *w;  // the lane's LDS row
  uint32_t rel;       // payload start inside the row
  const uint8_t *g;   // payload start in global memory
  uint64_t gavail;    // bytes of the input buffer from the payload start
  __device__ __forceinline__ uint32_t le32(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a + 4 <= (uint64_t)kRowWin) return lds_le32(w, (uint32_t)a);
    return u8g(q) | (u8g(q + 1) << 8) | (u8g(q + 2) << 16) | (u8g(q + 3) << 24);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a < (uint64_t)kRowWin) return ((const uint8_t *)w)[a];
    return u8g(q);
  }
  __device__ __forceinline__ uint32_t u8g(uint32_t q) const { return (uint64_t)q < gavail ? g[q] : 0u; }
};

// The record's payload window [payload & ~15, +kRowWin) in registers (six dwordx4 loads, issued
// back to back); false when the record or the window does not lie inside the buffer.
struct RowWin {
  uint4 v[kRowWin / 16];
};
// loaded instead of a window that does not lie inside the buffer (always mapped)
__device__ __attribute__((aligned(16))) uint4 kZeroWin[kRowWin / 16];
__device__ __forceinline__ bool window_fits(const uint8_t *buf, uint64_t len, const npr_record &rc) {
  const uint64_t off = rc.offset + 16;
  if (off > len || len - off < rc.actual_length) return false;
  const uint64_t a16 = (uint64_t)(uintptr_t)(buf + off) & ~15ull;
  return a16 + kRowWin <= (uint64_t)(uintptr_t)buf + len;
}
__device__ __forceinline__ void window_load(const uint8_t *buf, const npr_record &rc, RowWin &W) {
  const uint4 *src = reinterpret_cast<const uint4 *>((uint64_t)(uintptr_t)(buf + rc.offset + 16) & ~15ull);
#pragma unroll
  for (int k = 0; k < kRowWin / 16; ++k) W.v[k] = src[k];
}
__device__ __forceinline__ void window_store(const RowWin &W, uint32_t *row) {
#pragma unroll
  for (int k = 0; k < kRowWin / 16; ++k) {
    row[4 * k + 0] = W.v[k].x;
    row[4 * k + 1] = W.v[k].y;
    row[4 * k + 2] = W.v[k].z;
    row[4 * k + 3] = W.v[k].w;
  }
}
// decode a record whose window is staged in `row` (fits), or from global bytes (!fits)
__device__ __forceinline__ uint32_t decode_staged(const uint8_t *buf, uint64_t len, const npr_record &rc, bool fits,
                                                  const uint32_t *row, FlowWords &f) {
  const uint64_t off = rc.offset + 16;
  if (off > len || len - off < rc.actual_length) return 0xffu;  // not a record of this buffer
  if (fits) {
    const uint32_t rel = (uint32_t)((uint64_t)(uintptr_t)(buf + off) & 15u);
    uint32_t st = decode_fast<true>(row, rel, rc.actual_length, f);
    if (st == 0xffu) {
      RowReader r{row, rel, buf + off, len - off};
      st = decode<true>(r, rc.actual_length, f);
    }
    return st;
  }
  GlobalReader r{buf + off, len - off};  // the last bytes of the buffer
  return decode<true>(r, rc.actual_length, f);
}
// One record -> status + flow words.  0xff: the record does not lie inside the buffer.
__device__ __forceinline__ uint32_t extract_one(const uint8_t *buf, uint64_t len, const npr_record &rc, uint32_t *row,
                                                FlowWords &f) {
  const bool fits = window_fits(buf, len, rc);
  if (fits) {
    RowWin W;
    window_load(buf, rc, W);
    window_store(W, row);
  }
  return decode_staged(buf, len, rc, fits, row, f);
}

__device__ __forceinline__ npr_record load_record(const npr_record *recs, uint64_t i) {
  static_assert(sizeof(npr_record) == 24, "npr_record: three dwordx2 (8-B aligned rows)");
  const uint2 *s = reinterpret_cast<const uint2 *>(recs + i);
  const uint2 a = s[0], b = s[1], c = s[2];
  npr_record r;
  r.offset = (uint64_t)a.x | ((uint64_t)a.y << 32);
  r.ts_sec = b.x;
  r.ts_usec = b.y;
  r.actual_length = c.x;
  r.original_length = c.y;
  return r;
}

// one 16-B chunk (LDS -> global) with a non-temporal store
__device__ __forceinline__ void st_nt16(uint4 *dst, const uint4 *src) {
  __builtin_nontemporal_store(*reinterpret_cast<const u32x4 *>(src), reinterpret_cast<u32x4 *>(dst));
}

__device__ __forceinline__ void flow_rows(const FlowWords &f, uint64_t recoff, bool ok, bool is6, uint4 &r0, uint4 &r1,
                                          uint4 &s0, uint4 &s1) {
  r0 = ok ? make_uint4(f.d[0], f.d[1], f.d[2], f.d[3]) : make_uint4(0, 0, 0, 0);
  r1 = ok ? make_uint4(f.d[4], f.d[5], f.d[6] | ((uint32_t)(recoff & 0xffu) << 24), (uint32_t)(recoff >> 8))
          : make_uint4(0, 0, 0, 0);
  s0 = is6 ? make_uint4(f.v6[0], f.v6[1], f.v6[2], f.v6[3]) : make_uint4(0, 0, 0, 0);
  s1 = is6 ? make_uint4(f.v6[4], f.v6[5], f.v6[6], f.v6[7]) : make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(kBlock) void k_extract_dense(const uint8_t *buf, uint64_t len,
                                                          const npr_record *recs, uint64_t n,
                                                          uint32_t *flows, uint32_t *flows_v6,
                                                          uint8_t *status) {
  __shared__ __attribute__((aligned(16))) uint32_t rows[kBlock * kRowWords];
  static_assert((2 * kBlock + 8) * 4 <= kBlock * kRowWords, "the row staging fits the window rows");
  const uint64_t b0 = (uint64_t)blockIdx.x * kBlock, i = b0 + threadIdx.x;
  const bool act = i < n;
  uint4 r0{}, r1{}, s0{}, s1{};
  bool is6 = false;
  if (act) {
    const npr_record rc = load_record(recs, i);
    FlowWords f{};
    const uint32_t st = extract_one(buf, len, rc, rows + threadIdx.x * kRowWords, f);
    const bool ok = st == NPR_FLOW_OK;
    is6 = ok && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16));
    flow_rows(f, rc.offset, ok, is6, r0, r1, s0, s1);
    if (status) status[i] = (uint8_t)st;
  }
  // IPv6 side rows of IPv6 flows only (npr.h): an IPv4 record's side row is not written, so an
  // all-IPv4 batch writes 32 B per record, not 64 (C2: 32 MB of zero side rows before round 4)
  if (is6 && flows_v6) {
    uint4 *d6 = reinterpret_cast<uint4 *>(flows_v6 + i * 8);
    d6[0] = s0;
    d6[1] = s1;
  }
  // The block's rows are contiguous: stage them in LDS (the windows are done) and store whole
  // lines, 16-B chunk c by thread c % kBlock (one 32-B row per lane at a 32-B stride writes at a
  // fraction of the rate: scripts/microbench/store_pattern.hip)
  if (!flows) return;  // (uniform)
  const uint32_t nch = 2u * (uint32_t)(n - b0 < (uint64_t)kBlock ? n - b0 : (uint64_t)kBlock);
  uint4 *stg = reinterpret_cast<uint4 *>(rows);
  __syncthreads();
  stg[stg_slot<2 * kBlock>(2 * threadIdx.x)] = r0;
  stg[stg_slot<2 * kBlock>(2 * threadIdx.x + 1)] = r1;
  __syncthreads();
  // non-temporal (streaming) stores: 23.9 -> 23.4 us per 1M C2 records.  Write-through (sc1, or
  // sc0 sc1), which phase B's row blocks use since round 3, measured the same here: 23.3-23.9 us
  // for all three policies (profiles/r03_block_store_policy_ab.json)
  uint4 *dst = reinterpret_cast<uint4 *>(flows + b0 * 8);
  if (threadIdx.x < nch) st_nt16(dst + threadIdx.x, stg + stg_slot<2 * kBlock>(threadIdx.x));
  if (threadIdx.x + kBlock < nch) st_nt16(dst + threadIdx.x + kBlock, stg + stg_slot<2 * kBlock>(threadIdx.x + kBlock));
}

hipError_t launch_extract_dense(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n,
                                uint32_t *flows, uint32_t *flows_v6, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_extract_dense, dim3((uint32_t)blocks), dim3(kBlock), 0, s, buf, len, recs, n,
                     flows, flows_v6, status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// row f3: VXLAN inner flows over caller-supplied records.  One lane per record, bytes read
// through GlobalReader (an off-path decoder: the general decode<> twice, outer then inner).
//   outer: FlowExtraction::extract_flow of the record; Ok and UDP (to dst_port unless 0);
//   Vxlan::parse(udp payload, endianness) (src/layer4/vxlan.rs:31-48): flags, group policy id,
//     raw network identifier (u16, u16, u32), payload = rest -> Incomplete below 8 bytes;
//   <Vxlan as FlowExtraction>::extract_flow (src/flow/layer4/vxlan.rs:32-50): the inner
//     Ethernet frame's flow (its remainder is always empty).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_vxlan_flows(const uint8_t *buf, uint64_t len, const npr_record *recs,
                                                        uint64_t n, uint32_t dst_port, uint32_t big,
                                                        uint32_t *flows, uint32_t *flows_v6, uint8_t *status,
                                                        uint32_t *vni_out) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const npr_record rc = load_record(recs, i);
  const uint64_t off = rc.offset + 16;
  uint32_t st = 0xffu, vni = 0;  // 0xff: the record does not lie inside the buffer
  FlowWords f{};
  if (off <= len && len - off >= rc.actual_length) {
    const GlobalReader r{buf + off, len - off};
    st = decode<true>(r, rc.actual_length, f);
    if (st == NPR_FLOW_OK) {
      if (!(f.d[6] & (NPR_FLOW_KIND_UDP << 16))) {
        st = NPR_VXLAN_NOT_UDP;
      } else if (dst_port && (f.d[2] >> 16) != dst_port) {
        st = NPR_VXLAN_PORT;
      } else {
        // an Ok UDP flow: payload = [l4 + 8, l4 + L) with L the UDP length (== the IP payload)
        const uint32_t L = be16_of(r.le32(f.l4off + 4u));
        const uint32_t po = f.l4off + 8u, pl = L - 8u;
        if (pl < 8u) {
          st = NPR_VXLAN_INCOMPLETE;
        } else {
          const uint32_t w = r.le32(po + 4u);
          const uint32_t raw = big ? __builtin_bswap32(w) : w;  // u32!(endianness) (:40)
          vni = raw >> 8;                                        // network_identifier (:45)
          const GlobalReader ri{buf + off + po + 8u, len - off - po - 8u};
          FlowWords g{};
          const uint32_t s2 = decode<true>(ri, pl - 8u, g);
          if (s2 == NPR_FLOW_OK) {
            f = g;
            st = NPR_FLOW_OK;
          } else {
            st = NPR_VXLAN_INNER + s2;
          }
        }
      }
    }
  }
  const bool ok = st == NPR_FLOW_OK;
  const bool is6 = ok && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16));
  uint4 r0, r1, s0, s1;
  flow_rows(f, rc.offset, ok, is6, r0, r1, s0, s1);
  if (status) status[i] = (uint8_t)st;
  if (vni_out) vni_out[i] = vni;
  if (flows) {
    uint4 *dst = reinterpret_cast<uint4 *>(flows + i * 8);
    dst[0] = r0;
    dst[1] = r1;
  }
  if (flows_v6) {
    uint4 *d6 = reinterpret_cast<uint4 *>(flows_v6 + i * 8);
    d6[0] = s0;
    d6[1] = s1;
  }
}

// ---------------------------------------------------------------------------------------------
// The payload of each record's extract_flow error (npr_dev_flow_details): the general decoder in
// its DETAIL form, one lane per record, bytes through GlobalReader (off the hot path: the parse
// kernels carry none of this).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_flow_detail(const uint8_t *buf, uint64_t len, const npr_record *recs,
                                                        uint64_t n, uint8_t *status, uint64_t *detail) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const npr_record rc = load_record(recs, i);
  const uint64_t off = rc.offset + 16;
  uint32_t st = 0xffu;  // the record does not lie inside the buffer
  // (the payload goes straight to detail[i]: a private stand-in for a null `detail` put the pointer
  // in the flat address space and gave the kernel a scratch segment)
  if (off <= len && len - off >= rc.actual_length) {
    const GlobalReader r{buf + off, len - off};
    FlowWords f;
    st = detail ? decode<false, GlobalReader, true>(r, rc.actual_length, f, detail + i)
                : decode<false, GlobalReader, false>(r, rc.actual_length, f);
  } else if (detail) {
    detail[i] = 0;
  }
  if (status) status[i] = (uint8_t)st;
}

hipError_t launch_flow_detail(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n, uint8_t *status,
                              uint64_t *detail, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_flow_detail, dim3((uint32_t)blocks), dim3(kBlock), 0, s, buf, len, recs, n, status, detail);
  return hipGetLastError();
}

hipError_t launch_vxlan_flows(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n, uint32_t dst_port,
                              bool big, uint32_t *flows, uint32_t *flows_v6, uint8_t *status, uint32_t *vni,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_vxlan_flows, dim3((uint32_t)blocks), dim3(kBlock), 0, s, buf, len, recs, n, dst_port,
                     big ? 1u : 0u, flows, flows_v6, status, vni);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// convert_records in ONE pass.  One 1024-thread workgroup per CU: workgroup j takes the j-th block
// of rpb records FROM THE END of the list (launch_convert_records), so its Ok flows' reverse-order rows
// start at the number of Ok flows in the blocks after it: exactly the lower-numbered (earlier
// dispatched) workgroups.  A CU's 16 waves share its memory pipeline and finish their block
// together, so the counts all come in at about the same time.  (With four 256-thread workgroups
// per CU, the SIMD arbiter's age order made the youngest workgroup of each CU take 1.6x the
// oldest's time to decode, and every prefix above it waited for it: profiles/r05_convert_stamps.txt.)
// Each workgroup publishes its count A(j) (an epoch-tagged granule).  Waves 0..3 each read one
// window of 64 counts at once: the blocks below j in its own group of 64 and in the three groups
// below that.  Wave 0 adds the sums S(g) of the groups further down; each S(g) is published by the
// group's top member from its own group's window, never from another look-back.  Up to 256
// workgroups (1M records) that is ONE round trip, and no workgroup waits along a chain.
// The flows stay in registers (kCvtPer records per lane) until the start row is known.  The
// workgroup of the list's first block writes the total (~0 when a bounded wait timed out).
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kCvtBlock = 1024;  // threads per workgroup; its LDS (> 80 KB) keeps it alone on its CU
constexpr uint32_t kCvtWaves = kCvtBlock / kWave;
constexpr uint32_t kCvtGroup = 64;    // workgroups per group sum
constexpr uint32_t kCvtNear = 4;      // groups whose counts are read directly (waves 0..3)

__device__ __forceinline__ uint64_t cvt_wait_sum(const uint64_t *w, int64_t cnt, uint32_t epoch, uint64_t t0,
                                                 uint64_t timeout, bool &ok) {
  // sum of cnt (<= 64) tagged words w[0..cnt), waiting (bounded) until every one is this launch's
  const uint32_t lane = threadIdx.x & 63u;
  const bool inr = (int64_t)lane < cnt;
  uint64_t v = inr ? __hip_atomic_load(w + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ((uint64_t)epoch << 48);
  while (__ballot((v >> 48) != epoch)) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
      ok = false;
      return 0;
    }
    __builtin_amdgcn_s_sleep(8);
    if ((v >> 48) != epoch) v = __hip_atomic_load(w + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  uint64_t x = v & kMask48;
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

template <int kCvtPer, int kRows>
__global__ __launch_bounds__(kCvtBlock) void k_convert_records(const uint8_t *buf, uint64_t len,
                                                               const npr_record *recs, uint64_t n, uint32_t *out,
                                                               uint32_t *out_v6, uint64_t cap, uint64_t *look,
                                                               uint32_t epoch, uint64_t *total,
                                                               uint64_t timeout, uint32_t rpb) {
  __shared__ uint32_t rows[kRows][kCvtBlock * kRowWords];
  __shared__ uint32_t wc[kCvtPer][kCvtWaves];
  __shared__ uint64_t part[kCvtNear];
  __shared__ uint64_t excl_sh;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t j = blockIdx.x, nb = gridDim.x;
  const int64_t lo = (int64_t)n - (int64_t)(j + 1) * rpb;  // this block: records [lo, lo + rpb) clipped at 0
  uint32_t kd[kCvtPer][7];   // flow words d[0..6] (IPv6: d[0] = the address block's payload offset)
  uint64_t koff[kCvtPer];
  uint32_t okm = 0;
  // every record row in flight together; then the payload windows, one staged LDS row per lane
  npr_record rc[kCvtPer];
#pragma unroll
  for (int r = 0; r < kCvtPer; ++r) {
    const uint32_t k = (uint32_t)r * kCvtBlock + threadIdx.x;  // the lane's record of round r in the block
    const int64_t i = lo + (int64_t)k;
    rc[r] = i >= 0 && k < rpb ? load_record(recs, (uint64_t)i) : npr_record{len, 0, 0, 0, 0};  // (past the buffer: no flow)
  }
  // the payload windows: record r + 1's is loaded into registers while record r (staged in the
  // lane's LDS row) decodes, so one window's latency is in flight behind each decode.  The loads are
  // unconditional (a record whose window does not lie inside the buffer loads kZeroWin, unused) so
  // that the compiler counts them and waits for the older one only.
  static_assert(kRows == 1, "one staged row per lane (the next window waits in registers)");
  typedef const __attribute__((address_space(1))) u32x4 *gwin_t;  // global loads (not flat: counted by vmcnt only)
  auto win_load = [&](const npr_record &c, bool f, RowWin &W) {
    const uint64_t a = f ? ((uint64_t)(uintptr_t)(buf + c.offset + 16) & ~15ull) : (uint64_t)(uintptr_t)kZeroWin;
    const gwin_t src = (gwin_t)a;
#pragma unroll
    for (int k = 0; k < kRowWin / 16; ++k) {
      const u32x4 v = src[k];
      W.v[k] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  bool fnext = window_fits(buf, len, rc[0]);
  RowWin Wn;
  win_load(rc[0], fnext, Wn);
#pragma unroll
  for (int r = 0; r < kCvtPer; ++r) {
    const bool f = fnext;
    const RowWin W = Wn;
    if (r + 1 < kCvtPer) {
      fnext = window_fits(buf, len, rc[r + 1]);
      win_load(rc[r + 1], fnext, Wn);
    }
    if (f) window_store(W, rows[0] + threadIdx.x * kRowWords);
    FlowWords fw{};
    const uint32_t st = decode_staged(buf, len, rc[r], f, rows[0] + threadIdx.x * kRowWords, fw);
    koff[r] = rc[r].offset;
    const bool ok = st == NPR_FLOW_OK;
    okm |= ok ? 1u << r : 0u;
#pragma unroll
    for (int k = 0; k < 7; ++k) kd[r][k] = fw.d[k];
    if (fw.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) kd[r][0] = fw.v6off;
    const uint64_t bal = __ballot(ok);
    if (lane == 0) wc[r][wave] = (uint32_t)__builtin_popcountll(bal);
  }
  __syncthreads();
  uint32_t cnt = 0;
#pragma unroll
  for (int r = 0; r < kCvtPer; ++r)
#pragma unroll
    for (uint32_t w = 0; w < kCvtWaves; ++w) cnt += wc[r][w];
  const uint64_t tag = (uint64_t)epoch << 48;
  uint64_t *A = look, *S = look + nb;
  uint64_t *abortw = look + nb + (nb + kCvtGroup - 1) / kCvtGroup;
  if (wave < kCvtNear) {
    // start row = sum S(groups below gl - 3) + every count of groups gl - 3 .. gl below j
    const uint64_t gl = j / kCvtGroup;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    uint64_t sum = 0;
    if (wave == 0 && lane == 0) __hip_atomic_store(A + j, tag | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (wave <= gl) {  // (uniform) group gl - wave exists
      const uint64_t g = gl - wave, g0 = g * kCvtGroup;
      const bool a_in = g0 + lane < j;
      uint64_t av = a_in ? __hip_atomic_load(A + g0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag;
      for (;;) {
        const bool a_miss = a_in && (av >> 48) != epoch;
        if (!__ballot(a_miss)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(8);
        if (a_miss) av = __hip_atomic_load(A + g0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      uint64_t y = a_in ? av & kMask48 : 0ull;
      for (int o = 32; o > 0; o >>= 1) y += __shfl_xor(y, o);
      sum = y;
      // the group's top member publishes S(g) as soon as its own group's counts are in
      if (ok && wave == 0 && j == g0 + kCvtGroup - 1 && lane == 0)
        __hip_atomic_store(S + g, tag | (y + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (wave == 0 && gl >= kCvtNear) {  // groups 0 .. gl - 4 through their sums (lists > 1M records)
        const uint64_t nfar = gl - kCvtNear + 1;
        for (uint64_t k = 0; k < nfar && ok; k += 64)
          sum += cvt_wait_sum(S + k, (int64_t)(nfar - k < 64 ? nfar - k : 64), epoch, t0, timeout, ok);
      }
    }
    if (lane == 0) part[wave] = ok ? sum : ~0ull;
  }
  __syncthreads();
  // a workgroup whose wait timed out writes no rows: it raises the launch's abort granule, and the
  // block holding record 0 (which depends, through the group sums, on every count any other block
  // waits for, so it finishes its own wait after any such timeout) reports ~0 when it is raised
  if (threadIdx.x == 0) {
    bool ok = true;
    uint64_t acc = 0;
#pragma unroll
    for (uint32_t w = 0; w < kCvtNear; ++w) {
      ok = ok && part[w] != ~0ull;
      acc += part[w];
    }
    if (!ok) __hip_atomic_store(abortw, tag | 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    excl_sh = ok ? acc : ~0ull;
    if (j == nb - 1) {  // the block holding record 0
      const bool aborted =
          ok && (__hip_atomic_fetch_add(abortw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 48) == epoch;
      *total = ok && !aborted ? acc + cnt : ~0ull;
    }
  }
  __syncthreads();
  const uint64_t excl = excl_sh;
  if (excl == ~0ull) return;
  // rows: excl + the Ok flows of this block at higher record indices (later r, higher wave, higher
  // lane).  Each round's rows are one contiguous block: staged in LDS, stored as whole lines (one
  // 32-B row per lane at a 32-B stride writes at a fraction of the rate: store_pattern.hip)
  __shared__ __attribute__((aligned(16))) uint4 cstg[kCvtBlock * 2 + 8];  // stg_slot<2 kCvtBlock> layout
  uint64_t after = excl;
#pragma unroll
  for (int r = kCvtPer - 1; r >= 0; --r) {
    const bool ok = (okm >> r) & 1u;
    const uint64_t bal = __ballot(ok);
    uint32_t above = 0, rc = 0;
#pragma unroll
    for (uint32_t w = 0; w < kCvtWaves; ++w) {
      above += w > wave ? wc[r][w] : 0u;
      rc += wc[r][w];
    }
    const uint32_t lr = above + (uint32_t)__builtin_popcountll(bal & ~((2ull << lane) - 1ull));
    __syncthreads();  // the previous round's chunks are read
    if (ok) {
      const bool is6 = (kd[r][6] & (NPR_FLOW_KIND_IPV6 << 16)) != 0;
      cstg[stg_slot<2 * kCvtBlock>(2 * lr)] = make_uint4(is6 ? 0u : kd[r][0], kd[r][1], kd[r][2], kd[r][3]);
      cstg[stg_slot<2 * kCvtBlock>(2 * lr + 1)] = make_uint4(kd[r][4], kd[r][5], kd[r][6] | ((uint32_t)(koff[r] & 0xffu) << 24), (uint32_t)(koff[r] >> 8));
    }
    __syncthreads();
    uint4 *blk = reinterpret_cast<uint4 *>(out + after * 8);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t c = threadIdx.x + (uint32_t)h * kCvtBlock;
      if (c < 2u * rc && after + c / 2u < cap) st_nt16(blk + c, cstg + stg_slot<2 * kCvtBlock>(c));
    }
    if (ok) {
      const uint64_t rw = after + lr;
      if (rw < cap) {
        const bool is6 = (kd[r][6] & (NPR_FLOW_KIND_IPV6 << 16)) != 0;
        if (out_v6 && is6) {  // side rows of IPv6 flows only (as the resident pass: npr.h)
          uint32_t a[8];
          const uint64_t po = koff[r] + 16;  // the 32 address bytes, re-read (the payload lies inside the buffer)
          GlobalReader g{buf + po, len - po};
#pragma unroll
          for (int k = 0; k < 8; ++k) a[k] = g.le32(kd[r][0] + 4u * k);
          uint4 *d6 = reinterpret_cast<uint4 *>(out_v6 + rw * 8);
          d6[0] = make_uint4(a[0], a[1], a[2], a[3]);
          d6[1] = make_uint4(a[4], a[5], a[6], a[7]);
        }
      }
    }
    after += rc;
  }
}

// The list is dealt to one workgroup per CU in blocks of rpb = ceil(n / CUs) records, rounded up to
// 256 (at least one per lane, at most kCvtMaxPer per lane: longer lists take several generations
// of workgroups), so every CU gets the same share; a lane takes ceil(rpb / 1024) records, one staged
// window at a time, the next one prefetched into registers.  The rounding keeps a block's row runs
// on 8-KB boundaries when every record is Ok: 1M records in blocks of 3907 (256 workgroups, row runs
// splitting lines at every block edge) took 32.1 us, in blocks of 4096 (245 workgroups) 30.6 us
// (profiles/r05_convert_rework.txt).
constexpr int kCvtRows = 1, kCvtMaxPer = 4;
struct CvtShape {
  uint32_t rpb;  // records per block
  int per;       // records per lane (1 .. kCvtMaxPer)
  uint64_t nb;   // blocks
};
static CvtShape convert_shape(uint64_t n, int cus) {
  const uint64_t c = cus > 0 ? (uint64_t)cus : 256u;
  uint64_t rpb = (n + c - 1) / c;
  rpb = (rpb + 255) / 256 * 256;
  rpb = rpb < kCvtBlock ? kCvtBlock : rpb > (uint64_t)kCvtMaxPer * kCvtBlock ? (uint64_t)kCvtMaxPer * kCvtBlock : rpb;
  return {(uint32_t)rpb, (int)((rpb + kCvtBlock - 1) / kCvtBlock), n ? (n + rpb - 1) / rpb : 0};
}
uint64_t convert_look_words(uint64_t n, int cus) {  // counts, group sums, the abort granule
  const uint64_t nb = convert_shape(n, cus).nb;
  return nb + (nb + kCvtGroup - 1) / kCvtGroup + 1;
}

hipError_t launch_convert_records(const uint8_t *buf, uint64_t len, const npr_record *recs, uint64_t n,
                                  uint32_t *out, uint32_t *out_v6, uint64_t cap, uint64_t *look, uint32_t epoch,
                                  uint64_t *total, uint64_t timeout_ticks, int cus, hipStream_t s) {
  const CvtShape sh = convert_shape(n, cus);
  if (sh.nb == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), s);
  if (sh.nb > 0x7fffffffull) return hipErrorInvalidValue;
  auto k = sh.per == 1 ? k_convert_records<1, kCvtRows>
           : sh.per == 2 ? k_convert_records<2, kCvtRows>
           : sh.per == 3 ? k_convert_records<3, kCvtRows>
                         : k_convert_records<4, kCvtRows>;
  hipLaunchKernelGGL(k, dim3((uint32_t)sh.nb), dim3(kCvtBlock), 0, s, buf, len, recs, n, out, out_v6, cap,
                     look, epoch, total, timeout_ticks, sh.rpb);
  return hipGetLastError();
}


}  // namespace npr
