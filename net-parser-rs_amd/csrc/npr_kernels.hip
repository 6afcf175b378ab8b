// npr_kernels.hip — CDNA4 (gfx950) kernels for the pcap record chain + flow extraction.
//
// Replaces, on the device, the nom parse paths of protectwise/net-parser-rs 0.3.0:
//   PcapRecords::parse loop           src/record.rs:21-54     -> walk_tile() + decoupled look-back
//   PcapRecord::parse                 src/record.rs:102-121   -> hdr() / walk_tile()
//   FlowExtraction::extract_flow      src/flow/mod.rs:20-48   -> decode<>()
//     Ethernet::parse + vlan loop     src/layer2/ethernet.rs:143-216
//     IPv4::parse / parse_ipv4        src/layer3/ipv4.rs:76-160
//     IPv6::parse / parse_next_header src/layer3/ipv6.rs:29-99
//     Arp::parse                      src/layer3/arp.rs:54-76
//     Tcp::parse / Udp::parse         src/layer4/tcp.rs:59-101, src/layer4/udp.rs:33-50
//     per-layer flow dispatch         src/flow/layer2/ethernet.rs:39-133, src/flow/layer3/*.rs
//   flow::convert_records             src/flow/mod.rs:101-123 -> reverse-order compaction
//
// Design: one 256-thread workgroup per 16 KiB tile of the record stream.
//   1. stage the tile (+256 B halo) into LDS with 16-B buffer loads (OOB -> 0);
//   2. tile 0 starts at the exact first record; every other tile SPECULATES its first record
//      start from header plausibility (a 3-header chain check, lane-parallel);
//   3. wave 0 walks the record chain through the tile, 64 records per step when the lengths
//      repeat (a ballot confirms the stride), one per step otherwise;
//   4. every record is decoded (status only) to count Ok flows;
//   5. the tile publishes its speculative aggregate {entry, exit, count, ok} and then looks
//      back (64 predecessor tiles per poll) for an exact prefix.  Aggregates are combined with
//      a chain-consistency monoid: a predecessor's exit must equal the successor's speculated
//      entry.  Any mismatch is resolved by waiting for the exact prefix of the mismatching
//      tile, which re-walks itself from the true entry — so results equal the serial chain;
//   6. with the exact prefix the tile writes the dense record table / status and its Ok flows
//      at their reverse-order (convert_records) positions.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "npr_internal.hpp"

namespace npr {

constexpr uint64_t kNone = ~0ull;
constexpr uint64_t kMask48 = (1ull << 48) - 1;
constexpr uint32_t kTsWindow = 1u << 20;  // speculation: |ts_sec delta| between neighbours
constexpr uint32_t kInclMax = 1u << 18;   // speculation: plausible incl_len bound

// ---------------------------------------------------------------------------------------------
// byte access
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t be16_of(uint32_t w) { return ((w & 0xffu) << 8) | ((w >> 8) & 0xffu); }

// 4 bytes at LDS byte address a (any alignment) as a little-endian u32: two aligned dword reads
// (merged into ds_read2_b32) + v_alignbyte.
__device__ __forceinline__ uint32_t lds_le32(const uint32_t *w, uint32_t a) {
  const uint32_t i = a >> 2;
  return __builtin_amdgcn_alignbyte(w[i + 1], w[i], a & 3u);
}

// Record-header field k (0 ts_sec, 1 ts_usec, 2 incl_len, 3 orig_len) at LDS offset rel, in the
// capture's endianness (u32!(endianness), src/record.rs:107-110).
__device__ __forceinline__ uint32_t hdr(const uint32_t *w, uint32_t rel, int k, bool big) {
  const uint32_t v = lds_le32(w, rel + 4u * (uint32_t)k);
  return big ? __builtin_bswap32(v) : v;
}

// Payload reader over the LDS-staged tile with a bounds-checked global fallback for the rare
// bytes past the halo.  Offsets q are payload-relative.
struct TileReader {
  const uint32_t *w;
  const uint8_t *b;
  uint32_t rel;       // payload start relative to LDS byte 0
  const uint8_t *g;   // payload start in global memory
  uint64_t gavail;    // bytes of the input buffer from the payload start
  __device__ __forceinline__ uint32_t le32(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a + 4 <= (uint64_t)kStage) return lds_le32(w, (uint32_t)a);
    return slow32(q);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a < (uint64_t)kStage) return b[a];
    return (uint64_t)q < gavail ? g[q] : 0u;
  }
  __device__ __noinline__ uint32_t slow32(uint32_t q) const {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      const uint64_t k = (uint64_t)q + i;
      v |= (k < gavail ? (uint32_t)g[k] : 0u) << (8 * i);
    }
    return v;
  }
};

// Payload reader straight from global memory (dense extract over caller-supplied records).
struct GlobalReader {
  const uint8_t *g;
  uint64_t gavail;
  __device__ __forceinline__ uint32_t u8(uint32_t q) const { return (uint64_t)q < gavail ? g[q] : 0u; }
  __device__ __forceinline__ uint32_t le32(uint32_t q) const {
    return u8(q) | (u8(q + 1) << 8) | (u8(q + 2) << 16) | (u8(q + 3) << 24);
  }
};

// ---------------------------------------------------------------------------------------------
// per-record decode: FlowExtraction::extract_flow (src/flow/mod.rs:23-41) as one straight-line
// function.  Returns an npr_flow_status; with FIELDS it also fills the 32-B npr_flow words
// (d[0..6]; the record offset goes in by the caller) and the IPv6 addresses.
// Length checks are ordered exactly like the reference's do_parse! steps so the FIRST failing
// step decides between Incomplete / Failure / Custom.
// ---------------------------------------------------------------------------------------------
struct FlowWords {
  uint32_t d[7];
  uint32_t v6[8];
};

// InternetProtocolId::new (src/layer3/mod.rs:54-72)
__device__ __forceinline__ bool proto_known(uint32_t v) {
  return v == 0 || v == 1 || v == 6 || v == 17 || v == 43 || v == 44 || v == 50 || v == 51 ||
         v == 59 || v == 60;
}
// InternetProtocolId::has_next_option (src/layer3/mod.rs:74-84)
__device__ __forceinline__ bool proto_has_next(uint32_t v) {
  return v == 0 || v == 43 || v == 44 || v == 50 || v == 51 || v == 60;
}

template <bool FIELDS, class R>
__device__ __forceinline__ uint32_t decode(const R &r, uint32_t n, FlowWords &f) {
  // ---- Ethernet::parse (src/layer2/ethernet.rs:204-216): two mac_address (take!(6))
  if (n < 12) return NPR_FLOW_ETH_INCOMPLETE;
  uint32_t m0 = 0, m1 = 0, m2 = 0;
  if (FIELDS) {
    m0 = r.le32(0);  // dst[0..3]
    m1 = r.le32(4);  // dst[4..5] src[0..1]
    m2 = r.le32(8);  // src[2..5]
  }
  // parse_vlan_tag recursion (:163-202): map_opt!(be_u16, EthernetTypeId::new), 802.1Q/ad tags
  uint32_t pos = 12, vlan = 0, etype;
  bool tagged = false;
  for (;;) {
    if (n - pos < 2) return NPR_FLOW_ETH_INCOMPLETE;
    const uint32_t w = r.le32(pos);
    const uint32_t t = be16_of(w);
    if (t != 0x8100u && t != 0x88a8u) {
      // EthernetTypeId::new (:57-73): LLDP / IPv4 / IPv6 / ARP / <=1500 (length), else None
      if (!(t == 0x88ccu || t == 0x0800u || t == 0x86ddu || t == 0x0806u || t <= 1500u))
        return NPR_FLOW_ETH_FAILURE;
      etype = t;
      pos += 2;
      break;
    }
    if (n - pos - 2 < 2) return NPR_FLOW_ETH_INCOMPLETE;  // TCI: be_u16 (:176)
    if (!tagged) vlan = be16_of(w >> 16) & 0x0FFFu;         // vlans_to_vlan: first tag (:134-137)
    tagged = true;
    pos += 4;
  }
  // ---- layer-3 dispatch (src/flow/layer2/ethernet.rs:55-131); payload = rest
  const uint32_t l3 = pos, n3 = n - pos;
  uint32_t l4, n4, proto;
  bool v6;
  if (etype == 0x0800u) {
    // IPv4::parse (src/layer3/ipv4.rs:148-160) -> parse_ipv4 (:76-146)
    if (n3 < 1) return NPR_FLOW_L2_IPV4_INCOMPLETE;
    const uint32_t w0 = r.le32(l3);
    const uint32_t b0 = w0 & 0xffu;
    if ((b0 >> 4) != 4u) return NPR_FLOW_L2_IPV4_CUSTOM;
    const uint32_t hw = b0 & 0x0Fu, hl = hw * 4u, add = hw > 5u ? (hw - 5u) * 4u : 0u;
    if (n3 < 4) return NPR_FLOW_L2_IPV4_INCOMPLETE;          // tos, length
    const uint32_t length = (be16_of(w0 >> 16) - hl) & 0xffffu;  // u16 wrapping (:100)
    const uint64_t expected = (uint64_t)hl + add + length;        // (:107)
    if (n3 < 10) return NPR_FLOW_L2_IPV4_INCOMPLETE;         // id, flags, ttl, protocol
    proto = (r.le32(l3 + 8) >> 8) & 0xffu;
    if (!proto_known(proto)) return NPR_FLOW_L2_IPV4_FAILURE; // map_opt! (:119)
    if (n3 < 20) return NPR_FLOW_L2_IPV4_INCOMPLETE;         // checksum, src, dst
    if (n3 - 20u < length) return NPR_FLOW_L2_IPV4_INCOMPLETE;  // payload: take!(length)
    uint64_t p4 = 20ull + length;
    if (add) {                                                // options (:124)
      if ((uint64_t)n3 - p4 < add) return NPR_FLOW_L2_IPV4_INCOMPLETE;
      p4 += add;
    }
    if ((uint64_t)n3 > expected) {                            // padding (:125-129)
      const uint64_t pad = (uint64_t)n3 - expected;
      if ((uint64_t)n3 - p4 < pad) return NPR_FLOW_L2_IPV4_INCOMPLETE;
      p4 += pad;
    }
    if (p4 != n3) return NPR_FLOW_L2_IPV4_REMAINDER;         // rem.is_empty() (:67-76)
    if (FIELDS) {
      f.d[0] = r.le32(l3 + 12);
      f.d[1] = r.le32(l3 + 16);
    }
    l4 = l3 + 20u;  // the L4 parse starts right after the fixed header (quirk Q7)
    n4 = length;
    v6 = false;
  } else if (etype == 0x86ddu) {
    // IPv6::parse (src/layer3/ipv6.rs:87-99) -> parse_ipv6 (:58-71) -> parse_next_header (:29-56)
    if (n3 < 1) return NPR_FLOW_L2_IPV6_INCOMPLETE;
    if ((r.u8(l3) >> 4) != 6u) return NPR_FLOW_L2_IPV6_CUSTOM;
    if (n3 < 7) return NPR_FLOW_L2_IPV6_INCOMPLETE;          // take!(3), be_u16, be_u8
    const uint32_t w1 = r.le32(l3 + 4);
    const uint32_t plen = be16_of(w1);
    uint32_t nh = (w1 >> 16) & 0xffu;
    if (!proto_known(nh)) return NPR_FLOW_L2_IPV6_FAILURE;
    uint32_t p = 7;
    while (proto_has_next(nh)) {                              // one byte per extension (quirk Q11)
      if (n3 - p < 1) return NPR_FLOW_L2_IPV6_INCOMPLETE;
      nh = r.u8(l3 + p);
      if (!proto_known(nh)) return NPR_FLOW_L2_IPV6_FAILURE;
      ++p;
    }
    if (n3 - p < 33u) return NPR_FLOW_L2_IPV6_INCOMPLETE;    // hop limit, src, dst
    const uint32_t sa = l3 + p + 1u;
    p += 33u;
    if (n3 - p < plen) return NPR_FLOW_L2_IPV6_INCOMPLETE;   // payload: take!(p)
    if (n3 - p != plen) return NPR_FLOW_L2_IPV6_REMAINDER;
    if (FIELDS) {
#pragma unroll
      for (int k = 0; k < 8; ++k) f.v6[k] = r.le32(sa + 4u * (uint32_t)k);
      f.d[0] = 0;
      f.d[1] = 0;
    }
    l4 = l3 + p;
    n4 = plen;
    proto = nh;
    v6 = true;
  } else if (etype == 0x0806u) {
    // Arp::parse: 28 fixed bytes (src/layer3/arp.rs:54-76); the flow is always Err
    if (n3 < 28) return NPR_FLOW_L2_ARP_INCOMPLETE;
    if (n3 != 28) return NPR_FLOW_L2_ARP_REMAINDER;
    return NPR_FLOW_L3_ARP;
  } else {
    return NPR_FLOW_L2_ETHERTYPE;  // LLDP / PayloadLength (:125-130)
  }
  // ---- layer-4 dispatch (src/flow/layer3/ipv4.rs:49-101, ipv6.rs:49-100)
  bool udp;
  if (proto == 6u) {
    // Tcp::parse (src/layer4/tcp.rs:59-101)
    if (n4 < 14) return v6 ? NPR_FLOW_L3_IPV6_TCP_INCOMPLETE : NPR_FLOW_L3_IPV4_TCP_INCOMPLETE;
    const uint32_t thl = (be16_of(r.le32(l4 + 12)) >> 12) * 4u;  // extract_length (:54-57)
    if (thl < 20u || thl > 60u) return v6 ? NPR_FLOW_L3_IPV6_TCP_FAILURE : NPR_FLOW_L3_IPV4_TCP_FAILURE;
    if (n4 < thl) return v6 ? NPR_FLOW_L3_IPV6_TCP_INCOMPLETE : NPR_FLOW_L3_IPV4_TCP_INCOMPLETE;
    udp = false;  // payload: rest -> never a remainder
  } else if (proto == 17u) {
    // Udp::parse (src/layer4/udp.rs:33-50): take!(length - 8) with usize wrapping
    if (n4 < 8) return v6 ? NPR_FLOW_L3_IPV6_UDP_INCOMPLETE : NPR_FLOW_L3_IPV4_UDP_INCOMPLETE;
    const uint32_t L = be16_of(r.le32(l4 + 4));
    if (L < 8u || n4 - 8u < L - 8u)
      return v6 ? NPR_FLOW_L3_IPV6_UDP_INCOMPLETE : NPR_FLOW_L3_IPV4_UDP_INCOMPLETE;
    if (n4 != L) return v6 ? NPR_FLOW_L3_IPV6_UDP_REMAINDER : NPR_FLOW_L3_IPV4_UDP_REMAINDER;
    udp = true;
  } else {
    return v6 ? NPR_FLOW_L3_IPV6_PROTOCOL : NPR_FLOW_L3_IPV4_PROTOCOL;
  }
  if (FIELDS) {  // Flow::new (src/flow/mod.rs:64-86)
    const uint32_t wp = r.le32(l4);
    f.d[2] = be16_of(wp) | (be16_of(wp >> 16) << 16);
    f.d[3] = vlan | (m1 & 0xffff0000u);
    f.d[4] = m2;
    f.d[5] = m0;
    f.d[6] = (m1 & 0xffffu) | (((v6 ? NPR_FLOW_KIND_IPV6 : 0u) | (udp ? NPR_FLOW_KIND_UDP : 0u)) << 16);
  }
  return NPR_FLOW_OK;
}

// ---------------------------------------------------------------------------------------------
// tile hand-off granules (MI355X_MICROARCH.md "R2": the data IS the flag, {tag, value} 8-B)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t gran(uint32_t tag, uint64_t v) { return ((uint64_t)tag << 48) | (v & kMask48); }
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// A segment of consecutive tiles [first, last] under speculation.
struct Seg {
  uint64_t entry, exit, cnt, ok;
  int64_t first, last, mism;  // mism: lowest tile whose speculated entry is contradicted
  bool valid;
};

__device__ __forceinline__ uint64_t tile_end(const ParseParams &kp, int64_t k) {
  const uint64_t e = kp.org + (uint64_t)(k + 1) * kTile;
  return e < kp.len ? e : kp.len;
}

// Chain-consistency monoid: X then Y (Y starts right after X).
__device__ __forceinline__ Seg combine(const ParseParams &kp, const Seg &X, const Seg &Y) {
  Seg r = X;
  r.last = Y.last;
  if (!X.valid) return r;                                 // keep the lowest mismatch
  if (X.exit < tile_end(kp, X.last)) return r;            // chain ended inside X: Y is moot
  if (X.exit != Y.entry) {                                // Y's speculated start is wrong
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
  __builtin_amdgcn_s_sleep(1);
  if (__hip_atomic_load(kp.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kp.epoch) return false;
  if (__builtin_amdgcn_s_memrealtime() - t0 > kp.timeout_ticks) {
    __hip_atomic_store(kp.abort_word, kp.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}

struct Prefix {
  uint64_t exit, cnt, ok;
};

// Decoupled look-back for tile t (run by wave 0; every lane returns the same result).
__device__ bool lookback(const ParseParams &kp, uint32_t t, Prefix &out) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t ep = kp.epoch;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {  // restart point after waiting for a mismatching tile's exact prefix
    Seg S{};
    bool s_has = false;
    int64_t hi = (int64_t)t - 1;
    bool restart = false;
    while (!restart) {
      const int64_t k = hi - lane;
      uint64_t v0 = 0, v1 = 0, v2 = 0;
      bool isP = false, isA = false;
      if (k >= 0) {
        const TileSlot *s = kp.slots + k;
        const uint64_t p0 = ld_agent(&s->p[0]), p1 = ld_agent(&s->p[1]), p2 = ld_agent(&s->p[2]);
        isP = (p0 >> 48) == ep && (p1 >> 48) == ep && (p2 >> 48) == ep;
        if (isP) {
          v0 = p0 & kMask48; v1 = p1 & kMask48; v2 = p2 & kMask48;
        } else {
          const uint64_t a0 = ld_agent(&s->a[0]), a1 = ld_agent(&s->a[1]), a2 = ld_agent(&s->a[2]);
          isA = (a0 >> 48) == ep && (a1 >> 48) == ep && (a2 >> 48) == ep;
          v0 = a0 & kMask48; v1 = a1 & kMask48; v2 = a2 & kMask48;
        }
      }
      const uint64_t bP = __ballot(isP), bA = __ballot(isA), bIn = __ballot(k >= 0);
      const int jp = bP ? __builtin_ctzll(bP) : 64;
      const uint64_t need = jp == 64 ? bIn : (jp == 0 ? 0ull : ((1ull << jp) - 1ull));
      if ((bA & need) != need) {  // a predecessor has published nothing yet
        if (!spin_ok(kp, t0)) return false;
        continue;
      }
      // serial (wave-uniform) combine from the lowest tile of the window upward
      const int jlo = jp < 64 ? jp : 63;
      Seg cur;
      cur.first = cur.last = hi - jlo;
      cur.mism = -1;
      cur.valid = true;
      if (jp < 64) {  // exact prefix
        cur.entry = 0;
        cur.exit = rl64(v0, jlo);
        cur.cnt = rl64(v1, jlo);
        cur.ok = rl64(v2, jlo);
      } else {
        const uint64_t e1 = rl64(v1, jlo), c = rl64(v2, jlo);
        cur.entry = e1 ? e1 - 1 : kNone;
        cur.exit = rl64(v0, jlo);
        cur.cnt = c & 0xffffffull;
        cur.ok = (c >> 24) & 0xffffffull;
      }
      for (int j = jlo - 1; j >= 0; --j) {
        Seg y;
        const uint64_t e1 = rl64(v1, j), c = rl64(v2, j);
        y.entry = e1 ? e1 - 1 : kNone;
        y.exit = rl64(v0, j);
        y.cnt = c & 0xffffffull;
        y.ok = (c >> 24) & 0xffffffull;
        y.first = y.last = hi - j;
        y.mism = -1;
        y.valid = true;
        cur = combine(kp, cur, y);
      }
      if (s_has) cur = combine(kp, cur, S);
      if (jp < 64) {
        if (cur.valid) {
          out.exit = cur.exit;
          out.cnt = cur.cnt;
          out.ok = cur.ok;
          return true;
        }
        // tile cur.mism speculated wrong: wait for its exact prefix, then start over
        const TileSlot *s = kp.slots + cur.mism;
        for (;;) {
          const uint64_t p0 = ld_agent(&s->p[0]), p1 = ld_agent(&s->p[1]), p2 = ld_agent(&s->p[2]);
          const bool ok = (p0 >> 48) == ep && (p1 >> 48) == ep && (p2 >> 48) == ep;
          if (__ballot(ok) & 1ull) break;
          if (!spin_ok(kp, t0)) return false;
        }
        restart = true;
      } else {
        S = cur;
        s_has = true;
        hi -= 64;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// speculation + chain walk
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool plaus1(uint32_t frac, uint32_t incl, uint32_t orig, uint32_t frac_max) {
  return incl >= 1u && incl <= kInclMax && orig >= incl && frac < frac_max;
}

// Is LDS offset rel (absolute p) a plausible record start?  Checks up to 3 chained headers
// inside the staged window.  A heuristic only: the look-back verifies every guess.
__device__ bool plausible(const ParseParams &kp, const uint32_t *w, uint64_t tile_lo, uint32_t rel) {
  const bool big = kp.big;
  const uint64_t p = tile_lo + rel;
  if (kp.len - p < 16) return false;
  uint32_t ts = hdr(w, rel, 0, big);
  const uint32_t incl = hdr(w, rel, 2, big);
  if (!plaus1(hdr(w, rel, 1, big), incl, hdr(w, rel, 3, big), kp.frac_max)) return false;
  if (kp.len - p - 16 < incl) return false;
  uint64_t q = p + 16 + incl;
  for (int hop = 0; hop < 2; ++hop) {
    if (q == kp.len) return true;
    const uint64_t qr = q - tile_lo;
    if (qr + 16 > (uint64_t)kStage) return true;  // beyond the staged window: cannot refute
    if (kp.len - q < 16) return true;              // truncated tail of the capture
    const uint32_t r = (uint32_t)qr;
    const uint32_t ts2 = hdr(w, r, 0, big), incl2 = hdr(w, r, 2, big);
    if (!plaus1(hdr(w, r, 1, big), incl2, hdr(w, r, 3, big), kp.frac_max)) return false;
    if (ts2 - ts + kTsWindow > 2u * kTsWindow) return false;
    if (kp.len - q - 16 < incl2) return true;
    ts = ts2;
    q = q + 16 + incl2;
  }
  return true;
}

// PcapRecords::parse loop (src/record.rs:30-49) over one tile, from `entry`, by wave 0.
// Records whose header starts before tile_hi belong to this tile.  Returns the exit: the first
// chain offset >= tile_hi, or (chain END, Q3) the offset of the first incomplete record.
__device__ uint64_t walk_tile(const ParseParams &kp, const uint32_t *w, uint16_t *srec,
                              uint64_t tile_lo, uint64_t tile_hi, uint64_t entry, uint32_t &n_out) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool big = kp.big;
  uint64_t p = entry;
  uint32_t n = 0;
  while (p < tile_hi) {
    const uint32_t incl = hdr(w, (uint32_t)(p - tile_lo), 2, big);
    if (kp.len - p < 16 || kp.len - p - 16 < incl) break;  // Err(Incomplete) -> stop (:37-45)
    const uint64_t stride = 16ull + incl;
    // stride speculation: lane j confirms the record at p + j*stride has the same length
    const uint64_t q = p + (uint64_t)lane * stride;
    bool ok = lane == 0;
    if (lane != 0 && q < tile_hi)
      ok = hdr(w, (uint32_t)(q - tile_lo), 2, big) == incl && kp.len - q >= stride;
    const uint64_t b = __ballot(ok);
    const uint32_t m = (~b == 0ull) ? 64u : (uint32_t)__builtin_ctzll(~b);
    if (lane < m) srec[n + lane] = (uint16_t)(q - tile_lo);
    n += m;
    p += (uint64_t)m * stride;
  }
  n_out = n;
  return p;
}

// Decode every record of the tile (status only) and count Ok flows per (slot, wave).
__device__ uint32_t count_pass(const ParseParams &kp, const uint32_t *w, const uint16_t *srec,
                               uint32_t n, uint64_t tile_lo, uint32_t (*scnt)[4]) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint8_t *b = (const uint8_t *)w;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const uint32_t i = tid + (uint32_t)s * kBlock;
    bool ok = false;
    if (i < n) {
      const uint32_t rel = srec[i];
      const uint64_t p = tile_lo + rel;
      const uint32_t incl = hdr(w, rel, 2, kp.big);
      TileReader r{w, b, rel + 16u, kp.buf + p + 16, kp.len - p - 16};
      FlowWords f;
      ok = decode<false>(r, incl, f) == NPR_FLOW_OK;
    }
    const uint64_t bal = __ballot(ok);
    if (lane == 0) scnt[s][wave] = (uint32_t)__builtin_popcountll(bal);
  }
  __syncthreads();
  uint32_t tot = 0;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) tot += scnt[s][0] + scnt[s][1] + scnt[s][2] + scnt[s][3];
  return tot;
}

// ---------------------------------------------------------------------------------------------
// the fused kernel
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_parse_extract(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) uint32_t sw[kStage / 4 + 4];
  __shared__ uint16_t srec[kMaxRec];
  __shared__ uint32_t scnt[kSlots][4];
  __shared__ uint32_t s_cand, s_n, s_abort;
  __shared__ uint64_t s_entry, s_exit, s_pexit, s_pcnt, s_pok;

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t t = blockIdx.x;
  const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
  const uint64_t tile_hi = tile_lo + kTile < kp.len ? tile_lo + kTile : kp.len;
  const bool big = kp.big;

  // 1. stage [tile_lo, tile_lo + kStage) into LDS.  The descriptor range is rounded up to the
  //    16-B chunk so a partially valid last chunk is read whole (same page); bytes past it read 0.
  {
    const uint64_t avail = kp.len > tile_lo ? kp.len - tile_lo : 0;
    uint32_t nbytes = avail < (uint64_t)kStage ? (uint32_t)avail : (uint32_t)kStage;
    nbytes = (nbytes + 15u) & ~15u;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(kp.buf + tile_lo), 0, (int)nbytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < (kStage / 16 + kBlock - 1) / kBlock; ++i) {
      const uint32_t c = tid + (uint32_t)i * kBlock;
      if (c < kStage / 16) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(c * 16u), 0, 0);
        *reinterpret_cast<decltype(v) *>(&sw[c * 4]) = v;
      }
    }
    if (tid < 4) sw[kStage / 4 + tid] = 0;
  }
  __syncthreads();

  // 2. entry: exact for tile 0, speculated otherwise
  uint64_t entry;
  if (t == 0 && !(kp.flags & kFlagSpecFirst)) {
    entry = kp.start;
  } else {
    if (tid == 0) s_cand = 0xffffffffu;
    __syncthreads();
    const uint64_t lo = (t == 0) ? kp.start : tile_lo;
    const uint32_t span = (uint32_t)(tile_hi - tile_lo);
    for (uint32_t base = (uint32_t)(lo - tile_lo); base < span; base += kBlock) {
      const uint32_t rel = base + tid;
      const bool ok = rel < span && plausible(kp, sw, tile_lo, rel);
      if (ok) atomicMin(&s_cand, rel);
      if (__syncthreads_or(ok)) break;
    }
    entry = s_cand == 0xffffffffu ? kNone : tile_lo + s_cand;
  }

  // 3. speculative walk (wave 0)
  if (wave == 0) {
    uint32_t n = 0;
    uint64_t ex = 0;
    if (entry != kNone) ex = walk_tile(kp, sw, srec, tile_lo, tile_hi, entry, n);
    if (lane == 0) {
      s_n = n;
      s_entry = entry;
      s_exit = ex;
    }
  }
  __syncthreads();

  // 4. Ok-flow count of the speculative record set
  uint32_t okc = count_pass(kp, sw, srec, s_n, tile_lo, scnt);

  // 5. publish, 6. look back, 7. repair
  const uint32_t ep = kp.epoch;
  TileSlot *slot = kp.slots + t;
  uint64_t pexit = 0, pcnt = 0, pok = 0;
  if (t == 0) {
    if (tid == 0) {
      st_agent(&slot->p[0], gran(ep, s_exit));
      st_agent(&slot->p[1], gran(ep, s_n));
      st_agent(&slot->p[2], gran(ep, okc));
    }
  } else {
    if (tid == 0) {
      st_agent(&slot->a[0], gran(ep, s_exit));
      st_agent(&slot->a[1], gran(ep, s_entry == kNone ? 0ull : s_entry + 1));
      st_agent(&slot->a[2], gran(ep, (uint64_t)s_n | ((uint64_t)okc << 24)));
    }
    if (wave == 0) {
      Prefix pre{0, 0, 0};
      const bool ok = lookback(kp, t, pre);
      if (lane == 0) {
        s_abort = ok ? 0u : 1u;
        s_pexit = pre.exit;
        s_pcnt = pre.cnt;
        s_pok = pre.ok;
      }
    }
    __syncthreads();
    if (s_abort) return;
    pexit = s_pexit;
    pcnt = s_pcnt;
    pok = s_pok;
    if (pexit != s_entry) {
      // the speculation was wrong (or there is no record start here): redo from the truth
      if (wave == 0) {
        uint32_t n = 0;
        uint64_t ex = pexit;
        if (pexit >= tile_lo && pexit < tile_hi) ex = walk_tile(kp, sw, srec, tile_lo, tile_hi, pexit, n);
        if (lane == 0) {
          s_n = n;
          s_exit = ex;
        }
      }
      __syncthreads();
      okc = count_pass(kp, sw, srec, s_n, tile_lo, scnt);
    }
    if (tid == 0) {
      st_agent(&slot->p[0], gran(ep, s_exit));
      st_agent(&slot->p[1], gran(ep, pcnt + s_n));
      st_agent(&slot->p[2], gran(ep, pok + okc));
    }
  }
  const uint32_t n = s_n;

  // 8. totals (last tile)
  if (t == kp.ntiles - 1 && tid == 0) {
    const uint64_t tot_rec = pcnt + n, tot_ok = pok + okc;
    uint32_t fl = 0;
    if ((kp.rec_off || kp.recs || kp.rec_status) && tot_rec > kp.rec_cap) fl |= NPR_SUMMARY_RECORD_OVERFLOW;
    if (kp.flows && tot_ok > kp.flow_cap) fl |= NPR_SUMMARY_FLOW_OVERFLOW;
    kp.summary->n_records = tot_rec;
    kp.summary->n_flows = tot_ok;
    kp.summary->consumed = s_exit;
    kp.summary->flags = fl;
    kp.summary->epoch = ep;
  }

  // 9. outputs at their global positions
  const uint8_t *sb = (const uint8_t *)sw;
  uint32_t slot_base = 0;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) {
    const uint32_t i = tid + (uint32_t)s * kBlock;
    bool ok = false;
    FlowWords f;
    uint64_t p = 0;
    if (i < n) {
      const uint32_t rel = srec[i];
      p = tile_lo + rel;
      const uint32_t incl = hdr(sw, rel, 2, big);
      TileReader r{sw, sb, rel + 16u, kp.buf + p + 16, kp.len - p - 16};
      const uint32_t st = decode<true>(r, incl, f);
      ok = st == NPR_FLOW_OK;
      const uint64_t idx = pcnt + i;
      if (idx < kp.rec_cap) {
        if (kp.rec_off) kp.rec_off[idx] = p;
        if (kp.recs) {
          uint64_t *row = reinterpret_cast<uint64_t *>(kp.recs + idx);
          row[0] = p;
          row[1] = (uint64_t)hdr(sw, rel, 0, big) | ((uint64_t)hdr(sw, rel, 1, big) << 32);
          row[2] = (uint64_t)incl | ((uint64_t)hdr(sw, rel, 3, big) << 32);
        }
        if (kp.rec_status) kp.rec_status[idx] = (uint8_t)st;
      }
    }
    const uint64_t bal = __ballot(ok);
    if (ok && kp.flows) {
      uint32_t rank = slot_base + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      for (uint32_t v = 0; v < wave; ++v) rank += scnt[s][v];
      const uint64_t fi = pok + rank;
      if (fi < kp.flow_cap) {
        const uint64_t o = kp.flow_cap - 1 - fi;  // convert_records pops from the end
        uint4 *dst = reinterpret_cast<uint4 *>(kp.flows + o * 8);
        dst[0] = make_uint4(f.d[0], f.d[1], f.d[2], f.d[3]);
        dst[1] = make_uint4(f.d[4], f.d[5], f.d[6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8));
        if (kp.flows_v6 && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16))) {
          uint4 *d6 = reinterpret_cast<uint4 *>(kp.flows_v6 + o * 8);
          d6[0] = make_uint4(f.v6[0], f.v6[1], f.v6[2], f.v6[3]);
          d6[1] = make_uint4(f.v6[4], f.v6[5], f.v6[6], f.v6[7]);
        }
      }
    }
    slot_base += scnt[s][0] + scnt[s][1] + scnt[s][2] + scnt[s][3];
  }
}

hipError_t launch_parse_extract(const ParseParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_parse_extract, dim3(p.ntiles), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// dense extract over caller-supplied records (FlowExtraction::extract_flow per PcapRecord)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_extract_dense(const uint8_t *buf, uint64_t len,
                                                          const npr_record *recs, uint64_t n,
                                                          uint32_t *flows, uint32_t *flows_v6,
                                                          uint8_t *status) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const npr_record rc = recs[i];
  const uint64_t off = rc.offset + 16;
  uint32_t st = 0xffu;  // record does not lie inside the buffer
  FlowWords f{};
  if (off <= len && len - off >= rc.actual_length) {
    GlobalReader r{buf + off, len - off};
    st = decode<true>(r, rc.actual_length, f);
  }
  const bool ok = st == NPR_FLOW_OK;
  if (status) status[i] = (uint8_t)st;
  if (flows) {
    uint4 *dst = reinterpret_cast<uint4 *>(flows + i * 8);
    const uint64_t p = rc.offset;
    dst[0] = ok ? make_uint4(f.d[0], f.d[1], f.d[2], f.d[3]) : make_uint4(0, 0, 0, 0);
    dst[1] = ok ? make_uint4(f.d[4], f.d[5], f.d[6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8))
                : make_uint4(0, 0, 0, 0);
  }
  if (flows_v6) {
    const bool is6 = ok && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16));
    uint4 *d6 = reinterpret_cast<uint4 *>(flows_v6 + i * 8);
    d6[0] = is6 ? make_uint4(f.v6[0], f.v6[1], f.v6[2], f.v6[3]) : make_uint4(0, 0, 0, 0);
    d6[1] = is6 ? make_uint4(f.v6[4], f.v6[5], f.v6[6], f.v6[7]) : make_uint4(0, 0, 0, 0);
  }
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
// reverse-order compaction (convert_records over a dense extract): count / scan / scatter
// ---------------------------------------------------------------------------------------------
constexpr int kCompactItems = 1024;  // records per block

__global__ __launch_bounds__(kBlock) void k_compact_count(const uint8_t *status, uint64_t n, uint32_t *counts) {
  __shared__ uint32_t sc[4];
  const uint64_t b0 = (uint64_t)blockIdx.x * kCompactItems;
  uint32_t c = 0;
  for (int k = 0; k < kCompactItems / kBlock; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kBlock;
    c += (i < n && status[i] == NPR_FLOW_OK) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63u) == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
}

// exclusive scan of nb counts by one workgroup (chunks of 256)
__global__ __launch_bounds__(kBlock) void k_compact_scan(uint32_t *counts, uint64_t nb, uint64_t *total) {
  __shared__ uint64_t part[kBlock];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (uint64_t base = 0; base < nb; base += kBlock) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t v = i < nb ? counts[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kBlock; o <<= 1) {
      const uint64_t add = threadIdx.x >= (uint32_t)o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < nb) counts[i] = (uint32_t)(carry + part[threadIdx.x] - v);
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry += part[kBlock - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kBlock) void k_compact_scatter(const uint32_t *flows, const uint32_t *flows_v6,
                                                            const uint8_t *status, uint64_t n,
                                                            const uint32_t *offsets, const uint64_t *total,
                                                            uint32_t *out, uint32_t *out_v6, uint64_t cap) {
  __shared__ uint32_t sc[kCompactItems / kBlock][4];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kCompactItems;
  bool ok[kCompactItems / kBlock];
  for (int k = 0; k < kCompactItems / kBlock; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kBlock;
    ok[k] = i < n && status[i] == NPR_FLOW_OK;
    const uint64_t bal = __ballot(ok[k]);
    if (lane == 0) sc[k][wave] = (uint32_t)__builtin_popcountll(bal);
  }
  __syncthreads();
  const uint64_t tot = *total;
  uint64_t base = offsets[blockIdx.x];
  for (int k = 0; k < kCompactItems / kBlock; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kBlock;
    const uint64_t bal = __ballot(ok[k]);
    if (ok[k]) {
      uint64_t rank = base + (uint64_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      for (uint32_t v = 0; v < wave; ++v) rank += sc[k][v];
      const uint64_t o = tot - 1 - rank;  // reverse file order
      if (o < cap) {
        const uint4 *src = reinterpret_cast<const uint4 *>(flows + i * 8);
        uint4 *dst = reinterpret_cast<uint4 *>(out + o * 8);
        dst[0] = src[0];
        dst[1] = src[1];
        if (out_v6 && flows_v6) {
          const uint4 *s6 = reinterpret_cast<const uint4 *>(flows_v6 + i * 8);
          uint4 *d6 = reinterpret_cast<uint4 *>(out_v6 + o * 8);
          d6[0] = s6[0];
          d6[1] = s6[1];
        }
      }
    }
    base += sc[k][0] + sc[k][1] + sc[k][2] + sc[k][3];
  }
}

uint64_t compact_workspace_words(uint64_t n) { return (n + kCompactItems - 1) / kCompactItems; }

hipError_t launch_compact_reverse(const uint32_t *flows, const uint32_t *flows_v6, const uint8_t *status,
                                  uint64_t n, uint32_t *out, uint32_t *out_v6, uint64_t cap,
                                  uint32_t *block_counts, uint64_t *total, hipStream_t s) {
  const uint64_t nb = compact_workspace_words(n);
  if (nb == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), s);
  hipLaunchKernelGGL(k_compact_count, dim3((uint32_t)nb), dim3(kBlock), 0, s, status, n, block_counts);
  hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(kBlock), 0, s, block_counts, nb, total);
  hipLaunchKernelGGL(k_compact_scatter, dim3((uint32_t)nb), dim3(kBlock), 0, s, flows, flows_v6, status, n,
                     block_counts, total, out, out_v6, cap);
  return hipGetLastError();
}

}  // namespace npr
