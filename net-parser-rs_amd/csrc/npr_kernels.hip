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

// diagnostic counters of the current wave (kept in registers; written to the stamp row)
struct Diag {
  uint32_t spins = 0, slides = 0, mism = 0;
};

// One lane's view of one segment of the look-back window: a tile, or a group of kGroup tiles.
struct LaneSeg {
  uint64_t entry, exit, cnt, ok;
  int64_t first, last, mism;
  bool present;  // an aggregate or an exact prefix has been published
  bool anchor;   // exact inclusive prefix through `last` (cnt/ok are absolute)
  bool valid;
};

__device__ __forceinline__ bool tagged(uint64_t w, uint32_t ep) { return (w >> 48) == ep; }

// tile k: P (exact prefix) or A (speculative aggregate); all six granules are loaded at once
__device__ __forceinline__ LaneSeg load_tile(const ParseParams &kp, int64_t k, bool inr) {
  LaneSeg L{};
  L.first = L.last = k;
  L.mism = -1;
  L.valid = true;
  if (!inr) return L;
  const uint32_t ep = kp.epoch;
  const TileSlot *s = kp.slots + k;
  const uint64_t p0 = ld_agent(&s->p[0]), p1 = ld_agent(&s->p[1]), p2 = ld_agent(&s->p[2]);
  const uint64_t a0 = ld_agent(&s->a[0]), a1 = ld_agent(&s->a[1]), a2 = ld_agent(&s->a[2]);
  if (tagged(p0, ep) && tagged(p1, ep) && tagged(p2, ep)) {
    L.present = L.anchor = true;
    L.exit = p0 & kMask48;
    L.cnt = p1 & kMask48;
    L.ok = p2 & kMask48;
  } else if (tagged(a0, ep) && tagged(a1, ep) && tagged(a2, ep)) {
    L.present = true;
    const uint64_t e1 = a1 & kMask48, c = a2 & kMask48;
    L.entry = e1 ? e1 - 1 : kNone;
    L.exit = a0 & kMask48;
    L.cnt = c & 0xffffffull;
    L.ok = (c >> 24) & 0xffffffull;
  }
  return L;
}

// group gg (tiles [gg*kGroup, gg*kGroup + kGroup)): the exact prefix of its last tile, or the
// group aggregate G published by that tile (anchored when it was folded from an exact prefix)
__device__ __forceinline__ LaneSeg load_group(const ParseParams &kp, int64_t gg, bool inr) {
  LaneSeg L{};
  L.first = gg * kGroup;
  L.last = gg * kGroup + kGroup - 1;
  L.mism = -1;
  L.valid = true;
  if (!inr) return L;
  const uint32_t ep = kp.epoch;
  const TileSlot *s = kp.slots + L.last;
  const GroupSlot *g = kp.groups + gg;
  const uint64_t p0 = ld_agent(&s->p[0]), p1 = ld_agent(&s->p[1]), p2 = ld_agent(&s->p[2]);
  const uint64_t g0 = ld_agent(&g->g[0]), g1 = ld_agent(&g->g[1]), g2 = ld_agent(&g->g[2]),
                 g3 = ld_agent(&g->g[3]);
  if (tagged(p0, ep) && tagged(p1, ep) && tagged(p2, ep)) {
    L.present = L.anchor = true;
    L.exit = p0 & kMask48;
    L.cnt = p1 & kMask48;
    L.ok = p2 & kMask48;
  } else if (tagged(g0, ep) && tagged(g1, ep) && tagged(g2, ep) && tagged(g3, ep)) {
    L.present = true;
    const uint64_t e1 = g1 & kMask48, w3 = g3 & kMask48;
    L.entry = e1 ? e1 - 1 : kNone;
    L.exit = g0 & kMask48;
    L.cnt = g2 & kMask48;
    L.ok = w3 & ((1ull << 40) - 1);
    L.valid = (w3 >> 40) & 1ull;
    L.anchor = (w3 >> 41) & 1ull;
    L.mism = L.valid ? -1 : L.first + (int64_t)((w3 >> 42) & 63ull);
  }
  return L;
}

__device__ __forceinline__ uint64_t shfl_down64(uint64_t v) {
  const uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v, 1);
  const uint32_t hi = (uint32_t)__shfl_down((int)(uint32_t)(v >> 32), 1);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Fold the window lanes [lo .. 0] (ascending tile order = descending lane) into one segment.
// Every lane <= lo must be present.  Fast path: all links consistent, no END, all valid ->
// two wave sums; otherwise the serial monoid (wave-uniform, readlane).
__device__ Seg fold_window(const ParseParams &kp, const LaneSeg &L, int lo) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint64_t prev_exit = shfl_down64(L.exit);  // exit of the preceding segment (lane + 1)
  const bool inr = lane <= lo;
  const bool bad = lane < lo && (!L.valid || L.entry != prev_exit);
  const bool endc = inr && L.exit < tile_end(kp, L.last);
  const bool lo_bad = lane == lo && !L.valid;
  Seg r;
  if (__ballot(bad || endc || lo_bad) == 0ull) {
    r.cnt = wave_sum64(inr ? L.cnt : 0ull);
    r.ok = wave_sum64(inr ? L.ok : 0ull);
    r.entry = rl64(L.entry, lo);
    r.exit = rl64(L.exit, 0);
    r.first = (int64_t)rl64((uint64_t)L.first, lo);
    r.last = (int64_t)rl64((uint64_t)L.last, 0);
    r.mism = -1;
    r.valid = true;
    return r;
  }
  auto lane_seg = [&](int j) {
    Seg y;
    y.entry = rl64(L.entry, j);
    y.exit = rl64(L.exit, j);
    y.cnt = rl64(L.cnt, j);
    y.ok = rl64(L.ok, j);
    y.first = (int64_t)rl64((uint64_t)L.first, j);
    y.last = (int64_t)rl64((uint64_t)L.last, j);
    y.mism = (int64_t)rl64((uint64_t)L.mism, j);
    y.valid = (__ballot(L.valid) >> j) & 1ull;
    return y;
  };
  r = lane_seg(lo);
  for (int j = lo - 1; j >= 0; --j) r = combine(kp, r, lane_seg(j));
  return r;
}

// Wait for the exact prefix that resolves mismatching tile m: its own P when m is in tile t's
// group (the tile-level window will see it), else the P of the last tile of m's group.
__device__ bool wait_resolved(const ParseParams &kp, int64_t m, uint32_t g, uint64_t t0, Diag &dg) {
  dg.mism += 1;
  const int64_t gm = m / kGroup;
  const int64_t k = gm == (int64_t)g ? m : gm * kGroup + kGroup - 1;
  const TileSlot *s = kp.slots + k;
  for (;;) {
    const uint64_t p0 = ld_agent(&s->p[0]), p1 = ld_agent(&s->p[1]), p2 = ld_agent(&s->p[2]);
    const bool ok = tagged(p0, kp.epoch) && tagged(p1, kp.epoch) && tagged(p2, kp.epoch);
    if (__ballot(ok) & 1ull) return true;
    if (!spin_ok(kp, t0)) return false;
  }
}

// Two-level decoupled look-back for tile t (wave 0; every lane returns the same result).
//   L1: the tiles of t's own group before t — an exact prefix there ends the search;
//   L2: the groups before — exact group prefixes (P of a group's last tile) or group aggregates,
//       64 groups (4096 tiles) per poll, sliding further back only if no exact prefix is in range.
// Any inconsistency is resolved by waiting for the exact prefix of the offending tile/group.
__device__ bool lookback(const ParseParams &kp, uint32_t t, Prefix &out, Diag &dg) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t g = t / kGroup, i = t % kGroup;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {  // restart point after waiting for a mismatch to resolve
    bool restart = false;
    Seg S{};
    bool s_has = false;
    if (i > 0) {  // ---- L1
      for (;;) {
        const bool inr = lane < (int)i;
        const LaneSeg L = load_tile(kp, (int64_t)t - 1 - lane, inr);
        const uint64_t bAnc = __ballot(inr && L.anchor), bPres = __ballot(inr && L.present);
        const int jp = bAnc ? __builtin_ctzll(bAnc) : (int)i;
        const uint64_t need = jp >= 64 ? ~0ull : ((1ull << jp) - 1ull);
        const uint64_t need_in = jp < (int)i ? need : (i >= 64 ? ~0ull : ((1ull << i) - 1ull));
        if ((bPres & need_in) != need_in) {
          ++dg.spins;
          if (!spin_ok(kp, t0)) return false;
          continue;
        }
        const Seg cur = fold_window(kp, L, jp < (int)i ? jp : (int)i - 1);
        if (jp < (int)i) {
          if (cur.valid) {
            out.exit = cur.exit;
            out.cnt = cur.cnt;
            out.ok = cur.ok;
            return true;
          }
          if (!wait_resolved(kp, cur.mism, g, t0, dg)) return false;
          restart = true;
        } else {
          S = cur;
          s_has = true;
        }
        break;
      }
      if (restart) continue;
    }
    // ---- L2 (g >= 1 here: in group 0 tile 0's exact prefix is always inside the L1 window)
    int64_t gh = (int64_t)g - 1;
    for (;;) {
      const int64_t gg = gh - lane;
      const bool inr = gg >= 0;
      const LaneSeg L = load_group(kp, gg, inr);
      const int n = gh + 1 < 64 ? (int)(gh + 1) : 64;
      const uint64_t bAnc = __ballot(inr && L.anchor), bPres = __ballot(inr && L.present);
      const int jp = bAnc ? __builtin_ctzll(bAnc) : n;
      const uint64_t need = jp >= 64 ? ~0ull : ((1ull << jp) - 1ull);
      if ((bPres & need) != need) {
        ++dg.spins;
        if (!spin_ok(kp, t0)) return false;
        continue;
      }
      Seg cur = fold_window(kp, L, jp < n ? jp : n - 1);
      if (s_has) cur = combine(kp, cur, S);
      if (jp < n) {
        if (cur.valid) {
          out.exit = cur.exit;
          out.cnt = cur.cnt;
          out.ok = cur.ok;
          return true;
        }
        if (!wait_resolved(kp, cur.mism, g, t0, dg)) return false;
        restart = true;
        break;
      }
      dg.slides += 1;
      S = cur;
      s_has = true;
      gh -= 64;
    }
    (void)restart;
  }
}

// Tile gL*kGroup + kGroup-1 (wave 0), right after publishing its own aggregate: fold the group's
// 64 tile records into one group aggregate G (anchored when an exact prefix is among them).
__device__ bool publish_group(const ParseParams &kp, uint32_t gL) {
  const int lane = (int)(threadIdx.x & 63u);
  const uint32_t ep = kp.epoch;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const int64_t last = (int64_t)gL * kGroup + kGroup - 1;
  for (;;) {
    const LaneSeg L = load_tile(kp, last - lane, true);
    const uint64_t bAnc = __ballot(L.anchor), bPres = __ballot(L.present);
    const int jp = bAnc ? __builtin_ctzll(bAnc) : 64;
    const uint64_t need = jp >= 64 ? ~0ull : ((1ull << jp) - 1ull);
    if ((bPres & need) != need) {
      if (!spin_ok(kp, t0)) return false;
      continue;
    }
    const Seg cur = fold_window(kp, L, jp < 64 ? jp : 63);
    if (lane == 0) {
      GroupSlot *G = kp.groups + gL;
      const bool anchored = jp < 64;
      const uint64_t mrel = cur.valid ? 0ull : (uint64_t)(cur.mism - (int64_t)gL * kGroup) & 63ull;
      st_agent(&G->g[0], gran(ep, cur.exit));
      st_agent(&G->g[1], gran(ep, (anchored || cur.entry == kNone) ? 0ull : cur.entry + 1));
      st_agent(&G->g[2], gran(ep, cur.cnt));
      st_agent(&G->g[3], gran(ep, (cur.ok & ((1ull << 40) - 1)) | ((uint64_t)cur.valid << 40) |
                                      ((uint64_t)anchored << 41) | (mrel << 42)));
    }
    return true;
  }
}

// ---------------------------------------------------------------------------------------------
// speculation + chain walk
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool plaus1(uint32_t frac, uint32_t incl, uint32_t orig, uint32_t frac_max) {
  return incl >= 1u && incl <= kInclMax && orig >= incl && frac < frac_max;
}

// How plausible is LDS offset rel (absolute p) as a record start?  0 = no; 1 = weak (its header
// passes but fewer than two chained headers could be checked inside the staged window);
// 2 = strong (two further headers check out, or the chain ends exactly at EOF).  A heuristic
// only: the look-back verifies every guess, a wrong one costs a re-walk, never a wrong result.
__device__ int plausibility(const ParseParams &kp, const uint32_t *w, uint64_t tile_lo, uint32_t rel,
                            uint32_t frac_max) {
  const bool big = kp.big;
  const uint64_t p = tile_lo + rel;
  if (kp.len - p < 16) return 0;
  uint32_t ts = hdr(w, rel, 0, big);
  const uint32_t incl = hdr(w, rel, 2, big);
  if (!plaus1(hdr(w, rel, 1, big), incl, hdr(w, rel, 3, big), frac_max)) return 0;
  if (kp.len - p - 16 < incl) return 0;
  uint64_t q = p + 16 + incl;
  int verified = 0;
  for (int hop = 0; hop < 3; ++hop) {
    if (q == kp.len) return 2;                                // chain ends exactly at EOF
    const uint64_t qr = q - tile_lo;
    if (qr + 16 > (uint64_t)kStage) return verified >= 2 ? 2 : 1;  // beyond the window
    if (kp.len - q < 16) return verified >= 1 ? 2 : 1;         // truncated tail
    const uint32_t r = (uint32_t)qr;
    const uint32_t ts2 = hdr(w, r, 0, big), incl2 = hdr(w, r, 2, big);
    if (!plaus1(hdr(w, r, 1, big), incl2, hdr(w, r, 3, big), frac_max)) return 0;
    if (ts2 - ts + kTsWindow > 2u * kTsWindow) return 0;
    ++verified;
    if (kp.len - q - 16 < incl2) return verified >= 2 ? 2 : 1;  // truncated final record
    ts = ts2;
    q = q + 16 + incl2;
  }
  return 2;
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

__device__ __forceinline__ void stamp(const ParseParams &kp, uint32_t t, int k) {
  if (kp.stamps && threadIdx.x == 0) kp.stamps[(uint64_t)t * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------------------------
// the fused kernel
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_parse_extract(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) uint32_t sw[kStage / 4 + 4];
  __shared__ uint16_t srec[kMaxRec];
  __shared__ uint32_t scnt[kSlots][4];
  __shared__ uint32_t s_cand, s_weak, s_n, s_abort;
  __shared__ uint64_t s_entry, s_exit, s_pexit, s_pcnt, s_pok;

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t t = blockIdx.x;
  const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
  const uint64_t tile_hi = tile_lo + kTile < kp.len ? tile_lo + kTile : kp.len;
  const bool big = kp.big;
  stamp(kp, t, 0);

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
  stamp(kp, t, 1);

  // 2. entry: exact for tile 0, speculated otherwise (first strong candidate, else first weak)
  uint64_t entry;
  if (t == 0 && !(kp.flags & kFlagSpecFirst)) {
    entry = kp.start;
  } else {
    uint32_t frac_max = kp.frac_max;
    if (kp.flags & kFlagMagicAtZero) {  // pcap magic: microsecond captures bound ts_usec < 1e6
      const uint32_t m = *reinterpret_cast<const uint32_t *>(kp.buf);
      if (m == 0xA1B2C3D4u || m == 0xD4C3B2A1u) frac_max = 1000000u;
    }
    if (tid == 0) {
      s_cand = 0xffffffffu;
      s_weak = 0xffffffffu;
    }
    __syncthreads();
    const uint64_t lo = (t == 0) ? kp.start : tile_lo;
    const uint32_t span = (uint32_t)(tile_hi - tile_lo);
    for (uint32_t base = (uint32_t)(lo - tile_lo); base < span; base += kBlock) {
      const uint32_t rel = base + tid;
      const int grade = rel < span ? plausibility(kp, sw, tile_lo, rel, frac_max) : 0;
      if (grade == 2) atomicMin(&s_cand, rel);
      else if (grade == 1) atomicMin(&s_weak, rel);
      if (__syncthreads_or(grade == 2)) break;
    }
    const uint32_t c = s_cand != 0xffffffffu ? s_cand : s_weak;
    entry = c == 0xffffffffu ? kNone : tile_lo + c;
    if (kp.stats && tid == 0) {
      if (s_cand == 0xffffffffu) atomicAdd(&kp.stats[c == 0xffffffffu ? kStatNoEntry : kStatWeakEntry], 1u);  // rare
    }
  }

  stamp(kp, t, 2);
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
  stamp(kp, t, 3);

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
      bool ok = true;
      if (t % kGroup == kGroup - 1) ok = publish_group(kp, t / kGroup);
      Diag dg;
      if (ok) ok = lookback(kp, t, pre, dg);
      if (kp.stamps && lane == 0)
        kp.stamps[(uint64_t)t * 8 + 7] = (uint64_t)dg.spins | ((uint64_t)dg.slides << 20) | ((uint64_t)dg.mism << 40);
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
      if (kp.stats && tid == 0) atomicAdd(&kp.stats[kStatRewalk], 1u);
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
  stamp(kp, t, 4);

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
  stamp(kp, t, 5);
  if (kp.stamps && tid == 0) kp.stamps[(uint64_t)t * 8 + 6] = ((uint64_t)s_n << 32) | (pexit != s_entry ? 1u : 0u);
}

hipError_t launch_parse_extract(const ParseParams &p, hipStream_t s) {
  hipLaunchKernelGGL(k_parse_extract, dim3(p.ntiles), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

// =============================================================================================
// Persistent, software-pipelined kernel.  gridDim.x = G resident workgroups;
// workgroup b owns tiles b, b+G, b+2G, ...  Iteration k overlaps three tiles:
//   - registers receive tile k+1 from HBM (prefetch issued first, committed to LDS last);
//   - phase A, wave 0: speculate + walk tile k;  wave 1: resolve tile k-1 (its aggregate was
//     published one iteration ago; the look-back words were loaded at the top of the iteration)
//     and write its records/flows;  wave 2: fold the group-level look-back window for wave 1;
//   - phase B, all waves: decode tile k once (Ok flows parked in LDS in rank order), publish.
// HBM latency and hand-off latency hide behind a whole tile of LDS work; no wave waits for a
// store.  Inter-workgroup hand-offs use self-validating {tag, value} granules (agent scope).
// =============================================================================================
typedef unsigned int u32x4 __attribute__((__vector_size__(16)));  // the b128 buffer-load type

constexpr int kParkFlows = 288;  // >= max Ok flows per tile: an Ok record spans >= 16 + 42 bytes
constexpr int kPrefetch = (kStage / 16 + kBlock - 1) / kBlock;  // 16-B chunks per thread
constexpr uint32_t kOrigMax = 1u << 18;   // speculation: plausible orig_len bound
constexpr uint32_t kTsRefWindow = 1u << 26;  // speculation: |ts_sec - first record's ts_sec|

struct PipeShared {
  uint32_t data[kStage / 4 + 4];
  uint16_t srec[2][kMaxRec];
  uint32_t park[kParkFlows * 8];
  uint8_t pstat[kMaxRec];
  uint32_t scnt[kSlots][4];
  uint64_t entry[2], exit[2];
  uint32_t n[2], okc[2];
  uint64_t pexit, pcnt, pok;
  Seg l2;
  uint32_t l2_state, l2_tag, slow, abort;
};

__device__ __forceinline__ void prefetch_tile(const ParseParams &kp, uint32_t t, u32x4 (&q)[kPrefetch],
                                              bool valid = true) {
  const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
  const uint64_t avail = valid && kp.len > tile_lo ? kp.len - tile_lo : 0;
  uint32_t nbytes = avail < (uint64_t)kStage ? (uint32_t)avail : (uint32_t)kStage;
  nbytes = (nbytes + 15u) & ~15u;  // 0 when !valid: every load is out of range, nothing is fetched
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(kp.buf + tile_lo), 0, (int)nbytes, 0x00020000);
  // unconditional loads (chunks past the staged range are out of the descriptor's range -> 0):
  // one load sequence with one consumer keeps hipcc's waitcnt tracking exact
#pragma unroll
  for (int i = 0; i < kPrefetch; ++i) {
    const uint32_t c = threadIdx.x + (uint32_t)i * kBlock;
    q[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(c * 16u), 0, 0);
  }
}

__device__ __forceinline__ void commit_tile(uint32_t *data, const u32x4 (&q)[kPrefetch]) {
#pragma unroll
  for (int i = 0; i < kPrefetch; ++i) {
    const uint32_t c = threadIdx.x + (uint32_t)i * kBlock;
    if (c < kStage / 16) *reinterpret_cast<u32x4 *>(&data[c * 4]) = q[i];
  }
  if (threadIdx.x < 4) data[kStage / 4 + threadIdx.x] = 0;
}

// ---- speculation in tile-relative 32-bit arithmetic (wave 0, 64 candidates per round) --------
struct SpecCtx {
  uint32_t avail;    // bytes of the input from tile_lo, saturated to 32 bits
  bool exact_end;    // avail is exact (not saturated): q == avail means "chain ends at EOF"
  uint32_t frac_max, ts_ref;
  bool has_ref;
  bool big;
};

__device__ __forceinline__ bool plaus2(const SpecCtx &c, uint32_t ts, uint32_t frac, uint32_t incl, uint32_t orig) {
  return incl >= 1u && incl <= kInclMax && orig >= incl && orig <= kOrigMax && frac < c.frac_max &&
         (!c.has_ref || ts - c.ts_ref + kTsRefWindow <= 2u * kTsRefWindow);
}

// 0 = implausible, 1 = weak (fewer than two further headers checkable), 2 = strong
__device__ __forceinline__ int grade32(const SpecCtx &c, const uint32_t *w, uint32_t r) {
  if (c.avail - r < 16) return 0;
  uint32_t ts = hdr(w, r, 0, c.big);
  const uint32_t incl = hdr(w, r, 2, c.big);
  if (!plaus2(c, ts, hdr(w, r, 1, c.big), incl, hdr(w, r, 3, c.big))) return 0;
  if (c.avail - r - 16 < incl) return 0;
  uint32_t q = r + 16 + incl;
  int ver = 0;
  for (int hop = 0; hop < 3; ++hop) {
    if (q == c.avail && c.exact_end) return 2;
    if (q + 16 > (uint32_t)kStage) return ver >= 2 ? 2 : 1;
    if (c.avail - q < 16) return ver >= 1 ? 2 : 1;
    const uint32_t ts2 = hdr(w, q, 0, c.big), incl2 = hdr(w, q, 2, c.big);
    if (!plaus2(c, ts2, hdr(w, q, 1, c.big), incl2, hdr(w, q, 3, c.big))) return 0;
    if (ts2 - ts + kTsWindow > 2u * kTsWindow) return 0;
    ++ver;
    if (c.avail - q - 16 < incl2) return ver >= 2 ? 2 : 1;
    ts = ts2;
    q += 16 + incl2;
  }
  return 2;
}

// first strong candidate in [lo_rel, span), else the first weak one; kNone if neither (wave-uniform)
__device__ uint64_t speculate_wave(const SpecCtx &c, const uint32_t *w, uint64_t tile_lo, uint32_t lo_rel,
                                   uint32_t span) {
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t weak = 0xffffffffu;
  for (uint32_t base = lo_rel; base < span; base += 64) {
    const uint32_t r = base + lane;
    const int g = r < span ? grade32(c, w, r) : 0;
    const uint64_t b2 = __ballot(g == 2);
    if (b2) return tile_lo + base + (uint32_t)__builtin_ctzll(b2);
    const uint64_t b1 = __ballot(g == 1);
    if (weak == 0xffffffffu && b1) weak = base + (uint32_t)__builtin_ctzll(b1);
  }
  return weak == 0xffffffffu ? kNone : tile_lo + weak;
}

// ---- fast decode: Ethernet (no tag) / IPv4 (IHL 5) or IPv6 (no extension) / TCP or UDP -------
// Branch-light: 17 aligned LDS words + v_alignbyte, static field offsets, status by selects.
// Returns 0xff when the frame is not of that shape (the caller then runs the general decode).
template <bool FIELDS>
__device__ __forceinline__ uint32_t decode_fast(const uint32_t *w, uint32_t rel, uint32_t n, FlowWords &f) {
  const uint32_t sh = rel & 3u;
  const uint32_t *p = w + (rel >> 2);
  uint32_t a[17];
  uint32_t prev = p[0];
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    const uint32_t nx = p[k + 1];
    a[k] = __builtin_amdgcn_alignbyte(nx, prev, sh);
    prev = nx;
  }
  auto byte = [&](int i) { return (a[i >> 2] >> (8 * (i & 3))) & 0xffu; };
  auto be16 = [&](int i) { return (byte(i) << 8) | byte(i + 1); };
  const uint32_t etype = be16(12), b0 = byte(14);
  const uint32_t proto4 = byte(23), nh = byte(20);
  const bool v4 = etype == 0x0800u && b0 == 0x45u && n >= 34u && (proto4 == 6u || proto4 == 17u);
  const bool v6 = etype == 0x86ddu && (b0 >> 4) == 6u && n >= 54u && (nh == 6u || nh == 17u);
  if (!(v4 || v6)) return 0xffu;
  const uint32_t n3 = n - 14u;
  const uint32_t length = v4 ? ((be16(16) - 20u) & 0xffffu) : be16(18);
  const uint32_t hl3 = v4 ? 20u : 40u;
  const uint32_t st3 = (n3 - hl3 < length) ? (v4 ? NPR_FLOW_L2_IPV4_INCOMPLETE : NPR_FLOW_L2_IPV6_INCOMPLETE)
                       : (!v4 && n3 - hl3 != length) ? (uint32_t)NPR_FLOW_L2_IPV6_REMAINDER : 0u;
  const uint32_t proto = v4 ? proto4 : nh;
  const uint32_t n4 = length;
  const uint32_t hv = v4 ? be16(46) : be16(66);
  const uint32_t ulen = v4 ? be16(38) : be16(58);
  const uint32_t thl = (hv >> 12) * 4u;
  const uint32_t off = v4 ? 0u : 3u;  // IPv6 leaves are 3 codes after the IPv4 ones
  uint32_t st4;
  if (proto == 6u)
    st4 = n4 < 14u ? NPR_FLOW_L3_IPV4_TCP_INCOMPLETE + off
          : (thl < 20u || thl > 60u) ? NPR_FLOW_L3_IPV4_TCP_FAILURE + off
          : n4 < thl ? NPR_FLOW_L3_IPV4_TCP_INCOMPLETE + off : 0u;
  else
    st4 = n4 < 8u ? NPR_FLOW_L3_IPV4_UDP_INCOMPLETE + off
          : (ulen < 8u || n4 - 8u < ulen - 8u) ? NPR_FLOW_L3_IPV4_UDP_INCOMPLETE + off
          : n4 != ulen ? (v4 ? (uint32_t)NPR_FLOW_L3_IPV4_UDP_REMAINDER : (uint32_t)NPR_FLOW_L3_IPV6_UDP_REMAINDER)
                       : 0u;
  const uint32_t st = st3 ? st3 : st4;
  if (FIELDS) {
    const uint32_t sp = v4 ? be16(34) : be16(54), dp = v4 ? be16(36) : be16(56);
    f.d[0] = v4 ? __builtin_amdgcn_alignbyte(a[7], a[6], 2) : 0u;  // src ip bytes 26..29
    f.d[1] = v4 ? __builtin_amdgcn_alignbyte(a[8], a[7], 2) : 0u;  // dst ip bytes 30..33
    f.d[2] = sp | (dp << 16);
    f.d[3] = a[1] & 0xffff0000u;  // vlan 0 | src mac 0..1
    f.d[4] = a[2];
    f.d[5] = a[0];
    f.d[6] = (a[1] & 0xffffu) | (((v6 ? NPR_FLOW_KIND_IPV6 : 0u) | (proto == 17u ? NPR_FLOW_KIND_UDP : 0u)) << 16);
  }
  return st;
}

// ---- raw look-back words, issued early and decoded late ------------------------------------
struct RawWin {
  uint64_t w[7];
};

// wave 1: the previous tile's group mates; wave 2: the groups before; others: a dummy word.
// Every wave issues the same 7 loads so none of them is conditional.
__device__ __forceinline__ void issue_window(const ParseParams &kp, uint32_t tp, bool has_prev, RawWin &r) {
  const int lane = (int)(threadIdx.x & 63u), wave = (int)(threadIdx.x >> 6);
  const uint32_t pg = tp / kGroup, pi = tp % kGroup;
  const int64_t k = (int64_t)tp - 1 - lane;
  const int64_t gg = (int64_t)pg - 1 - lane;
  const bool tile_lane = has_prev && wave == 1 && lane < (int)pi;
  const bool group_lane = has_prev && wave == 2 && gg >= 0;
  const TileSlot *ts = kp.slots + (group_lane ? gg * kGroup + kGroup - 1 : (tile_lane ? k : 0));
  const uint64_t *ext = group_lane ? kp.groups[gg].g : ts->a;
  r.w[0] = ld_agent(&ts->p[0]);
  r.w[1] = ld_agent(&ts->p[1]);
  r.w[2] = ld_agent(&ts->p[2]);
  r.w[3] = ld_agent(ext + 0);
  r.w[4] = ld_agent(ext + 1);
  r.w[5] = ld_agent(ext + 2);
  r.w[6] = ld_agent(group_lane ? ext + 3 : &ts->p[0]);
}
__device__ __forceinline__ LaneSeg decode_tile_lanes(const ParseParams &kp, int64_t k, bool inr, const RawWin &r) {
  LaneSeg L{};
  L.first = L.last = k;
  L.mism = -1;
  L.valid = true;
  if (!inr) return L;
  const uint32_t ep = kp.epoch;
  if (tagged(r.w[0], ep) && tagged(r.w[1], ep) && tagged(r.w[2], ep)) {
    L.present = L.anchor = true;
    L.exit = r.w[0] & kMask48; L.cnt = r.w[1] & kMask48; L.ok = r.w[2] & kMask48;
  } else if (tagged(r.w[3], ep) && tagged(r.w[4], ep) && tagged(r.w[5], ep)) {
    L.present = true;
    const uint64_t e1 = r.w[4] & kMask48, c = r.w[5] & kMask48;
    L.entry = e1 ? e1 - 1 : kNone;
    L.exit = r.w[3] & kMask48;
    L.cnt = c & 0xffffffull;
    L.ok = (c >> 24) & 0xffffffull;
  }
  return L;
}
__device__ __forceinline__ LaneSeg decode_group_lanes(const ParseParams &kp, int64_t gg, bool inr, const RawWin &r) {
  LaneSeg L{};
  L.first = gg * kGroup;
  L.last = gg * kGroup + kGroup - 1;
  L.mism = -1;
  L.valid = true;
  if (!inr) return L;
  const uint32_t ep = kp.epoch;
  if (tagged(r.w[0], ep) && tagged(r.w[1], ep) && tagged(r.w[2], ep)) {
    L.present = L.anchor = true;
    L.exit = r.w[0] & kMask48; L.cnt = r.w[1] & kMask48; L.ok = r.w[2] & kMask48;
  } else if (tagged(r.w[3], ep) && tagged(r.w[4], ep) && tagged(r.w[5], ep) && tagged(r.w[6], ep)) {
    L.present = true;
    const uint64_t e1 = r.w[4] & kMask48, w3 = r.w[6] & kMask48;
    L.entry = e1 ? e1 - 1 : kNone;
    L.exit = r.w[3] & kMask48;
    L.cnt = r.w[5] & kMask48;
    L.ok = w3 & ((1ull << 40) - 1);
    L.valid = (w3 >> 40) & 1ull;
    L.anchor = (w3 >> 41) & 1ull;
    L.mism = L.valid ? -1 : L.first + (int64_t)((w3 >> 42) & 63ull);
  }
  return L;
}

enum : uint32_t { kWinFail = 0, kWinResolved = 1, kWinAgg = 2, kWinEmpty = 3, kWinAnchored = 4 };

// one record of the tile -> status (+ flow words); fast shape first, general decoder otherwise
__device__ __forceinline__ uint32_t decode_rec(const ParseParams &kp, const uint32_t *data, uint64_t tile_lo,
                                               uint32_t rel, FlowWords &f) {
  const uint32_t incl = hdr(data, rel, 2, kp.big);
  uint32_t st = decode_fast<true>(data, rel + 16u, incl, f);
  if (st == 0xffu) {
    const uint64_t p = tile_lo + rel;
    TileReader r{data, (const uint8_t *)data, rel + 16u, kp.buf + p + 16, kp.len - p - 16};
    st = decode<true>(r, incl, f);
  }
  return st;
}

// Phase B: decode every record of the tile once: status -> pstat, Ok flows -> park (rank order).
// `direct` (slow path) writes the flows straight to their global positions instead.
__device__ uint32_t decode_tile(const ParseParams &kp, PipeShared &sh, uint64_t tile_lo, int slot, bool direct,
                                uint64_t pok) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t n = sh.n[slot];
  uint32_t base = 0;
  for (int s = 0; s < kSlots; ++s) {
    if ((uint32_t)s * kBlock >= n) break;  // uniform
    const uint32_t i = tid + (uint32_t)s * kBlock;
    FlowWords f;
    bool ok = false;
    uint64_t p = 0;
    if (i < n) {
      const uint32_t rel = sh.srec[slot][i];
      p = tile_lo + rel;
      const uint32_t st = decode_rec(kp, sh.data, tile_lo, rel, f);
      if (!direct) sh.pstat[i] = (uint8_t)st;
      else if (kp.rec_status && kp.pcnt_slow + i < kp.rec_cap) kp.rec_status[kp.pcnt_slow + i] = (uint8_t)st;
      ok = st == NPR_FLOW_OK;
    }
    const uint64_t bal = __ballot(ok);
    if (lane == 0) sh.scnt[s][wave] = (uint32_t)__builtin_popcountll(bal);
    __syncthreads();
    if (ok) {
      uint32_t rank = base + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      for (uint32_t v = 0; v < wave; ++v) rank += sh.scnt[s][v];
      const u32x4 lo4 = u32x4{f.d[0], f.d[1], f.d[2], f.d[3]};
      const u32x4 hi4 = u32x4{f.d[4], f.d[5], f.d[6] | ((uint32_t)(p & 0xffu) << 24), (uint32_t)(p >> 8)};
      if (!direct) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(&sh.park[rank * 8]);
        dst[0] = lo4;
        dst[1] = hi4;
      } else if (kp.flows && pok + rank < kp.flow_cap) {
        const uint64_t o = kp.flow_cap - 1 - (pok + rank);
        u32x4 *dst = reinterpret_cast<u32x4 *>(kp.flows + o * 8);
        dst[0] = lo4;
        dst[1] = hi4;
        if (kp.flows_v6 && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16))) {
          GlobalReader gr{kp.buf + p + 16, kp.len - p - 16};
          FlowWords g;
          decode<true>(gr, hdr(sh.data, (uint32_t)(p - tile_lo), 2, kp.big), g);
          u32x4 *d6 = reinterpret_cast<u32x4 *>(kp.flows_v6 + o * 8);
          d6[0] = u32x4{g.v6[0], g.v6[1], g.v6[2], g.v6[3]};
          d6[1] = u32x4{g.v6[4], g.v6[5], g.v6[6], g.v6[7]};
        }
      }
    }
    base += sh.scnt[s][0] + sh.scnt[s][1] + sh.scnt[s][2] + sh.scnt[s][3];
    __syncthreads();  // scnt is reused by the next slot
  }
  return base;
}

__device__ __forceinline__ void write_summary(const ParseParams &kp, uint64_t tot_rec, uint64_t tot_ok, uint64_t consumed) {
  uint32_t fl = 0;
  if ((kp.rec_off || kp.recs || kp.rec_status) && tot_rec > kp.rec_cap) fl |= NPR_SUMMARY_RECORD_OVERFLOW;
  if (kp.flows && tot_ok > kp.flow_cap) fl |= NPR_SUMMARY_FLOW_OVERFLOW;
  kp.summary->n_records = tot_rec;
  kp.summary->n_flows = tot_ok;
  kp.summary->consumed = consumed;
  kp.summary->flags = fl;
  kp.summary->epoch = kp.epoch;
}

// dense record rows [i0, n) of a tile (record offsets from srec)
__device__ __forceinline__ void write_records(const ParseParams &kp, const uint16_t *srec, uint32_t n,
                                              uint64_t tile_lo, uint64_t pcnt, const uint8_t *pstat,
                                              uint32_t i0, uint32_t step) {
  for (uint32_t i = i0; i < n; i += step) {
    const uint64_t idx = pcnt + i;
    if (idx >= kp.rec_cap) break;
    const uint64_t p = tile_lo + srec[i];
    if (kp.rec_off) kp.rec_off[idx] = p;
    if (kp.rec_status && pstat) kp.rec_status[idx] = pstat[i];
    if (kp.recs) {
      GlobalReader gr{kp.buf + p, kp.len - p};
      const uint32_t h0 = gr.le32(0), h1 = gr.le32(4), h2 = gr.le32(8), h3 = gr.le32(12);
      const bool big = kp.big;
      uint64_t *row = reinterpret_cast<uint64_t *>(kp.recs + idx);
      row[0] = p;
      row[1] = (uint64_t)(big ? __builtin_bswap32(h0) : h0) | ((uint64_t)(big ? __builtin_bswap32(h1) : h1) << 32);
      row[2] = (uint64_t)(big ? __builtin_bswap32(h2) : h2) | ((uint64_t)(big ? __builtin_bswap32(h3) : h3) << 32);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_parse_pipe(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) PipeShared sh;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  if (b >= kp.ntiles) return;
  const uint32_t nmine = (kp.ntiles - 1 - b) / G + 1;
  const uint32_t ep = kp.epoch;

  SpecCtx sc;
  sc.big = kp.big;
  sc.frac_max = kp.frac_max;
  sc.has_ref = false;
  sc.ts_ref = 0;
  if (kp.flags & kFlagMagicAtZero) {  // pcap magic: microsecond captures bound ts_usec < 1e6
    const uint32_t m = *reinterpret_cast<const uint32_t *>(kp.buf);
    if (m == 0xA1B2C3D4u || m == 0xD4C3B2A1u) sc.frac_max = 1000000u;
  }
  if (!(kp.flags & kFlagSpecFirst) && kp.len >= kp.start + 16) {  // the first record's ts_sec
    GlobalReader gr{kp.buf + kp.start, 4};
    const uint32_t v = gr.le32(0);
    sc.ts_ref = kp.big ? __builtin_bswap32(v) : v;
    sc.has_ref = true;
  }
  u32x4 q[kPrefetch];
  prefetch_tile(kp, b, q);
  commit_tile(sh.data, q);
  if (tid == 0) {
    sh.abort = 0;
    sh.l2_tag = 0xffffffffu;
  }
  __syncthreads();

  for (uint32_t k = 0; k <= nmine; ++k) {
    const bool has_cur = k < nmine, has_prev = k >= 1, has_next = k + 1 < nmine;
    const uint32_t t = b + k * G, tp = t - G;
    const int cur = (int)(k & 1u), prv = cur ^ 1;
    const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
    const uint64_t tile_hi = tile_lo + kTile < kp.len ? tile_lo + kTile : kp.len;
    const uint64_t ptile_lo = kp.org + (uint64_t)tp * kTile;
    if (kp.stamps && has_cur && tid == 0) kp.stamps[(uint64_t)t * 8 + 0] = __builtin_amdgcn_s_memrealtime();

    // (1) next tile -> registers;  (2) look-back words of the previous tile
    prefetch_tile(kp, has_next ? t + G : b, q, has_next);
    RawWin win;
    issue_window(kp, has_prev ? tp : 0u, has_prev, win);

    // ---- phase A ----------------------------------------------------------------------------
    if (wave == 0) {
      if (has_cur) {  // speculate + walk tile t
        const bool exact = t == 0 && !(kp.flags & kFlagSpecFirst);
        uint64_t entry = kp.start;
        if (!exact) {
          const uint64_t avail = kp.len - tile_lo;
          sc.avail = avail > 0xffffffffull ? 0xffffffffu : (uint32_t)avail;
          sc.exact_end = avail <= 0xffffffffull;
          const uint64_t lo = (t == 0) ? kp.start : tile_lo;
          entry = speculate_wave(sc, sh.data, tile_lo, (uint32_t)(lo - tile_lo), (uint32_t)(tile_hi - tile_lo));
        }
        if (kp.stamps && lane == 0) kp.stamps[(uint64_t)t * 8 + 4] = __builtin_amdgcn_s_memrealtime();
        uint32_t n = 0;
        uint64_t ex = entry;
        if (entry != kNone && entry >= tile_lo && entry < tile_hi)
          ex = walk_tile(kp, sh.data, sh.srec[cur], tile_lo, tile_hi, entry, n);
        else if (entry == kNone)
          ex = 0;
        if (lane == 0) {
          sh.n[cur] = n;
          sh.entry[cur] = entry;
          sh.exit[cur] = ex;
        }
        if (kp.stamps && lane == 0) kp.stamps[(uint64_t)t * 8 + 5] = __builtin_amdgcn_s_memrealtime();
      }
    } else if (wave == 2) {
      if (has_prev) {  // fold the group window for wave 1
        const uint32_t pg = tp / kGroup;
        uint32_t st = kWinEmpty;
        Seg c{};
        if (pg > 0) {
          const bool inr = (int64_t)pg - 1 - (int64_t)lane >= 0;
          const LaneSeg L = decode_group_lanes(kp, (int64_t)pg - 1 - lane, inr, win);
          const int nwin = pg < 64 ? (int)pg : 64;
          const uint64_t bAnc = __ballot(inr && L.anchor), bPres = __ballot(inr && L.present);
          const int jp = bAnc ? __builtin_ctzll(bAnc) : nwin;
          const uint64_t need = jp >= 64 ? ~0ull : ((1ull << jp) - 1ull);
          st = kWinFail;
          if (jp < nwin && (bPres & need) == need) {
            c = fold_window(kp, L, jp);
            st = kWinAnchored;
          }
        }
        if (lane == 0) {
          sh.l2 = c;
          sh.l2_state = st;
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the fold is in LDS before the tag
          __hip_atomic_store(&sh.l2_tag, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    } else if (wave == 1) {
      if (has_prev) {  // resolve tile tp, then write its outputs
        const uint32_t pi = tp % kGroup;
        uint32_t s1 = kWinEmpty;
        Seg l1{};
        if (pi > 0) {
          const bool inr = (int)lane < (int)pi;
          const LaneSeg L = decode_tile_lanes(kp, (int64_t)tp - 1 - lane, inr, win);
          const uint64_t bAnc = __ballot(inr && L.anchor), bPres = __ballot(inr && L.present);
          const int jp = bAnc ? __builtin_ctzll(bAnc) : (int)pi;
          const uint64_t need = (1ull << jp) - 1ull;
          s1 = kWinFail;
          if ((bPres & need) == need) {
            l1 = fold_window(kp, L, jp < (int)pi ? jp : (int)pi - 1);
            s1 = jp < (int)pi ? (l1.valid ? kWinResolved : kWinFail) : kWinAgg;
          }
        }
        Prefix pre{kp.start, 0, 0};
        bool ok = true;
        if (tp != 0) {
          bool done = false;
          if (s1 == kWinResolved) {
            pre = Prefix{l1.exit, l1.cnt, l1.ok};
            done = true;
          } else if (s1 == kWinAgg || s1 == kWinEmpty) {
            while (__hip_atomic_load(&sh.l2_tag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != k)
              __builtin_amdgcn_s_sleep(1);
            if (sh.l2_state == kWinAnchored) {
              const Seg c = s1 == kWinEmpty ? sh.l2 : combine(kp, sh.l2, l1);
              if (c.valid) {
                pre = Prefix{c.exit, c.cnt, c.ok};
                done = true;
              }
            }
          }
          if (!done) {  // not resolvable from the early words: the blocking look-back
            Diag dg;
            ok = lookback(kp, tp, pre, dg);
          }
        }
        const bool slow = ok && tp != 0 && pre.exit != sh.entry[prv];
        if (lane == 0) {
          sh.pexit = pre.exit;
          sh.pcnt = pre.cnt;
          sh.pok = pre.ok;
          sh.abort = ok ? 0u : 1u;
          sh.slow = slow ? 1u : 0u;
        }
        if (ok && !slow) {
          const uint32_t n = sh.n[prv], okc = sh.okc[prv];
          if (tp != 0 && lane == 0) {
            TileSlot *slot = kp.slots + tp;
            st_agent(&slot->p[0], gran(ep, sh.exit[prv]));
            st_agent(&slot->p[1], gran(ep, pre.cnt + n));
            st_agent(&slot->p[2], gran(ep, pre.ok + okc));
          }
          if (tp == kp.ntiles - 1 && lane == 0) write_summary(kp, pre.cnt + n, pre.ok + okc, sh.exit[prv]);
          if (kp.stamps && lane == 0) kp.stamps[(uint64_t)tp * 8 + 2] = __builtin_amdgcn_s_memrealtime();
          if (kp.rec_off || kp.recs || kp.rec_status)
            write_records(kp, sh.srec[prv], n, ptile_lo, pre.cnt, sh.pstat, lane, 64);
          if (kp.flows) {
            for (uint32_t r = lane; r < okc; r += 64) {
              const uint64_t fi = pre.ok + r;
              if (fi >= kp.flow_cap) break;
              const uint64_t o = kp.flow_cap - 1 - fi;  // convert_records pops from the end
              const u32x4 *src = reinterpret_cast<const u32x4 *>(&sh.park[r * 8]);
              const u32x4 a0 = src[0], a1 = src[1];
              u32x4 *dst = reinterpret_cast<u32x4 *>(kp.flows + o * 8);
              dst[0] = a0;
              dst[1] = a1;
              if (kp.flows_v6 && ((a1[2] >> 16) & NPR_FLOW_KIND_IPV6)) {  // IPv6: re-read the addresses
                const uint64_t p = ((uint64_t)a1[3] << 8) | (a1[2] >> 24);
                GlobalReader gh{kp.buf + p, kp.len - p};
                const uint32_t incl = kp.big ? __builtin_bswap32(gh.le32(8)) : gh.le32(8);
                GlobalReader gr{kp.buf + p + 16, kp.len - p - 16};
                FlowWords f;
                decode<true>(gr, incl, f);
                u32x4 *d6 = reinterpret_cast<u32x4 *>(kp.flows_v6 + o * 8);
                d6[0] = u32x4{f.v6[0], f.v6[1], f.v6[2], f.v6[3]};
                d6[1] = u32x4{f.v6[4], f.v6[5], f.v6[6], f.v6[7]};
              }
            }
          }
          if (kp.stamps && lane == 0) kp.stamps[(uint64_t)tp * 8 + 3] = __builtin_amdgcn_s_memrealtime();
        }
      }
    }
    __syncthreads();
    if (sh.abort) return;

    // ---- phase B: decode tile t once, publish its aggregate --------------------------------
    if (has_cur) {
      const uint32_t okc = decode_tile(kp, sh, tile_lo, cur, false, 0);
      if (tid == 0) {
        sh.okc[cur] = okc;
        TileSlot *slot = kp.slots + t;
        if (t == 0 && !(kp.flags & kFlagSpecFirst)) {
          st_agent(&slot->p[0], gran(ep, sh.exit[cur]));
          st_agent(&slot->p[1], gran(ep, sh.n[cur]));
          st_agent(&slot->p[2], gran(ep, okc));
        } else {
          st_agent(&slot->a[0], gran(ep, sh.exit[cur]));
          st_agent(&slot->a[1], gran(ep, sh.entry[cur] == kNone ? 0ull : sh.entry[cur] + 1));
          st_agent(&slot->a[2], gran(ep, (uint64_t)sh.n[cur] | ((uint64_t)okc << 24)));
        }
        if (kp.stamps) kp.stamps[(uint64_t)t * 8 + 1] = __builtin_amdgcn_s_memrealtime();
      }
    }

    // ---- slow path: tile tp speculated wrong -> reload it, redo from the exact entry --------
    if (sh.slow) {
      __syncthreads();  // everyone is done with tile t's data
      u32x4 r2[kPrefetch];
      prefetch_tile(kp, tp, r2);
      commit_tile(sh.data, r2);
      __syncthreads();
      const uint64_t ptile_hi = ptile_lo + kTile < kp.len ? ptile_lo + kTile : kp.len;
      const uint64_t e = sh.pexit;
      if (wave == 0) {
        uint32_t n = 0;
        uint64_t ex = e;
        if (e >= ptile_lo && e < ptile_hi) ex = walk_tile(kp, sh.data, sh.srec[prv], ptile_lo, ptile_hi, e, n);
        if (lane == 0) {
          sh.n[prv] = n;
          sh.exit[prv] = ex;
        }
      }
      __syncthreads();
      const uint32_t n = sh.n[prv];
      if (kp.rec_off || kp.recs)
        write_records(kp, sh.srec[prv], n, ptile_lo, sh.pcnt, nullptr, tid, kBlock);
      ParseParams kq = kp;
      kq.pcnt_slow = sh.pcnt;
      const uint32_t okc = decode_tile(kq, sh, ptile_lo, prv, true, sh.pok);
      if (tid == 0) {
        TileSlot *slot = kp.slots + tp;
        st_agent(&slot->p[0], gran(ep, sh.exit[prv]));
        st_agent(&slot->p[1], gran(ep, sh.pcnt + n));
        st_agent(&slot->p[2], gran(ep, sh.pok + okc));
        if (tp == kp.ntiles - 1) write_summary(kp, sh.pcnt + n, sh.pok + okc, sh.exit[prv]);
        sh.slow = 0;
      }
    }

    // (6) tile t+G: registers -> LDS (every wave is done with the buffer)
    __syncthreads();
    if (has_next) commit_tile(sh.data, q);
    // group aggregate of t's group (its last tile), for the next iteration's resolvers
    if (has_cur && t % kGroup == kGroup - 1 && wave == 3) {
      if (!publish_group(kp, t / kGroup) && lane == 0) sh.abort = 1u;
    }
    __syncthreads();
    if (sh.abort) return;
  }
}

hipError_t launch_parse_pipe(const ParseParams &p, uint32_t grid, hipStream_t s) {
  hipLaunchKernelGGL(k_parse_pipe, dim3(grid), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

int pipe_blocks_per_cu() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_parse_pipe, kBlock, 0) != hipSuccess) return 1;
  return n;
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
