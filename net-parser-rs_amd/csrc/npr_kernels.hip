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
// Design: two persistent passes of ONE-WAVE workgroups over 4 KiB tiles; each
// wave owns a contiguous run of tiles staged into its LDS ring by DMA (no workgroup barriers).
//   pass 1 (scan_chunk): the entry of a run's first tile is SPECULATED from header plausibility
//     (later tiles continue the wave's own chain); the wave walks the chain (stride speculation,
//     up to 256 records per step), decodes every record's status, and publishes the tile's
//     aggregate A = {entry, exit, records, Ok flows}; the last arrival of each 64-tile group
//     (and 4096-tile block) folds the group aggregates G1 (G2);
//   pass 2 (emit_chunk): the exact chain state before a run is start ⊕ G2 ⊕ G1 ⊕ A, folded
//     with a chain-consistency monoid (an aggregate counts only if its speculated entry is
//     where the chain really continues; a contradiction waits for the offending tile's exact
//     prefix P, which its own wave publishes here); then every tile is decoded again from the
//     exact position (reusing pass 1's record offsets when its entry was right) and its Ok
//     flows are written straight to their reverse-order (convert_records) rows.
// A wrong speculation costs a wait or a re-walk, never a wrong result.
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
// fast decode: Ethernet (untagged) / IPv4 (IHL 5) or IPv6 (no extension) / TCP or UDP.
// Branch-light: 17 aligned LDS words + v_alignbyte, static field offsets, status by selects;
// bit-identical to decode<> for these shapes.  Returns 0xff for any other frame (the caller then
// runs the general decode<>).
// ---------------------------------------------------------------------------------------------
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
  // pin the window in registers: otherwise the backend turns the IPv4/IPv6 selects below into
  // divergent branches that each load only their own words (select-to-branch on loads)
#pragma unroll
  for (int k = 0; k < 17; ++k) asm volatile("" : "+v"(a[k]));
  auto byte = [&](int i) { return (a[i >> 2] >> (8 * (i & 3))) & 0xffu; };
  auto be16 = [&](int i) { return (byte(i) << 8) | byte(i + 1); };
  // Every quantity is computed for every lane and combined by selects (no data-dependent
  // branches: divergent if/else here costs more scalar exec-mask work than the arithmetic).
  const uint32_t etype = be16(12), b0 = byte(14);
  const uint32_t proto4 = byte(23), nh = byte(20);
  const bool v4 = (etype == 0x0800u) & (b0 == 0x45u) & (n >= 34u) & ((proto4 == 6u) | (proto4 == 17u));
  const bool v6 = (etype == 0x86ddu) & ((b0 >> 4) == 6u) & (n >= 54u) & ((nh == 6u) | (nh == 17u));
  const uint32_t n3 = n - 14u;
  // IPv4 (IHL 5): wrapping u16 payload length; options/padding absent -> never a remainder
  const uint32_t length = v4 ? ((be16(16) - 20u) & 0xffffu) : be16(18);
  const uint32_t hl3 = v4 ? 20u : 40u;
  const bool l3_short = n3 - hl3 < length, l3_rem = !v4 & (n3 - hl3 != length);
  const uint32_t st3 = l3_short ? (v4 ? (uint32_t)NPR_FLOW_L2_IPV4_INCOMPLETE : (uint32_t)NPR_FLOW_L2_IPV6_INCOMPLETE)
                                : (l3_rem ? (uint32_t)NPR_FLOW_L2_IPV6_REMAINDER : 0u);
  const uint32_t proto = v4 ? proto4 : nh;
  const uint32_t n4 = length;
  const uint32_t hv = v4 ? be16(46) : be16(66);
  const uint32_t ulen = v4 ? be16(38) : be16(58);
  const uint32_t thl = (hv >> 12) * 4u;
  const uint32_t off = v4 ? 0u : 3u;  // the IPv6 TCP/UDP leaves are 3 codes after the IPv4 ones
  // TCP (src/layer4/tcp.rs:59-101): 14 bytes, data offset in [20, 60], then the whole header
  const bool t_short = n4 < 14u, t_bad = (thl < 20u) | (thl > 60u);
  const uint32_t st_tcp = t_short ? NPR_FLOW_L3_IPV4_TCP_INCOMPLETE + off
                        : (t_bad ? NPR_FLOW_L3_IPV4_TCP_FAILURE + off : (n4 < thl ? NPR_FLOW_L3_IPV4_TCP_INCOMPLETE + off : 0u));
  // UDP (src/layer4/udp.rs:33-50): OK iff 8 <= L == payload length
  const bool u_inc = (n4 < 8u) | (ulen < 8u) | (n4 - 8u < ulen - 8u);
  const uint32_t st_udp = u_inc ? NPR_FLOW_L3_IPV4_UDP_INCOMPLETE + off
                        : (n4 != ulen ? (v4 ? (uint32_t)NPR_FLOW_L3_IPV4_UDP_REMAINDER : (uint32_t)NPR_FLOW_L3_IPV6_UDP_REMAINDER) : 0u);
  const uint32_t st4 = proto == 6u ? st_tcp : st_udp;
  if (FIELDS) {
    const uint32_t sp = v4 ? be16(34) : be16(54), dp = v4 ? be16(36) : be16(56);
    f.d[0] = v4 ? __builtin_amdgcn_alignbyte(a[7], a[6], 2) : 0u;  // IPv4 src, bytes 26..29
    f.d[1] = v4 ? __builtin_amdgcn_alignbyte(a[8], a[7], 2) : 0u;  // IPv4 dst, bytes 30..33
    f.d[2] = sp | (dp << 16);
    f.d[3] = a[1] & 0xffff0000u;  // vlan 0 | src mac 0..1
    f.d[4] = a[2];
    f.d[5] = a[0];
    f.d[6] = (a[1] & 0xffffu) | ((((v6 ? NPR_FLOW_KIND_IPV6 : 0u) | (proto == 17u ? NPR_FLOW_KIND_UDP : 0u))) << 16);
#pragma unroll
    for (int k = 0; k < 8; ++k) f.v6[k] = __builtin_amdgcn_alignbyte(a[6 + k], a[5 + k], 2);  // bytes 22..53
  }
  return (v4 | v6) ? (st3 ? st3 : st4) : 0xffu;
}

// one record (header at LDS offset rel) -> status (+ flow words); fast shape first
template <bool FIELDS>
__device__ __forceinline__ uint32_t decode_rec(const ParseParams &kp, const uint32_t *w, uint64_t tile_lo,
                                               uint32_t rel, FlowWords &f, bool valid = true) {
  const uint32_t incl = hdr(w, rel, 2, kp.big);
  uint32_t st = decode_fast<FIELDS>(w, rel + 16u, incl, f);
  if (__ballot(valid && st == 0xffu)) {  // uniform test: most tiles never take the general path
    if (valid && st == 0xffu) {
      const uint64_t p = tile_lo + rel;
      TileReader r{w, (const uint8_t *)w, rel + 16u, kp.buf + p + 16, kp.len - p - 16};
      st = decode<FIELDS>(r, incl, f);
    }
  }
  return st;
}

// ---------------------------------------------------------------------------------------------
// hand-off granules (MI355X_MICROARCH.md "R2": the data IS the flag, {tag, value} 8-B)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t gran(uint32_t tag, uint64_t v) { return ((uint64_t)tag << 48) | (v & kMask48); }
__device__ __forceinline__ void st_agent(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool tagged(uint64_t w, uint32_t ep) { return (w >> 48) == ep; }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

// a value every lane holds identically, made visibly wave-uniform (scalar registers)
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)v);
}

// A segment of consecutive tiles [first, last] under speculation.
struct Seg {
  uint64_t entry, exit, cnt, ok;
  int64_t first, last, mism;  // mism: lowest tile whose speculated entry is contradicted
  bool valid;
};

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

// One lane's element of a 64-wide fold: a tile aggregate (level 0), a 64-tile group aggregate
// (level 1) or a 4096-tile block aggregate (level 2).
struct LaneSeg {
  uint64_t entry, exit, cnt, ok;
  int64_t first, last, mism;
  bool valid, present;
};

// level 0: A = {exit, entry + 1, n | okc << 24};  levels 1/2: {exit, entry + 1, cnt, ok | valid << 32 | mism_rel << 33}
__device__ __forceinline__ LaneSeg load_agg(const ParseParams &kp, int lvl, int64_t idx, bool inr) {
  LaneSeg L{};
  L.mism = -1;
  L.valid = true;
  const int sh = 6 * lvl;
  L.first = idx << sh;
  const int64_t last = ((idx + 1) << sh) - 1;
  L.last = last < (int64_t)kp.ntiles - 1 ? last : (int64_t)kp.ntiles - 1;
  if (!inr) return L;
  const uint32_t ep = kp.epoch;
  const uint64_t *w = lvl == 0 ? kp.slots[idx].a : (lvl == 1 ? kp.groups1[idx].g : kp.groups2[idx].g);
  const uint64_t w0 = ld_agent(w + 0), w1 = ld_agent(w + 1), w2 = ld_agent(w + 2);
  const uint64_t w3 = lvl == 0 ? w0 : ld_agent(w + 3);
  L.present = tagged(w0, ep) && tagged(w1, ep) && tagged(w2, ep) && tagged(w3, ep);
  const uint64_t e1 = w1 & kMask48;
  L.entry = e1 ? e1 - 1 : kNone;
  L.exit = w0 & kMask48;
  if (lvl == 0) {
    L.cnt = w2 & 0xffffffull;
    L.ok = (w2 >> 24) & 0xffffffull;
  } else {
    const uint64_t v3 = w3 & kMask48;
    L.cnt = w2 & kMask48;
    L.ok = v3 & 0xffffffffull;
    L.valid = (v3 >> 32) & 1ull;
    L.mism = L.valid ? -1 : L.first + (int64_t)((v3 >> 33) & 0x7fffull);
  }
  return L;
}

// lane i <- lane i+1 (DPP wave_shl:1, no LDS round trip); lane 63 gets 0
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x130, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x130, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
// whole-wave sum (DPP reduction of the device library); every lane must be active
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

// Fold lanes [lo .. 0] (ascending tile order = descending lane) into one segment.  Fast path:
// every link consistent, no END, no pass-through, all valid -> two wave sums; otherwise the
// serial monoid (wave-uniform, readlane).
__device__ Seg fold_window(const ParseParams &kp, const LaneSeg &L, int lo) {
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

__device__ __forceinline__ Seg start_seg(const ParseParams &kp) {
  Seg X;
  X.entry = X.exit = kp.start;
  X.cnt = X.ok = 0;
  X.first = X.last = -1;
  X.mism = -1;
  X.valid = true;
  return X;
}

// Generic exact prefix of tiles [a, t) continuing X (wave 0): ascending, largest aligned
// aggregates first; every contradiction is settled by the exact prefix of the offending tile.
__device__ bool prefix_generic(const ParseParams &kp, Seg X, int64_t a, int64_t t, Seg &out, uint64_t t0) {
  for (;;) {
    if (!X.valid) {
      const int64_t m = X.mism;
      if (!wait_exact(kp, m, X, t0)) return false;
      if (kp.stats && (threadIdx.x & 63u) == 0) atomicAdd(kp.stats + kStatMismWait, 1u);
      a = m + 1;
    }
    if (a >= t) break;
    int lvl;
    int64_t cnt;
    if ((a & 4095) == 0 && t - a >= 4096) {
      lvl = 2;
      cnt = (t - a) >> 12;
    } else if ((a & 63) == 0 && t - a >= 64) {
      lvl = 1;
      cnt = (t - a) >> 6;
      const int64_t to_blk = (4096 - (a & 4095)) >> 6;
      cnt = cnt < to_blk ? cnt : to_blk;
    } else {
      lvl = 0;
      cnt = t - a;
      const int64_t to_grp = 64 - (a & 63);
      cnt = cnt < to_grp ? cnt : to_grp;
    }
    cnt = cnt < 64 ? cnt : 64;
    Seg Y;
    if (!fold_range(kp, lvl, a >> (6 * lvl), (int)cnt, Y, t0)) return false;
    X = combine(kp, X, Y);
    a += cnt << (6 * lvl);
  }
  out = X;
  return true;
}

// ---------------------------------------------------------------------------------------------
// speculation (tile-relative 32-bit arithmetic) + chain walk
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kOrigMax = 1u << 18;       // plausible orig_len bound
constexpr uint32_t kTsRefWindow = 1u << 26;   // |ts_sec - the first record's ts_sec| (~2 years)

struct SpecCtx {
  uint32_t avail;    // bytes of the input from tile_lo, saturated to 32 bits
  bool exact_end;    // avail is exact: q == avail means "the chain ends exactly at EOF"
  uint32_t frac_max, ts_ref;
  bool has_ref, big;
};

__device__ __forceinline__ bool plaus(const SpecCtx &c, uint32_t ts, uint32_t frac, uint32_t incl, uint32_t orig) {
  return incl >= 1u && incl <= kInclMax && orig >= incl && orig <= kOrigMax && frac < c.frac_max &&
         (!c.has_ref || ts - c.ts_ref + kTsRefWindow <= 2u * kTsRefWindow);
}

// How plausible is LDS offset r as a record start?  0 = no; 1 = weak (its header passes but
// fewer than two chained headers could be checked inside the staged window); 2 = strong.
// A heuristic only: k_emit_tiles verifies every guess; a wrong one costs a wait, never a result.
__device__ __forceinline__ int grade(const SpecCtx &c, const uint32_t *w, uint32_t r) {
  if (c.avail - r < 16) return 0;
  uint32_t ts = hdr(w, r, 0, c.big);
  const uint32_t incl = hdr(w, r, 2, c.big);
  if (!plaus(c, ts, hdr(w, r, 1, c.big), incl, hdr(w, r, 3, c.big))) return 0;
  if (c.avail - r - 16 < incl) return 0;
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

// PcapRecords::parse loop (src/record.rs:30-49) over one tile, from `entry`, by one wave.
// Records whose header starts before tile_hi belong to this tile.  Returns the exit: the first
// chain offset >= tile_hi, or (chain END, Q3) the offset of the first incomplete record.
// Stride speculation: while the record length repeats, lane j confirms records j, j+64, j+128,
// j+192 ahead in one LDS round trip (up to 256 records per step); one record per step otherwise.
constexpr int kWalkUnroll = 4;
__device__ uint64_t walk_tile(const ParseParams &kp, const uint32_t *w, uint16_t *srec, uint64_t tile_lo,
                              uint64_t tile_hi, uint64_t entry, uint32_t &n_out) {
  const uint32_t lane = threadIdx.x & 63u;
  const bool big = kp.big;
  const uint32_t span = (uint32_t)(tile_hi - tile_lo);
  const uint64_t av = kp.len - tile_lo;
  const uint32_t avail = av > 0xffffffffull ? 0xffffffffu : (uint32_t)av;  // bytes from tile_lo
  uint64_t p = uni64(entry);
  uint32_t n = 0;
  while (p < tile_hi) {
    const uint32_t r = (uint32_t)(p - tile_lo);
    // wave-uniform (one address): readfirstlane keeps the chain position scalar
    const uint32_t incl = __builtin_amdgcn_readfirstlane(hdr(w, r, 2, big));
    if (kp.len - p < 16 || kp.len - p - 16 < incl) break;  // Err(Incomplete) -> stop (:37-45)
    if (incl > (uint32_t)kTile) {  // a record longer than a tile: no stride to speculate on
      if (lane == 0) srec[n] = (uint16_t)r;
      n += 1;
      p += 16ull + incl;
      continue;
    }
    const uint32_t stride = 16u + incl;
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
    p += (uint64_t)m * stride;
  }
  n_out = n;
  return p;
}

// diagnostics (DIAG kernel variants only: the production kernels carry none of this)
template <bool DIAG>
__device__ __forceinline__ void stamp(const ParseParams &kp, uint32_t t, int k) {
  if (DIAG && kp.stamps && (threadIdx.x & 63u) == 0) kp.stamps[(uint64_t)t * kStampWords + k] = __builtin_amdgcn_s_memrealtime();
}

// LDS written by some lanes of this wave, then read by others: LDS executes one wave's requests
// in order, so only the compiler must not move the accesses across this point.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

typedef unsigned int u32x4 __attribute__((__vector_size__(16)));
// speculation context of this launch: ts_usec bound from the file magic, the first record's
// ts_sec as a reference (both read once per wave)
__device__ __forceinline__ SpecCtx spec_ctx(const ParseParams &kp) {
  SpecCtx sc;
  sc.big = kp.big;
  sc.frac_max = kp.frac_max;
  if (kp.flags & kFlagMagicAtZero) {  // microsecond pcap magic: ts_usec < 1e6
    GlobalReader gm{kp.buf, 4};
    const uint32_t m = gm.le32(0);
    if (m == 0xA1B2C3D4u || m == 0xD4C3B2A1u) sc.frac_max = 1000000u;
  }
  sc.has_ref = kp.ref != kNone && kp.len >= kp.ref + 16;
  GlobalReader gr{kp.buf + (sc.has_ref ? kp.ref : 0ull), sc.has_ref ? 4ull : 0ull};
  const uint32_t v = gr.le32(0);
  sc.ts_ref = __builtin_amdgcn_readfirstlane(kp.big ? __builtin_bswap32(v) : v);
  sc.frac_max = __builtin_amdgcn_readfirstlane(sc.frac_max);
  sc.avail = 0;
  sc.exact_end = true;
  return sc;
}

// first strong (else first weak) record-start candidate in [0, span) of the staged tile, 64
// candidates per round; kNone if neither (wave-uniform)
__device__ uint64_t speculate(SpecCtx sc, const ParseParams &kp, const uint32_t *w, uint64_t tile_lo, uint32_t lo,
                              uint32_t span) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t avail = kp.len - tile_lo;
  sc.avail = avail > 0xffffffffull ? 0xffffffffu : (uint32_t)avail;
  sc.exact_end = avail <= 0xffffffffull;
  uint32_t weak = 0xffffffffu;
  for (uint32_t base = lo; base < span; base += 64) {
    const uint32_t r = base + lane;
    const int g = r < span ? grade(sc, w, r) : 0;
    const uint64_t b2 = __ballot(g == 2);
    if (b2) return tile_lo + base + (uint32_t)__builtin_ctzll(b2);
    const uint64_t b1 = __ballot(g == 1);
    if (weak == 0xffffffffu && b1) weak = base + (uint32_t)__builtin_ctzll(b1);
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

// ---- LDS-DMA staging ring (per wave) -------------------------------------------------------
// Tiles land in LDS straight from HBM (`buffer_load_dwordx4 ... lds`, 1 KiB per instruction,
// range-checked: bytes past the input read 0) with no registers held in flight.  The next
// tile's DMA is issued before the wait for the current one, so the youngest vector-memory
// instructions at the wait are exactly the next tiles' DMAs: `s_waitcnt vmcnt(k * per-tile)`
// retires the current tile and nothing later, whatever stores came before.
#ifndef NPR_RING
#define NPR_RING 2
#endif
constexpr int kRing = NPR_RING;       // tiles staged per wave (1 processed + kRing-1 in flight)
constexpr int kRows = kTile / 1024;   // 1-KiB rows of a tile (16-B DMA), then one 256-B halo row (4-B DMA)
constexpr int kSlotWords = kTile / 4 + 64;
constexpr int kDmaScan = kRows + 1;   // DMA instructions per tile, pass 1
constexpr int kDmaEmit = kRows + 4;   // + 2 record-offset rows + 1 aggregate row, pass 2
static_assert(kTile % 1024 == 0 && kHalo <= 256 - 80, "halo row must hold the halo + the decode over-read");
typedef __attribute__((address_space(3))) void *lds_ptr_t;

__device__ __forceinline__ void dma_tile(const ParseParams &kp, uint64_t tile_lo, uint32_t *dst) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t avail = kp.len > tile_lo ? kp.len - tile_lo : 0;
  const uint32_t nbytes = avail < (uint64_t)kStage ? (uint32_t)avail : (uint32_t)kStage;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(kp.buf + tile_lo), 0, (int)((nbytes + 15u) & ~15u), 0x00020000);
#pragma unroll
  for (int i = 0; i < kRows; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + i * 256), 16, (lane + 64u * (uint32_t)i) * 16u, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + kRows * 256), 4, (uint32_t)kTile + lane * 4u, 0, 0, 0);
}
// pass 2 extras: pass 1's record-offset pairs of tile t and its A granules (dwords 0..5), sc1
__device__ __forceinline__ void dma_extras(const ParseParams &kp, uint32_t t, uint32_t *off, uint32_t *agg) {
  const uint32_t lane = threadIdx.x & 63u;
  const __amdgpu_buffer_rsrc_t ro =  // light mode has no offset scratch: an empty range reads nothing
      __builtin_amdgcn_make_buffer_rsrc(kp.srec_g ? (void *)(kp.srec_g + (uint64_t)t * kMaxRec) : (void *)kp.slots, 0,
                                        kp.srec_g ? kMaxRec * 2 : 0, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, (lds_ptr_t)off, 4, lane * 4u, 0, 0, 16);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(ro, (lds_ptr_t)(off + 64), 4, lane * 4u + 256u, 0, 0, 16);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void *)(kp.slots + t), 0, 24, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)agg, 4, lane * 4u, 0, 0, 16);
}
// wait until at most `ahead` tiles' DMAs (of `per` instructions each) are outstanding
template <int PER>
__device__ __forceinline__ void wait_dma(uint32_t ahead) {
  constexpr int w1 = PER, w2 = 2 * PER;
  static_assert(2 * PER < 64, "vmcnt field is 6 bits");
  if (ahead == 0) __builtin_amdgcn_s_waitcnt(0x0F70);
  else if (ahead == 1 || kRing <= 2) __builtin_amdgcn_s_waitcnt(0x0F70 | (w1 & 15) | ((w1 >> 4) << 14));
  else __builtin_amdgcn_s_waitcnt(0x0F70 | (w2 & 15) | ((w2 >> 4) << 14));
  wave_sync();  // LDS reads of the landed tile stay below the wait
}

struct ParseShared {  // one wave's LDS
  uint32_t data[kRing][kSlotWords];     // tile + 256-B halo row (>= kStage bytes + the decoder's 72-B over-read)
  uint32_t off[kRing][kMaxRec / 2];     // pass 2: pass 1's record-offset pairs (DMA)
  uint32_t agg[kRing][64];              // pass 2: the tile's A granules (DMA, dwords 0..5)
  uint16_t srec[2 * kMaxRec];           // record offsets (+ room for the walk's unconditional stores)
};

__device__ __forceinline__ void publish_fold(const ParseParams &kp, GroupSlot *G, const Seg &c, int64_t first) {
  const uint32_t ep = kp.epoch;
  const uint64_t mrel = c.valid ? 0ull : (uint64_t)(c.mism - first) & 0x7fffull;
  st_agent(&G->g[0], gran(ep, c.exit));
  st_agent(&G->g[1], gran(ep, c.entry == kNone ? 0ull : c.entry + 1));
  st_agent(&G->g[2], gran(ep, c.cnt));
  st_agent(&G->g[3], gran(ep, (c.ok & 0xffffffffull) | ((uint64_t)c.valid << 32) | (mrel << 33)));
}

// contiguous tile range [c0, c1) of worker w out of W (balanced)
__device__ __forceinline__ void chunk_of(uint32_t nt, uint32_t w, uint32_t W, uint32_t &c0, uint32_t &c1) {
  c0 = (uint32_t)((uint64_t)w * nt / W);
  c1 = (uint32_t)((uint64_t)(w + 1) * nt / W);
}

__device__ __forceinline__ uint32_t group_size(const ParseParams &kp, uint32_t g) {
  return kp.ntiles - (g << 6) < 64u ? kp.ntiles - (g << 6) : 64u;
}

// group g's last arriver: G1(g), and when g is the last group of block h to finish, G2(h)
__device__ __forceinline__ void fold_groups(const ParseParams &kp, uint32_t g) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  Seg c;
  if (!fold_range(kp, 0, (int64_t)g << 6, (int)group_size(kp, g), c, t0)) return;
  uint32_t last2 = 0;
  const uint32_t h = g >> 6;
  const uint32_t hsize = kp.ngroups1 - (h << 6) < 64u ? kp.ngroups1 - (h << 6) : 64u;
  if (lane == 0) {
    publish_fold(kp, kp.groups1 + g, c, (int64_t)g << 6);
    __hip_atomic_store(kp.cnt1 + 2 * g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last2 = __hip_atomic_fetch_add(kp.cnt2 + 2 * h, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == hsize - 1u;
  }
  if (__builtin_amdgcn_readfirstlane(last2) && fold_range(kp, 1, (int64_t)h << 6, (int)hsize, c, t0) && lane == 0) {
    publish_fold(kp, kp.groups2 + h, c, (int64_t)h << 12);
    __hip_atomic_store(kp.cnt2 + 2 * h, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------------------------
// pass 1: scan_chunk — ONE WAVE owns the contiguous tiles [c0, c1) and never waits on another
// wave (no workgroup barriers anywhere).  Per tile: (the next tile -> LDS by DMA) | entry = the
// previous tile's exit while the chain continues, else a speculated start | walk -> record
// offsets, also kept in the offset scratch for pass 2 | status-only decode -> Ok count (light
// mode: decode with fields, Ok flows parked) | publish A = {entry, exit, n, Ok count}.  At the
// end of the chunk the wave arrives once at each 64-tile group it touched: the arrival that
// completes a group folds its G1, and the group that completes a 4096-tile block folds G2.
// ---------------------------------------------------------------------------------------------
template <bool DIAG, bool LIGHT>
__device__ __forceinline__ void scan_chunk(const ParseParams &kp, ParseShared &sh, uint32_t c0, uint32_t c1) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int k = 0; k < kRing - 1; ++k)
    if (c0 + k < c1) dma_tile(kp, kp.org + (uint64_t)(c0 + k) * kTile, sh.data[k]);
  const SpecCtx sc = spec_ctx(kp);
  uint64_t carry = kNone;  // exact continuation of the chain
  uint64_t chunk_ok = 0;   // light mode: Ok flows parked so far in this chunk
  for (uint32_t t = c0; t < c1; ++t) {
    const uint32_t slot = (t - c0) % kRing;
    const uint32_t *w = sh.data[slot];
    const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
    const uint64_t tile_hi = tile_lo + kTile < kp.stop ? tile_lo + kTile : kp.stop;
    stamp<DIAG>(kp, t, 0);
    // refill the slot processed last iteration with the tile kRing-1 ahead, then wait for this one
    const uint32_t ahead = c1 - 1 - t < (uint32_t)(kRing - 1) ? c1 - 1 - t : (uint32_t)(kRing - 1);
    if (t + kRing - 1 < c1) dma_tile(kp, tile_lo + (uint64_t)(kRing - 1) * kTile, sh.data[(slot + kRing - 1) % kRing]);
    wait_dma<kDmaScan>(ahead);

    uint64_t entry = carry;
    const bool spec0 = (kp.flags & kFlagSpecStart) != 0;
    if (t == 0 && !spec0) {
      entry = kp.start;
    } else if (carry == kNone) {
      const uint32_t lo = t == 0 ? (uint32_t)(kp.start - tile_lo) : 0u;  // a range starts at `start`
      entry = tile_hi > tile_lo + lo ? speculate(sc, kp, w, tile_lo, lo, (uint32_t)(tile_hi - tile_lo)) : kNone;
      if (DIAG && kp.stats && lane == 0 && entry == kNone) atomicAdd(kp.stats + kStatNoEntry, 1u);
    }
    stamp<DIAG>(kp, t, 1);
    entry = uni64(entry);
    uint32_t n = 0;
    uint64_t ex = entry == kNone ? 0ull : entry;
    if (entry != kNone && entry >= tile_lo && entry < tile_hi) ex = walk_tile(kp, w, sh.srec, tile_lo, tile_hi, entry, n);
    ex = uni64(ex);
    wave_sync();
    stamp<DIAG>(kp, t, 2);

    // ---- full mode: offsets -> scratch (pairs of u16) + Ok count (status-only decode);
    //      light mode: decode with fields, Ok flows parked in tile order
    if (!LIGHT && kp.srec_g) {  // (n + 1) / 2 offset pairs; the descriptor's range drops the rest
      const uint32_t *src = reinterpret_cast<const uint32_t *>(sh.srec);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)(kp.srec_g + (uint64_t)t * kMaxRec), 0, (int)(((n + 1) / 2) * 4u), 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(src[lane], rs, (int)(lane * 4u), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(src[lane + 64], rs, (int)(lane * 4u + 256u), 0, 0);
    }
    uint32_t okc = 0;
    for (int s = 0; s < kRounds; ++s) {
      if ((uint32_t)s * 64u >= n) break;
      const uint32_t i = lane + (uint32_t)s * 64u;
      const bool valid = i < n;  // every lane decodes (stale offsets are in-bounds), masked after
      FlowWords f;
      const uint32_t rel = sh.srec[i];
      const bool ok = decode_rec<LIGHT>(kp, w, tile_lo, rel, f, valid) == NPR_FLOW_OK && valid;
      const uint64_t bal = __ballot(ok);
      if (LIGHT && ok) {  // parked contiguously per chunk, in chain order (<= kMaxOk per tile)
        const uint64_t row = ((uint64_t)c0 * kMaxOk + chunk_ok + okc + (uint32_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull))) * 8;
        put_flow(kp.park + row, f, tile_lo + rel);
        if (kp.park_v6 && (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16))) put_v6(kp.park_v6 + row, f);
      }
      okc += (uint32_t)__builtin_popcountll(bal);
    }
    stamp<DIAG>(kp, t, 3);
    if (lane == 0) {
      TileSlot *slot_t = kp.slots + t;
      const uint32_t ep = kp.epoch;
      st_agent(&slot_t->a[0], gran(ep, ex));
      st_agent(&slot_t->a[1], gran(ep, entry == kNone ? 0ull : entry + 1));
      st_agent(&slot_t->a[2], gran(ep, (uint64_t)n | ((uint64_t)okc << 24)));
    }
    // the chain continues into the next tile unless it ended here (Q3) or nothing was found
    carry = uni64((entry != kNone && ex >= tile_hi) ? ex : kNone);
    chunk_ok += okc;
    stamp<DIAG>(kp, t, 4);
    wave_sync();  // done with this slot's LDS before it is refilled
  }
  // arrive at the chunk's groups (one add per group; the add that completes a group folds it)
  stamp<DIAG>(kp, c0, 11);
  for (uint32_t g = c0 >> 6; g <= (c1 - 1) >> 6; ++g) {
    const uint32_t lo = c0 > (g << 6) ? c0 : (g << 6), hi = c1 < ((g + 1) << 6) ? c1 : ((g + 1) << 6);
    uint32_t last = 0;
    if (lane == 0)
      last = __hip_atomic_fetch_add(kp.cnt1 + 2 * g, hi - lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (hi - lo) ==
             group_size(kp, g);
    if (__builtin_amdgcn_readfirstlane(last)) fold_groups(kp, g);
  }
  stamp<DIAG>(kp, c0, 12);
}

// ---------------------------------------------------------------------------------------------
// pass 2: emit_chunk — ONE WAVE owns the contiguous tiles [c0, c1).
//   exact prefix before c0 = start ⊕ G2(blocks) ⊕ G1(groups) ⊕ A(tiles): the three 64-wide
//   windows are loaded together, then folded; a contradiction (a mis-speculated tile m < c0)
//   is settled by m's exact prefix P(m), published below by m's owner.  Then per tile,
//   carrying the exact chain position and counts: (the next tile, its A granules and pass 1's
//   record offsets -> LDS by DMA) | the offsets: pass 1's when its entry equals the exact
//   position (the common case), else a walk | decode every record | record table / status |
//   Ok flows at their convert_records (reverse-order) positions, ranked by ballot | publish P(t).
// ---------------------------------------------------------------------------------------------
// The chain's anchor: `start`, or with kFlagSpecStart the entry pass 1 speculated for tile 0
// (none found: the range yields nothing and reports NPR_NO_ENTRY; the chain passes `stop`).
__device__ bool anchor_of(const ParseParams &kp, Seg &X, uint64_t &entry0, uint64_t t0) {
  X = start_seg(kp);
  entry0 = kp.start;
  if (!(kp.flags & kFlagSpecStart)) return true;
  for (;;) {
    const uint64_t a1 = uni64(ld_agent(&kp.slots[0].a[1]));
    if (tagged(a1, kp.epoch)) {
      const uint64_t e1 = a1 & kMask48;
      entry0 = e1 ? e1 - 1 : kNone;
      X.entry = X.exit = e1 ? e1 - 1 : kp.stop;
      return true;
    }
    if (!spin_ok(kp, t0)) return false;
  }
}

// exact chain state before tile c: false when a hand-off timed out
__device__ bool prefix_of(const ParseParams &kp, uint32_t c, Seg &X, uint64_t &entry0) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if (!anchor_of(kp, X, entry0, t0)) return false;
  const int64_t h = c >> 12, g = c >> 6;
  if (h > 64) return prefix_generic(kp, X, 0, c, X, t0);  // > 1 GiB before c: the generic walker
  const int n2 = (int)h, n1 = (int)(g - (h << 6)), n0 = (int)((int64_t)c - (g << 6));
  // all three windows in flight at once
  const LaneSeg L2 = load_agg(kp, 2, h - 1 - lane, (int)lane < n2);
  const LaneSeg L1 = load_agg(kp, 1, g - 1 - lane, (int)lane < n1);
  const LaneSeg L0 = load_agg(kp, 0, (int64_t)c - 1 - lane, (int)lane < n0);
  const bool all = __ballot(((int)lane < n2 && !L2.present) || ((int)lane < n1 && !L1.present) ||
                            ((int)lane < n0 && !L0.present)) == 0ull;
  Seg y;
  if (all) {
    if (n2) X = combine(kp, X, fold_window(kp, L2, n2 - 1));
    if (n1) X = combine(kp, X, fold_window(kp, L1, n1 - 1));
    if (n0) X = combine(kp, X, fold_window(kp, L0, n0 - 1));
  } else {  // not all published yet (fused launch): fold each window as it completes
    if (n2) {
      if (!fold_range(kp, 2, 0, n2, y, t0)) return false;
      X = combine(kp, X, y);
    }
    if (n1) {
      if (!fold_range(kp, 1, h << 6, n1, y, t0)) return false;
      X = combine(kp, X, y);
    }
    if (n0) {
      if (!fold_range(kp, 0, g << 6, n0, y, t0)) return false;
      X = combine(kp, X, y);
    }
  }
  if (!X.valid) return prefix_generic(kp, X, 0, c, X, t0);
  return true;
}

__device__ __forceinline__ void emit_prologue(const ParseParams &kp, ParseShared &sh, uint32_t c0, uint32_t c1) {
#pragma unroll
  for (int k = 0; k < kRing - 1; ++k)
    if (c0 + k < c1) {
      dma_tile(kp, kp.org + (uint64_t)(c0 + k) * kTile, sh.data[k]);
      dma_extras(kp, c0 + k, sh.off[k], sh.agg[k]);
    }
}

// Tiles [c0, c1) from the exact chain state (pos, pcnt, pok); emit_prologue has been issued.
template <bool DIAG>
__device__ void emit_tiles(const ParseParams &kp, ParseShared &sh, uint32_t c0, uint32_t c1, uint64_t pos,
                           uint64_t pcnt, uint64_t pok, uint64_t entry0) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t t = c0; t < c1; ++t) {
    const uint32_t slot = (t - c0) % kRing;
    const uint32_t *w = sh.data[slot];
    const uint64_t tile_lo = kp.org + (uint64_t)t * kTile;
    const uint64_t tile_hi = tile_lo + kTile < kp.stop ? tile_lo + kTile : kp.stop;
    stamp<DIAG>(kp, t, 5);
    const uint32_t ahead = c1 - 1 - t < (uint32_t)(kRing - 1) ? c1 - 1 - t : (uint32_t)(kRing - 1);
    if (t + kRing - 1 < c1) {
      const uint32_t ns = (slot + kRing - 1) % kRing;
      dma_tile(kp, tile_lo + (uint64_t)(kRing - 1) * kTile, sh.data[ns]);
      dma_extras(kp, t + kRing - 1, sh.off[ns], sh.agg[ns]);
    }
    wait_dma<kDmaEmit>(ahead);
    const uint32_t *ag = sh.agg[slot];
    const uint64_t a1 = uni64((uint64_t)ag[2] | ((uint64_t)ag[3] << 32));
    const uint64_t a2 = uni64((uint64_t)ag[4] | ((uint64_t)ag[5] << 32));
    const bool reuse = kp.srec_g && tagged(a1, kp.epoch) && tagged(a2, kp.epoch) && (a1 & kMask48) == pos + 1;
    // the record offsets: pass 1's (same exact entry) or a walk from the exact position
    const uint16_t *srec = reuse ? reinterpret_cast<const uint16_t *>(sh.off[slot]) : sh.srec;
    uint32_t n = 0;
    uint64_t ex = pos;
    if (pos >= tile_lo && pos < tile_hi) {
      if (reuse) {
        n = (uint32_t)(a2 & 0xffffffull);
        if (n) {  // exit = just past the last record (the walk advances by whole records)
          const uint32_t rl = __builtin_amdgcn_readfirstlane(srec[n - 1]);
          ex = tile_lo + rl + 16u + __builtin_amdgcn_readfirstlane(hdr(w, rl, 2, kp.big));
        }
      } else {
        ex = walk_tile(kp, w, sh.srec, tile_lo, tile_hi, pos, n);
        wave_sync();
        if (DIAG && kp.stats && lane == 0) atomicAdd(kp.stats + kStatRewalk, 1u);
      }
    }
    stamp<DIAG>(kp, t, 6);

    // ---- decode, record table, Ok flows at reverse positions (rank = ballot prefix)
    uint32_t okbase = 0;
    for (int s = 0; s < kRounds; ++s) {
      if ((uint32_t)s * 64u >= n) break;
      const uint32_t i = lane + (uint32_t)s * 64u;
      const bool valid = i < n;  // every lane decodes (stale offsets are in-bounds), masked after
      FlowWords f;
      const uint32_t rel = srec[i];
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
    pos = uni64(ex);
    pcnt += n;
    pok += okbase;
    if (lane == 0) {
      const uint32_t ep = kp.epoch;
      TileSlot *slot_t = kp.slots + t;
      st_agent(&slot_t->p[0], gran(ep, pos));
      st_agent(&slot_t->p[1], gran(ep, pcnt));
      st_agent(&slot_t->p[2], gran(ep, pok));
      if (t == kp.ntiles - 1) {
        uint32_t fl = 0;
        if ((kp.rec_off || kp.recs || kp.rec_status) && pcnt > kp.rec_cap) fl |= NPR_SUMMARY_RECORD_OVERFLOW;
        if (kp.flows && pok > kp.flow_cap) fl |= NPR_SUMMARY_FLOW_OVERFLOW;
        kp.summary->n_records = pcnt;
        kp.summary->n_flows = pok;
        kp.summary->consumed = pos;
        kp.summary->flags = fl;
        kp.summary->entry = entry0;
        kp.summary->epoch = kp.epoch;
      }
    }
    stamp<DIAG>(kp, t, 7);
    wave_sync();  // done with this slot's LDS before it is refilled
  }
}

template <bool DIAG>
__device__ __forceinline__ void emit_chunk(const ParseParams &kp, ParseShared &sh, uint32_t c0, uint32_t c1) {
  stamp<DIAG>(kp, c0, 8);
  emit_prologue(kp, sh, c0, c1);
  Seg X;
  uint64_t entry0;
  stamp<DIAG>(kp, c0, 9);
  if (!prefix_of(kp, c0, X, entry0)) return;
  stamp<DIAG>(kp, c0, 10);
  emit_tiles<DIAG>(kp, sh, c0, c1, uni64(X.exit), uni64(X.cnt), uni64(X.ok), entry0);
}

// ---------------------------------------------------------------------------------------------
// pass 2, light mode (flows only): emit_light_chunk — ONE WAVE owns the tiles [c0, c1).
//   Pass 1 parked the chunk's Ok flows contiguously in chain order.  When the chunk's first tile
//   started at the exact chain position (the norm), the whole chunk is exact up to a chain END,
//   so pass 2 is: the exact prefix, the chunk's counts summed up to that END, and ONE contiguous
//   reversed copy of the parked rows into convert_records order — no staging, walk or decode.
//   A chunk that started elsewhere runs the full per-tile path (emit_tiles), which also
//   publishes the exact prefixes P(t) a waiting fold may need.
// ---------------------------------------------------------------------------------------------
template <bool DIAG>
__device__ __forceinline__ void emit_light_chunk(const ParseParams &kp, ParseShared &sh, uint32_t c0, uint32_t c1) {
  const uint32_t lane = threadIdx.x & 63u;
  Seg X;
  uint64_t entry0;
  stamp<DIAG>(kp, c0, 8);
  stamp<DIAG>(kp, c0, 9);
  if (!prefix_of(kp, c0, X, entry0)) return;
  stamp<DIAG>(kp, c0, 10);
  const uint64_t pos = uni64(X.exit), pcnt = uni64(X.cnt), pok = uni64(X.ok);
  const uint64_t lo0 = kp.org + (uint64_t)c0 * kTile;
  bool valid = pos < lo0;  // the chain ended before this chunk: nothing here
  uint64_t n = 0, k = 0, ex = pos;
  if (!valid) {
    bool live = true;  // the chunk's chain has not ended yet
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t b = c0; b < c1 && live; b += 64) {
      const uint32_t cnt = c1 - b < 64u ? c1 - b : 64u;
      uint64_t w0 = 0, w1 = 0, w2 = 0;
      for (;;) {  // the chunk's own aggregates (pass 1 published them before this point)
        if (lane < cnt) {
          w0 = ld_agent(&kp.slots[b + lane].a[0]);
          w1 = ld_agent(&kp.slots[b + lane].a[1]);
          w2 = ld_agent(&kp.slots[b + lane].a[2]);
        }
        const bool ok = lane >= cnt || (tagged(w0, kp.epoch) && tagged(w1, kp.epoch) && tagged(w2, kp.epoch));
        if (__ballot(!ok) == 0ull) break;
        if (!spin_ok(kp, t0)) return;
      }
      if (b == c0) valid = (rl64(w1, 0) & kMask48) == pos + 1;  // the chunk started at the exact position
      if (!valid) break;
      for (uint32_t j = 0; j < cnt; ++j) {  // uniform: sum up to (and including) a chain END
        const uint64_t e = rl64(w0, (int)j) & kMask48, c = rl64(w2, (int)j) & kMask48;
        n += c & 0xffffffull;
        k += (c >> 24) & 0xffffffull;
        ex = e;
        if (e < tile_end(kp, (int64_t)(b + j))) {  // END (Q3): the rest of the capture is void
          live = false;
          break;
        }
      }
    }
  }
  if (!valid) {  // mis-speculated run: decode it here from the exact position
    if (DIAG && kp.stats && lane == 0) atomicAdd(kp.stats + kStatRewalk, 1u);
    emit_prologue(kp, sh, c0, c1);
    emit_tiles<DIAG>(kp, sh, c0, c1, pos, pcnt, pok, entry0);
    return;
  }
  stamp<DIAG>(kp, c0, 11);
  // ONE contiguous copy: parked row j -> flow row flow_cap-1-(pok+j) (convert_records order).
  // Range-checked buffer accesses (rows past flow_cap are out of range: nothing written).  A plain
  // two-loads-in-flight loop: the parked rows were just written by pass 1 and are still in L2 /
  // MALL; deeper batching (4 rows per lane) measured 3x slower here (r21 A/B) — it thrashes them.
  if (kp.flows && k) {
    const uint64_t base = (uint64_t)c0 * kMaxOk;
    const uint64_t kk = pok >= kp.flow_cap ? 0 : (k < kp.flow_cap - pok ? k : kp.flow_cap - pok);  // rows that fit
    const __amdgpu_buffer_rsrc_t src = __builtin_amdgcn_make_buffer_rsrc((void *)(kp.park + base * 8), 0, (int)(kk * 32), 0x00020000);
    // destination rows [flow_cap-pok-kk, flow_cap-pok): row j lands at (kk-1-j) in this window
    const __amdgpu_buffer_rsrc_t dst = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(kp.flows + (kp.flow_cap - pok - kk) * 8), 0, (int)(kk * 32), 0x00020000);
    for (uint64_t j = lane; j < kk; j += 64) {
      const u32x4 x0 = __builtin_amdgcn_raw_buffer_load_b128(src, (int)(j * 32u), 0, 2);  // nt: read once
      const u32x4 x1 = __builtin_amdgcn_raw_buffer_load_b128(src, (int)(j * 32u + 16u), 0, 2);
      const uint32_t o = (uint32_t)(kk - 1 - j) * 32u;
      __builtin_amdgcn_raw_buffer_store_b128(x0, dst, (int)o, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(x1, dst, (int)(o + 16u), 0, 0);
      if (kp.flows_v6 && (x1[2] >> 16) & NPR_FLOW_KIND_IPV6) {  // IPv6 rows: their parked side row too
        const u32x4 *s6 = reinterpret_cast<const u32x4 *>(kp.park_v6 + (base + j) * 8);
        u32x4 *d6 = reinterpret_cast<u32x4 *>(kp.flows_v6 + (kp.flow_cap - 1 - (pok + j)) * 8);
        d6[0] = s6[0], d6[1] = s6[1];
      }
    }
  }
  stamp<DIAG>(kp, c0, 12);
  if (c1 == kp.ntiles && lane == 0) {  // this run holds the capture's last tile
    const uint64_t tot_rec = pcnt + n, tot_ok = pok + k;
    uint32_t fl = 0;
    if (kp.flows && tot_ok > kp.flow_cap) fl |= NPR_SUMMARY_FLOW_OVERFLOW;
    kp.summary->n_records = tot_rec;
    kp.summary->n_flows = tot_ok;
    kp.summary->consumed = ex;
    kp.summary->flags = fl;
    kp.summary->entry = entry0;
    kp.summary->epoch = kp.epoch;
  }
}

// pass 1 alone / pass 2 alone (two launches; diagnostics) and both fused in one persistent grid:
// a wave moves from its scan chunk straight to its emit chunk, whose prefix fold waits only for
// the aggregates of earlier chunks (lower, earlier-dispatched workgroups: no deadlock).
template <bool DIAG, bool LIGHT>
__global__ __launch_bounds__(kWave) void k_scan_tiles(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) ParseShared sh;
  uint32_t c0, c1;
  chunk_of(kp.ntiles, blockIdx.x, gridDim.x, c0, c1);
  if (c0 < c1) scan_chunk<DIAG, LIGHT>(kp, sh, c0, c1);
}
template <bool DIAG, bool LIGHT>
__global__ __launch_bounds__(kWave) void k_emit_tiles(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) ParseShared sh;
  uint32_t c0, c1;
  chunk_of(kp.ntiles, blockIdx.x, gridDim.x, c0, c1);
  if (c0 >= c1) return;
  if (LIGHT) emit_light_chunk<DIAG>(kp, sh, c0, c1);
  else emit_chunk<DIAG>(kp, sh, c0, c1);
}
template <bool DIAG, bool LIGHT>
__global__ __launch_bounds__(kWave) void k_parse_fused(ParseParams kp) {
  __shared__ __attribute__((aligned(16))) ParseShared sh;
  uint32_t c0, c1;
  chunk_of(kp.ntiles, blockIdx.x, gridDim.x, c0, c1);
  if (c0 >= c1) return;
  scan_chunk<DIAG, LIGHT>(kp, sh, c0, c1);
  if (LIGHT) emit_light_chunk<DIAG>(kp, sh, c0, c1);
  else emit_chunk<DIAG>(kp, sh, c0, c1);
}

static int per_cu(const void *k) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, kWave, 0) != hipSuccess) return 1;
  return n > 0 ? n : 1;
}
// resident one-wave workgroups per CU of the production variants (light = the bench / FFI mode)
int scan_blocks_per_cu() { return per_cu((const void *)k_scan_tiles<false, true>); }
int emit_blocks_per_cu() { return per_cu((const void *)k_emit_tiles<false, true>); }
int fused_blocks_per_cu() { return per_cu((const void *)k_parse_fused<false, true>); }

template <bool DIAG, bool LIGHT>
static hipError_t launch(const ParseParams &p, uint32_t grid_scan, uint32_t grid_emit, hipStream_t s) {
  const uint32_t g1 = grid_scan < p.ntiles ? grid_scan : p.ntiles;
  if (grid_emit == 0) {  // fused
    hipLaunchKernelGGL((k_parse_fused<DIAG, LIGHT>), dim3(g1), dim3(kWave), 0, s, p);
    return hipGetLastError();
  }
  const uint32_t g2 = grid_emit < p.ntiles ? grid_emit : p.ntiles;
  hipLaunchKernelGGL((k_scan_tiles<DIAG, LIGHT>), dim3(g1), dim3(kWave), 0, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_emit_tiles<DIAG, LIGHT>), dim3(g2), dim3(kWave), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_parse_extract(const ParseParams &p, uint32_t grid_scan, uint32_t grid_emit, hipStream_t s) {
  const bool diag = p.stats || p.stamps, light = (p.flags & kFlagLight) != 0;
  if (diag) return light ? launch<true, true>(p, grid_scan, grid_emit, s) : launch<true, false>(p, grid_scan, grid_emit, s);
  return light ? launch<false, true>(p, grid_scan, grid_emit, s) : launch<false, false>(p, grid_scan, grid_emit, s);
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
