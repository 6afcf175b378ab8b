// npr_device.hpp — device helpers shared by the parse kernels (npr_kernels.hip) and the sparse
// record walk (npr_sparse.hip): byte access, the branch-light fast decode, hand-off granules, the
// chain-consistency segment, wave scans and the speculation context.  Not installed.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "npr_decode.hpp"
#include "npr_internal.hpp"

namespace npr {

typedef unsigned int u32x4 __attribute__((__vector_size__(16)));
constexpr uint64_t kNone = ~0ull;
constexpr uint64_t kMask48 = (1ull << 48) - 1;
constexpr uint32_t kTsWindow = 1u << 20;  // speculation: |ts_sec delta| between neighbours
constexpr uint32_t kInclMax = 1u << 18;   // speculation: plausible incl_len bound

// ---------------------------------------------------------------------------------------------
// byte access
// ---------------------------------------------------------------------------------------------

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
    return slow32(g, gavail, q);
  }
  __device__ __forceinline__ uint32_t u8(uint32_t q) const {
    const uint64_t a = (uint64_t)rel + q;
    if (a < (uint64_t)kStage) return b[a];
    return (uint64_t)q < gavail ? g[q] : 0u;
  }
  // out of line and by value: a `this` pointer would pin the reader in scratch memory
  static __device__ __noinline__ uint32_t slow32(const uint8_t *g, uint64_t gavail, uint32_t q) {
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
// fast decode: Ethernet (untagged) / IPv4 (IHL 5) or IPv6 (no extension) / TCP or UDP.
// Branch-light: 17 aligned LDS words + v_alignbyte, static field offsets, status by selects;
// bit-identical to decode<> for these shapes.  Returns 0xff for any other frame (the caller then
// runs the general decode<>).
// ---------------------------------------------------------------------------------------------
template <bool FIELDS, bool BALLOT4>
__device__ __forceinline__ uint32_t decode_fast_core(uint32_t (&a)[17], uint32_t n, FlowWords &f, bool valid);
// A16: w is 16-byte aligned in LDS (the staged tiles; not the per-record rows)
// valid: lanes whose result is used (A16: when every such lane is IPv4, the IPv4-only variant)
template <bool FIELDS, bool A16 = false>
__device__ __forceinline__ uint32_t decode_fast(const uint32_t *w, uint32_t rel, uint32_t n, FlowWords &f,
                                                bool valid = true) {
  const uint32_t sh = rel & 3u;
  uint32_t a[17];
  // Every lane's window offset mod 16 the same (fixed-length records at a stride that is a
  // multiple of 16, e.g. C2's 80 B): 16-B ds_read_b128 from the aligned base, conflict-free at
  // such strides (the b32 reads at an 80-B stride are 4-way bank conflicts, MI355X_MICROARCH.md
  // §LDS).  Otherwise per-dword reads.
  const uint32_t m16 = rel & 15u, u16 = __builtin_amdgcn_readfirstlane(m16);
  if (A16 && __ballot(m16 != u16) == 0ull) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(w + ((rel & ~15u) >> 2));
    // a[k] = bytes [rel + 4k, rel + 4k + 4): dwords J + k, J + k + 1 (Z: 4-aligned, dword J + k)
    auto fill = [&](auto J, auto Z) {
      constexpr int j = decltype(J)::value;
      constexpr bool z = decltype(Z)::value;
      uint32_t W[j + 18];
#pragma unroll
      for (int c = 0; c < (j + 18 + 3) / 4; ++c) {
        const u32x4 v = q[c];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * c + e < j + 18) W[4 * c + e] = v[e];
      }
#pragma unroll
      for (int k = 0; k < 17; ++k) a[k] = z ? W[j + k] : __builtin_amdgcn_alignbyte(W[j + k + 1], W[j + k], sh);
    };
    using Y = std::true_type;
    using N = std::false_type;
    switch (u16) {  // (wave-uniform)
      case 0: fill(std::integral_constant<int, 0>{}, Y{}); break;
      case 4: fill(std::integral_constant<int, 1>{}, Y{}); break;
      case 8: fill(std::integral_constant<int, 2>{}, Y{}); break;
      case 12: fill(std::integral_constant<int, 3>{}, Y{}); break;
      default:
        switch (u16 >> 2) {
          case 0: fill(std::integral_constant<int, 0>{}, N{}); break;
          case 1: fill(std::integral_constant<int, 1>{}, N{}); break;
          case 2: fill(std::integral_constant<int, 2>{}, N{}); break;
          default: fill(std::integral_constant<int, 3>{}, N{}); break;
        }
    }
  } else {
    const uint32_t *p = w + (rel >> 2);
    uint32_t prev = p[0];
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      const uint32_t nx = p[k + 1];
      a[k] = __builtin_amdgcn_alignbyte(nx, prev, sh);
      prev = nx;
    }
  }
  return decode_fast_core<FIELDS, A16>(a, n, f, valid);
}

// decode_fast on the frame's first 68 bytes, a[k] = payload bytes [4k, 4k + 4) (any source).
// BALLOT4: when every valid lane is IPv4, the IPv4-only variant (a[12..16] are then not read).
template <bool FIELDS, bool BALLOT4>
__device__ __forceinline__ uint32_t decode_fast_core(uint32_t (&a)[17], uint32_t n, FlowWords &f, bool valid) {
  // pin the window in registers: otherwise the backend turns the IPv4/IPv6 selects below into
  // divergent branches that each load only their own words (select-to-branch on loads)
#pragma unroll
  for (int k = 0; k < 17; ++k) asm volatile("" : "+v"(a[k]));
  auto byte = [&](int i) { return (a[i >> 2] >> (8 * (i & 3))) & 0xffu; };
  // big-endian u16 at byte i: one v_perm_b32 over the two words that may hold it
  auto be16 = [&](int i) {
    const int k = i >> 2, k1 = k + 1 < 17 ? k + 1 : 16;
    return __builtin_amdgcn_perm(a[k1], a[k], 0x0c0c0000u | ((uint32_t)(i & 3) << 8) | (uint32_t)((i & 3) + 1));
  };
  // Every quantity is computed for every lane and combined by selects (no data-dependent
  // branches: divergent if/else here costs more scalar exec-mask work than the arithmetic).
  const uint32_t etype = be16(12), b0 = byte(14);
  const uint32_t proto4 = byte(23), nh = byte(20);
  const bool is4 = (etype == 0x0800u) & (b0 == 0x45u) & (n >= 34u) & ((proto4 == 6u) | (proto4 == 17u));
  auto core = [&](auto ONLY4) -> uint32_t {
  // ONLY4: every used lane is IPv4 (the selects below fold; unused lanes return garbage)
  constexpr bool only4 = decltype(ONLY4)::value;
  const bool v4 = only4 ? true : is4;
  const bool v6 = only4 ? false : (etype == 0x86ddu) & ((b0 >> 4) == 6u) & (n >= 54u) & ((nh == 6u) | (nh == 17u));
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
    f.v6off = 22u;
  }
  return (v4 | v6) ? (st3 ? st3 : st4) : 0xffu;
  };
  if (BALLOT4 && __ballot(valid & !is4) == 0ull) return core(std::true_type{});
  return core(std::false_type{});
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
  // (readfirstlane returns int: widen through uint32_t, or offsets past 2 GiB sign-extend)
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
}

// A segment of consecutive tiles [first, last] under speculation: the chain entered at `entry`
// (speculated) and left at `exit`, with `cnt` records and `ok` Ok flows in between.
struct Seg {
  uint64_t entry, exit, cnt, ok;
  int64_t first, last, mism;  // mism: lowest tile whose speculated entry is contradicted
  uint32_t valid, spare;      // (no padding bytes: a padded copy is left in scratch memory)
};

// lane i <- lane i+1 (DPP wave_shl:1, no LDS round trip); lane 63 gets 0
__device__ __forceinline__ uint64_t shfl_down64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x130, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x130, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
// lane i <- lane i-1 (lane 0 gets lane 63's value; callers ignore it)
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v) {
  const int src = ((int)(threadIdx.x & 63u) + 63) & 63;
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
  return ((uint64_t)hi << 32) | lo;
}
// exclusive prefix sum over the 64 lanes (every lane active)
__device__ __forceinline__ uint32_t excl_scan_u32(uint32_t v) {
  // inclusive scan by DPP: row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15 / :31
  // carry the row totals (no LDS round trips)
  uint32_t x = v;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x - v;
}
// whole-wave sum (DPP reduction of the device library); every lane must be active
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);

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

// LDS written by some lanes of this wave, then read by others: LDS executes one wave's requests
// in order, so only the compiler must not move the accesses across this point.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// speculation context of this launch: ts_usec bound from the file magic, the first record's
// ts_sec as a reference (both read once per wave)
// Issue the (byte) loads of the speculation context: lanes 0..3 the pcap magic, lanes 4..7 the
// reference record's ts_sec (range-checked: a byte outside the input reads 0).  spec_ctx()
// finishes it once the loads landed.
__device__ __forceinline__ uint32_t spec_ctx_load(const ParseParams &kp) {
  if (kp.flags & kFlagHostSpec) return 0u;  // a shard: bytes 0..3 are not in its buffer
  const uint32_t lane = threadIdx.x & 63u;
  const bool has_ref = kp.ref != kNone && kp.len >= kp.ref + 16;
  const uint64_t lim = kp.len < 0x7fffffffull ? kp.len : 0x7fffffffull;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)kp.buf, 0, (int)lim, 0x00020000);
  uint32_t off = lane < 4 ? lane : (uint32_t)(has_ref && kp.ref < 0x7ffffff0ull ? kp.ref : 0x7ffffff0ull) + (lane - 4);
  if (lane >= 8) off = 0x7ffffff0u;  // out of range: 0
  return __builtin_amdgcn_raw_buffer_load_b8(rs, (int)off, 0, 0);
}
// speculation context of this launch: ts_usec bound from the file magic, the first record's
// ts_sec as a reference
__device__ __forceinline__ SpecCtx spec_ctx(const ParseParams &kp, uint32_t b) {
  SpecCtx sc;
  sc.big = kp.big;
  sc.avail = 0;
  sc.exact_end = true;
  if (kp.flags & kFlagHostSpec) {  // a shard: the host supplies the magic's bound and the reference ts_sec
    sc.frac_max = kp.frac_max;
    sc.has_ref = (kp.flags & kFlagHostRef) != 0;
    sc.ts_ref = kp.ts_ref;
    return sc;
  }
  uint32_t v = b << (8 * (threadIdx.x & 3u));
  v |= __shfl_xor((int)v, 1, 64);
  v |= __shfl_xor((int)v, 2, 64);
  const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
  const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)v, 4);
  // microsecond pcap magic (either byte order) at byte 0: ts_usec < 1e6
  sc.frac_max = ((kp.flags & kFlagMagicAtZero) && (m == 0xA1B2C3D4u || m == 0xD4C3B2A1u)) ? 1000000u : kp.frac_max;
  sc.has_ref = kp.ref != kNone && kp.len >= kp.ref + 16;
  sc.ts_ref = kp.big ? __builtin_bswap32(r) : r;
  return sc;
}

}  // namespace npr
