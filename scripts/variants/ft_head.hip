// npr_flowtable.hip — row f4: the distinct-flow table (new; not in the reference).
//
// Input: a flow table as the device path writes it (npr_flow rows, the IPv6 side rows), e.g. the
// convert_records output of npr_dev_parse_extract (src/flow/mod.rs:101-123), optionally with a
// weight per row (merging already-aggregated tables, e.g. one per GPU of a sharded capture).
// Output: one row per distinct 5-tuple {family, protocol, src ip, dst ip, src port, dst port},
// in the order of the input rows that first carry it (for a convert_records table: reverse file
// order of first appearance), with
//   the flow of its FIRST-SEEN record (lowest record offset; its offset is in the row),
//   count = the sum of the weights of its rows (1 each without weights).
//
// Layout: an open-addressing hash table of S = 2^k >= 2n slots in HBM.  A slot word is
// {hash32 | 1 : 32, claiming row : 32}, claimed by one 64-bit CAS, so a probe compares the full key
// only against the one row that claimed a slot with the same hash; count (u64, atomic add) and
// first-seen offset (u64, atomic min) live beside it.  Then the first-seen row of each slot is
// marked and the marked rows are compacted in input order (block counts, one-workgroup scan,
// scatter).  Everything is integer work on HBM-resident tables: memory-bound, no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "npr_internal.hpp"

namespace npr {
namespace {

constexpr int kB = 256;          // threads per workgroup
constexpr int kAggItems = 1024;  // rows per compaction block

struct Key {
  uint32_t w[11];  // kind, ports, src ip (1 or 4 words), dst ip (1 or 4 words)
  uint32_t nw;
};

// the flow row's 5-tuple (+ family / protocol bits); IPv6 addresses from the side row
__device__ __forceinline__ Key row_key(const uint32_t *row, const uint32_t *v6row) {
  Key k;
  const uint32_t kind = (row[6] >> 16) & 0xffu;
  k.w[0] = kind;
  k.w[1] = row[2];  // src port | dst port << 16
  if (kind & NPR_FLOW_KIND_IPV6) {
#pragma unroll
    for (int i = 0; i < 8; ++i) k.w[2 + i] = v6row ? v6row[i] : 0u;
    k.nw = 10;
  } else {
    k.w[2] = row[0];
    k.w[3] = row[1];
    k.nw = 4;
  }
  return k;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

__device__ __forceinline__ uint64_t key_hash(const Key &k) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
  for (uint32_t i = 0; i < k.nw; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  return h;
}

__device__ __forceinline__ bool key_eq(const Key &a, const Key &b) {
  if (a.nw != b.nw) return false;
  for (uint32_t i = 0; i < a.nw; ++i)
    if (a.w[i] != b.w[i]) return false;
  return true;
}

__device__ __forceinline__ uint64_t row_offset(const uint32_t *row) {  // 40-bit record offset
  return ((uint64_t)row[7] << 8) | (row[6] >> 24);
}

// One workgroup inserts kInsRows rows: each finds (or claims) its slot in the global table, then
// the workgroup folds its rows per slot in an LDS table (count sum, first-seen minimum), so a
// popular flow costs one pair of global atomics per workgroup, not one per row.
constexpr int kInsPer = 4, kInsRows = kB * kInsPer, kLdsSlots = 2 * kInsRows;

__global__ __launch_bounds__(kB) void k_agg_insert(const uint32_t *flows, const uint32_t *flows_v6,
                                                   const uint64_t *weights, uint64_t n, uint64_t *slot_word,
                                                   uint64_t *slot_first, uint64_t *slot_count, uint32_t *slot_of_row,
                                                   uint64_t mask) {
  __shared__ uint32_t lkey[kLdsSlots];
  __shared__ unsigned long long lcnt[kLdsSlots], lfirst[kLdsSlots];
  for (int e = threadIdx.x; e < kLdsSlots; e += kB) {
    lkey[e] = ~0u;
    lcnt[e] = 0;
    lfirst[e] = ~0ull;
  }
  __syncthreads();
  for (int q = 0; q < kInsPer; ++q) {
    const uint64_t i = (uint64_t)blockIdx.x * kInsRows + (uint64_t)q * kB + threadIdx.x;
    if (i >= n) continue;
    const uint32_t *row = flows + i * 8;
    const Key k = row_key(row, flows_v6 ? flows_v6 + i * 8 : nullptr);
    const uint64_t h = key_hash(k);
    const uint32_t h32 = (uint32_t)(h >> 32) | 1u;  // never 0: 0 marks an empty slot
    const uint64_t mine = ((uint64_t)h32 << 32) | (uint32_t)i;
    uint64_t pos = h & mask;
    for (;;) {
      uint64_t w = __hip_atomic_load(slot_word + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (w == 0) {
        uint64_t expect = 0;
        if (__hip_atomic_compare_exchange_strong(slot_word + pos, &expect, mine, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
          break;  // claimed
        w = expect;
      }
      if ((uint32_t)(w >> 32) == h32) {  // same hash: compare with the claiming row's key
        const uint64_t j = (uint32_t)w;
        const Key o = row_key(flows + j * 8, flows_v6 ? flows_v6 + j * 8 : nullptr);
        if (key_eq(k, o)) break;
      }
      pos = (pos + 1) & mask;
    }
    slot_of_row[i] = (uint32_t)pos;
    // fold into the workgroup's LDS table (at most kInsRows distinct slots in 2x as many entries)
    uint32_t e = (uint32_t)mix64(pos) & (kLdsSlots - 1);
    for (;;) {
      const uint32_t old = atomicCAS(&lkey[e], ~0u, (uint32_t)pos);
      if (old == ~0u || old == (uint32_t)pos) break;
      e = (e + 1) & (kLdsSlots - 1);
    }
    atomicAdd(&lcnt[e], (unsigned long long)(weights ? weights[i] : 1ull));
    atomicMin(&lfirst[e], (unsigned long long)row_offset(row));
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kLdsSlots; e += kB) {
    const uint32_t pos = lkey[e];
    if (pos == ~0u) continue;
    atomicAdd((unsigned long long *)(slot_count + pos), lcnt[e]);
    atomicMin((unsigned long long *)(slot_first + pos), lfirst[e]);
  }
}

// Ties: several rows of one slot may carry the slot's first-seen offset (a record listed twice,
// or tables of several captures merged: every capture's first record sits at offset 24).  The
// slot's first-seen ROW is the lowest row index among them (the input order the output keeps):
// one atomic min per tied row into the slot's word, which the insert no longer needs (its claims
// are done), reset to ~0 in between.
__global__ __launch_bounds__(kB) void k_agg_tie(const uint32_t *flows, const uint32_t *slot_of_row,
                                                const uint64_t *slot_first, uint64_t n, uint64_t *slot_row) {
  const uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint32_t pos = slot_of_row[i];
  if (row_offset(flows + i * 8) == slot_first[pos]) atomicMin((unsigned long long *)(slot_row + pos), (unsigned long long)i);
}

// is row i its slot's first-seen row?
__device__ __forceinline__ bool is_first(const uint32_t *slot_of_row, const uint64_t *slot_row, uint64_t i) {
  return slot_row[slot_of_row[i]] == i;
}

__global__ __launch_bounds__(kB) void k_agg_count(const uint32_t *slot_of_row, const uint64_t *slot_row, uint64_t n,
                                                  uint32_t *block_counts) {
  __shared__ uint32_t sc[kB / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * kAggItems;
  uint32_t c = 0;
  for (int k = 0; k < kAggItems / kB; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kB;
    c += (i < n && is_first(slot_of_row, slot_row, i)) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63u) == 0) sc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) block_counts[blockIdx.x] = sc[0] + sc[1] + sc[2] + sc[3];
}

// exclusive scan of nb block counts by one workgroup; *total = their sum
__global__ __launch_bounds__(kB) void k_agg_scan(uint32_t *counts, uint64_t nb, uint64_t *total) {
  __shared__ uint64_t part[kB];
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nb; base += kB) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t v = i < nb ? counts[i] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < kB; o <<= 1) {
      const uint64_t add = threadIdx.x >= (uint32_t)o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < nb) counts[i] = (uint32_t)(carry + part[threadIdx.x] - v);
    carry += part[kB - 1];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(kB) void k_agg_scatter(const uint32_t *flows, const uint32_t *flows_v6,
                                                    const uint32_t *slot_of_row, const uint64_t *slot_row,
                                                    const uint64_t *slot_count, uint64_t n, const uint32_t *offsets,
                                                    uint32_t *out, uint32_t *out_v6, uint64_t *counts, uint64_t cap) {
  __shared__ uint32_t sc[kAggItems / kB][kB / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kAggItems;
  bool first[kAggItems / kB];
#pragma unroll
  for (int k = 0; k < kAggItems / kB; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kB;
    first[k] = i < n && is_first(slot_of_row, slot_row, i);
    const uint64_t bal = __ballot(first[k]);
    if (lane == 0) sc[k][wave] = (uint32_t)__builtin_popcountll(bal);
  }
  __syncthreads();
  uint64_t base = offsets[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kAggItems / kB; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kB;
    const uint64_t bal = __ballot(first[k]);
    if (first[k]) {
      uint64_t r = base + (uint64_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      for (uint32_t w = 0; w < wave; ++w) r += sc[k][w];
      if (r < cap) {
        const uint4 *src = reinterpret_cast<const uint4 *>(flows + i * 8);
        uint4 *dst = reinterpret_cast<uint4 *>(out + r * 8);
        dst[0] = src[0];
        dst[1] = src[1];
        if (out_v6) {
          uint4 *d6 = reinterpret_cast<uint4 *>(out_v6 + r * 8);
          if (flows_v6) {
            const uint4 *s6 = reinterpret_cast<const uint4 *>(flows_v6 + i * 8);
            d6[0] = s6[0];
            d6[1] = s6[1];
          } else {
            d6[0] = d6[1] = make_uint4(0, 0, 0, 0);
          }
        }
        if (counts) counts[r] = slot_count[slot_of_row[i]];
      }
    }
    base += sc[k][0] + sc[k][1] + sc[k][2] + sc[k][3];
  }
}

}  // namespace

uint64_t flow_table_slots(uint64_t n) {  // n <= kMaxAggRows: S <= 2^31, so a slot index < 2^31 never equals ~0
  uint64_t s = 1024;
  while (s < 2 * n) s <<= 1;
  return s;
}
uint64_t flow_table_bytes(uint64_t n) {
  const uint64_t s = flow_table_slots(n), nb = (n + kAggItems - 1) / kAggItems;
  return s * 24 + n * 4 + nb * 4 + 64;
}

hipError_t launch_flow_aggregate(const uint32_t *flows, const uint32_t *flows_v6, const uint64_t *weights, uint64_t n,
                                 void *work, uint32_t *out, uint32_t *out_v6, uint64_t *counts, uint64_t cap,
                                 uint64_t *total, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), s);
  if (n > kMaxAggRows) return hipErrorInvalidValue;  // slot indices are 32-bit, ~0 marks an empty LDS entry
  const uint64_t S = flow_table_slots(n), nb = (n + kAggItems - 1) / kAggItems;
  uint64_t *slot_word = (uint64_t *)work, *slot_first = slot_word + S, *slot_count = slot_first + S;
  uint32_t *slot_of_row = (uint32_t *)(slot_count + S), *block = slot_of_row + n;
  hipError_t e;
  if ((e = hipMemsetAsync(slot_word, 0, S * 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(slot_first, 0xff, S * 8, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(slot_count, 0, S * 8, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_agg_insert, dim3((uint32_t)((n + kInsRows - 1) / kInsRows)), dim3(kB), 0, s, flows, flows_v6, weights, n,
                     slot_word, slot_first, slot_count, slot_of_row, S - 1);
  uint64_t *slot_row = slot_word;  // the claims are done: the word now holds the first-seen row
  if ((e = hipMemsetAsync(slot_row, 0xff, S * 8, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_agg_tie, dim3((uint32_t)((n + kB - 1) / kB)), dim3(kB), 0, s, flows, slot_of_row, slot_first, n,
                     slot_row);
  hipLaunchKernelGGL(k_agg_count, dim3((uint32_t)nb), dim3(kB), 0, s, slot_of_row, slot_row, n, block);
  hipLaunchKernelGGL(k_agg_scan, dim3(1), dim3(kB), 0, s, block, nb, total);
  hipLaunchKernelGGL(k_agg_scatter, dim3((uint32_t)nb), dim3(kB), 0, s, flows, flows_v6, slot_of_row, slot_row,
                     slot_count, n, block, out, out_v6, counts, cap);
  return hipGetLastError();
}

}  // namespace npr
