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
constexpr int kPackBits = 24;    // row bits beside the 40-bit record offset in a packed first-seen word

struct Key {
  uint32_t w[10];  // kind, ports, src ip, dst ip (IPv4: one word each, the rest 0; IPv6: four each)
  bool v6;
};

// the flow row's 5-tuple (+ family / protocol bits); IPv6 addresses from the side row.  Fixed-size
// and fully unrolled (a loop over a run-time word count put two keys in scratch memory).
__device__ __forceinline__ Key row_key(const uint32_t *row, const uint32_t *v6row) {
  Key k;
  const uint32_t kind = (row[6] >> 16) & 0xffu;
  k.w[0] = kind;
  k.w[1] = row[2];  // src port | dst port << 16
  k.v6 = (kind & NPR_FLOW_KIND_IPV6) != 0;
  if (k.v6) {
#pragma unroll
    for (int i = 0; i < 8; ++i) k.w[2 + i] = v6row ? v6row[i] : 0u;
  } else {
    k.w[2] = row[0];
    k.w[3] = row[1];
#pragma unroll
    for (int i = 4; i < 10; ++i) k.w[i] = 0u;
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

// the first 4 words (IPv4) or all 10 (IPv6)
__device__ __forceinline__ uint64_t key_hash(const Key &k) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  if (k.v6) {
#pragma unroll
    for (uint32_t i = 4; i < 10; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  }
  return h;
}

// w[0] holds the family bit, and IPv4 keys are zero past their fourth word.  No short circuit: an
// early exit per word let the compiler sink each row word's load behind the previous compare
// (serial global loads; the Zipf aggregate went 0.186 -> 0.279 ms)
__device__ __forceinline__ bool key_eq(const Key &a, const Key &b) {
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) diff |= a.w[i] ^ b.w[i];
  return diff == 0;
}

__device__ __forceinline__ uint64_t row_offset(const uint32_t *row) {  // 40-bit record offset
  return ((uint64_t)row[7] << 8) | (row[6] >> 24);
}

// Find (or claim) the global slot of key k (hash h) for row i: linear probing over slot words
// {hash32 | 1, claiming row}; a slot with the same hash is compared against its claiming row's key.
__device__ __forceinline__ uint64_t probe(const uint32_t *flows, const uint32_t *flows_v6, uint64_t *slot_word,
                                          uint64_t mask, const Key &k, uint64_t h, uint64_t i) {
  const uint32_t h32 = (uint32_t)(h >> 32) | 1u;  // never 0: 0 marks an empty slot
  const uint64_t mine = ((uint64_t)h32 << 32) | (uint32_t)i;
  uint64_t pos = h & mask;
  for (;;) {
    uint64_t w = __hip_atomic_load(slot_word + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == 0) {
      uint64_t expect = 0;
      if (__hip_atomic_compare_exchange_strong(slot_word + pos, &expect, mine, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        return pos;  // claimed
      w = expect;
    }
    if ((uint32_t)(w >> 32) == h32) {  // same hash: compare with the claiming row's key
      const uint64_t j = (uint32_t)w;
      if (key_eq(k, row_key(flows + j * 8, flows_v6 ? flows_v6 + j * 8 : nullptr))) return pos;
    }
    pos = (pos + 1) & mask;
  }
}

// One workgroup inserts kInsRows rows in three steps:
//  1. every row claims (or finds) the LDS entry of its 32-bit hash; the claiming row leads it;
//  2. leaders probe the global table; the other rows compare their key with their leader's and
//     join its entry (count sum, first-seen minimum in LDS), or, on a 32-bit hash collision inside
//     the workgroup, probe the global table themselves and fold straight into it;
//  3. leaders publish their slot in the entry, joiners take it, and each entry costs one pair of
//     global atomics.
// So a popular flow costs one global probe per workgroup, not one per row: with one probe per row,
// a Zipf mix's hottest slots took a CAS from every row that saw them empty at the start (all
// workgroups are resident at once) and every later row's read on one L2 channel.  512 rows per
// workgroup (24-KB LDS tables): 1024 measured the same on the Zipf mix but 12 % slower all-distinct
// (48 KB, 3 workgroups per CU).
constexpr int kInsPer = 2, kInsRows = kB * kInsPer, kLdsSlots = 2 * kInsRows;

__global__ __launch_bounds__(kB) void k_agg_insert(const uint32_t *flows, const uint32_t *flows_v6,
                                                   const uint64_t *weights, uint64_t n, uint64_t *slot_word,
                                                   uint64_t *slot_first, uint64_t *slot_count, uint32_t *slot_of_row,
                                                   uint64_t mask, bool packed) {
  __shared__ uint32_t lhash[kLdsSlots];  // the entry's hash32 (0: empty)
  __shared__ uint32_t llead[kLdsSlots];  // the leader's row in the workgroup, then (step 3) its slot
  __shared__ unsigned long long lcnt[kLdsSlots], lfirst[kLdsSlots];
  for (int e = threadIdx.x; e < kLdsSlots; e += kB) {
    lhash[e] = 0;
    lcnt[e] = 0;
    lfirst[e] = ~0ull;
  }
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kInsRows;
  Key k[kInsPer];
  uint64_t h[kInsPer];
  uint32_t ent[kInsPer];
  uint32_t lead = 0, join = 0;  // bit q: row q leads / joined its entry
#pragma unroll
  for (int q = 0; q < kInsPer; ++q) {
    const uint32_t r = (uint32_t)q * kB + threadIdx.x;
    const uint64_t i = base + r;
    ent[q] = 0;
    h[q] = 0;
    if (i >= n) continue;
    k[q] = row_key(flows + i * 8, flows_v6 ? flows_v6 + i * 8 : nullptr);
    h[q] = key_hash(k[q]);
    const uint32_t h32 = (uint32_t)(h[q] >> 32) | 1u;
    uint32_t e = (uint32_t)h[q] & (kLdsSlots - 1);
    for (;;) {
      const uint32_t old = atomicCAS(&lhash[e], 0u, h32);
      if (old == 0u) {
        llead[e] = r;
        lead |= 1u << q;
        break;
      }
      if (old == h32) break;
      e = (e + 1) & (kLdsSlots - 1);
    }
    ent[q] = e;
  }
  __syncthreads();
  uint32_t pos[kInsPer];
#pragma unroll
  for (int q = 0; q < kInsPer; ++q) {
    const uint64_t i = base + (uint32_t)q * kB + threadIdx.x;
    pos[q] = 0;
    if (i >= n) continue;
    const uint32_t *row = flows + i * 8;
    const bool ld = (lead >> q) & 1u;
    bool jn = false;
    if (!ld) {
      const uint64_t j = base + llead[ent[q]];
      jn = key_eq(k[q], row_key(flows + j * 8, flows_v6 ? flows_v6 + j * 8 : nullptr));
    }
    const unsigned long long wt = weights ? weights[i] : 1ull;
    const unsigned long long off = packed ? (row_offset(row) << kPackBits) | i : row_offset(row);
    if (ld || jn) {
      if (ld) {
        pos[q] = (uint32_t)probe(flows, flows_v6, slot_word, mask, k[q], h[q], i);
        slot_of_row[i] = pos[q];
      }
      join |= (uint32_t)jn << q;
      atomicAdd(&lcnt[ent[q]], wt);
      atomicMin(&lfirst[ent[q]], off);
    } else {  // a different key with the same 32-bit hash inside the workgroup
      const uint32_t p = (uint32_t)probe(flows, flows_v6, slot_word, mask, k[q], h[q], i);
      slot_of_row[i] = p;
      atomicAdd((unsigned long long *)(slot_count + p), wt);
      atomicMax((unsigned long long *)(slot_first + p), ~off);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kInsPer; ++q)
    if ((lead >> q) & 1u) llead[ent[q]] = pos[q];
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kInsPer; ++q)
    if ((join >> q) & 1u) slot_of_row[base + (uint32_t)q * kB + threadIdx.x] = llead[ent[q]];
  for (int e = threadIdx.x; e < kLdsSlots; e += kB) {
    if (lhash[e] == 0u) continue;
    const uint32_t p = llead[e];
    atomicAdd((unsigned long long *)(slot_count + p), lcnt[e]);
    atomicMax((unsigned long long *)(slot_first + p), ~lfirst[e]);
  }
}

// Ties: several rows of one slot may carry the slot's first-seen offset (a record listed twice,
// or tables of several captures merged: every capture's first record sits at offset 24).  The
// slot's first-seen ROW is the lowest row index among them (the input order the output keeps).
// Up to 2^24 rows the packed minimum of the insert settles it; beyond, this pass: one atomic min
// per tied row into the slot's word, which the insert no longer needs (its claims are done), reset
// to ~0 in between.
__global__ __launch_bounds__(kB) void k_agg_tie(const uint32_t *flows, const uint32_t *slot_of_row,
                                                const uint64_t *slot_first, uint64_t n, uint64_t *slot_row) {
  const uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const uint32_t pos = slot_of_row[i];
  if (row_offset(flows + i * 8) == ~slot_first[pos]) atomicMin((unsigned long long *)(slot_row + pos), (unsigned long long)i);
}

// is row i its slot's first-seen row?
// slot_row ^ rxor, masked by rmask: the packed first-seen word (stored complemented) or the tie pass's row
__device__ __forceinline__ bool is_first(const uint32_t *slot_of_row, const uint64_t *slot_row, uint64_t rxor,
                                         uint64_t rmask, uint64_t i) {
  return ((slot_row[slot_of_row[i]] ^ rxor) & rmask) == i;
}

// Block counts of first-seen rows, and the first-seen flags themselves as one 64-bit mask per wave
// and round (kMaskWords per block), so the scatter reads 128 B per block instead of a random slot
// word per row.
constexpr int kRounds = kAggItems / kB, kMaskWords = kAggItems / 64;
static_assert(kB == 256, "the scatter sums four waves' masks");
__global__ __launch_bounds__(kB) void k_agg_count(const uint32_t *slot_of_row, const uint64_t *slot_row, uint64_t rxor, uint64_t rmask, uint64_t n,
                                                  uint32_t *block_counts, uint64_t *first_bits) {
  __shared__ uint32_t sc[kB / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kAggItems;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kB;
    const uint64_t bal = __ballot(i < n && is_first(slot_of_row, slot_row, rxor, rmask, i));
    if (lane == 0) first_bits[(uint64_t)blockIdx.x * kMaskWords + k * (kB / 64) + wave] = bal;
    c += (uint32_t)__builtin_popcountll(bal);
  }
  if (lane == 0) sc[wave] = c;
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
                                                    const uint32_t *slot_of_row, const uint64_t *first_bits,
                                                    const uint64_t *slot_count, uint64_t n, const uint32_t *offsets,
                                                    uint32_t *out, uint32_t *out_v6, uint64_t *counts, uint64_t cap) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t b0 = (uint64_t)blockIdx.x * kAggItems;
  const uint64_t *fb = first_bits + (uint64_t)blockIdx.x * kMaskWords;  // uniform: scalar loads
  uint64_t base = offsets[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kRounds; ++k) {
    const uint64_t i = b0 + threadIdx.x + (uint64_t)k * kB;
    const uint64_t m0 = fb[k * 4], m1 = fb[k * 4 + 1], m2 = fb[k * 4 + 2], m3 = fb[k * 4 + 3];
    const uint32_t c0 = (uint32_t)__builtin_popcountll(m0), c1 = (uint32_t)__builtin_popcountll(m1),
                   c2 = (uint32_t)__builtin_popcountll(m2);
    const uint64_t bal = wave == 0 ? m0 : wave == 1 ? m1 : wave == 2 ? m2 : m3;
    if ((bal >> lane) & 1ull) {
      uint64_t r = base + (uint64_t)__builtin_popcountll(bal & ((1ull << lane) - 1ull));
      r += (wave > 0 ? c0 : 0u) + (wave > 1 ? c1 : 0u) + (wave > 2 ? c2 : 0u);
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
    base += c0 + c1 + c2 + (uint32_t)__builtin_popcountll(m3);
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
  return s * 24 + n * 4 + nb * 4 + nb * kMaskWords * 8 + 64;
}

hipError_t launch_flow_aggregate(const uint32_t *flows, const uint32_t *flows_v6, const uint64_t *weights, uint64_t n,
                                 void *work, uint32_t *out, uint32_t *out_v6, uint64_t *counts, uint64_t cap,
                                 uint64_t *total, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(total, 0, sizeof(uint64_t), s);
  if (n > kMaxAggRows) return hipErrorInvalidValue;  // slot indices are 32-bit, ~0 marks an empty LDS entry
  const uint64_t S = flow_table_slots(n), nb = (n + kAggItems - 1) / kAggItems;
  uint64_t *slot_word = (uint64_t *)work, *slot_first = slot_word + S, *slot_count = slot_first + S;
  uint64_t *first_bits = slot_count + S;
  uint32_t *slot_of_row = (uint32_t *)(first_bits + nb * kMaskWords), *block = slot_of_row + n;
  hipError_t e;
  // one zero fill: claim words, first-seen words (stored complemented: the minimum is an atomic max
  // from 0) and counts are consecutive
  if ((e = hipMemsetAsync(slot_word, 0, S * 24, s)) != hipSuccess) return e;
  // up to 2^24 rows the first-seen minimum runs over {offset, row} packed in one word: ties settle
  // inside it and the first-seen row is its low bits; beyond, a second pass settles ties
  const bool packed = n <= (1ull << kPackBits);
  hipLaunchKernelGGL(k_agg_insert, dim3((uint32_t)((n + kInsRows - 1) / kInsRows)), dim3(kB), 0, s, flows, flows_v6, weights, n,
                     slot_word, slot_first, slot_count, slot_of_row, S - 1, packed);
  uint64_t *slot_row = slot_first, rxor = ~0ull, rmask = (1ull << kPackBits) - 1;
  if (!packed) {
    slot_row = slot_word;  // the claims are done: the word now holds the first-seen row
    rxor = 0;
    rmask = ~0ull;
    if ((e = hipMemsetAsync(slot_row, 0xff, S * 8, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_agg_tie, dim3((uint32_t)((n + kB - 1) / kB)), dim3(kB), 0, s, flows, slot_of_row, slot_first, n,
                       slot_row);
  }
  hipLaunchKernelGGL(k_agg_count, dim3((uint32_t)nb), dim3(kB), 0, s, slot_of_row, slot_row, rxor, rmask, n, block, first_bits);
  hipLaunchKernelGGL(k_agg_scan, dim3(1), dim3(kB), 0, s, block, nb, total);
  hipLaunchKernelGGL(k_agg_scatter, dim3((uint32_t)nb), dim3(kB), 0, s, flows, flows_v6, slot_of_row, first_bits,
                     slot_count, n, block, out, out_v6, counts, cap);
  return hipGetLastError();
}

}  // namespace npr
