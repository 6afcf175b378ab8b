// rw_floor — the combined read + write floor of the C2 launch on this MI355X (VERDICT r04 item 1,
// r05 items 1 and 3): read the 80 MB capture and write the flow table in ONE kernel, in the
// resident pass's geometry (256 workgroups x 16 waves, one per CU; each wave a contiguous range of
// 4 KiB tiles through a two-slot LDS-DMA ring, nt loads; rows stored as whole-line sc1 blocks of
// 51 rows x W bytes per tile, the resident pass's phase-B store).  Nothing is parsed: this is the
// memory system and the hand-off alone.
//   R    read only
//   W    write only (each wave its ranges' blocks)
//   I    writes independent of the reads: each tile's rows are stored right after it lands
//   L    each wave stores its range's rows after its own last tile (other waves still read)
//   H    one grid-wide hand-off (every workgroup arrives on one counter after its reads, wave 0
//        polls it by returning atomics + s_sleep), then the rows
//   K    the look-back's dependency without the fold: workgroup b waits for workgroups 0..b-1
//        only (a 4-B flag per workgroup, packed; a window read by wave 0, returning atomics), then
//        its rows
//   P    K with each flag an 8-B tagged granule on its own 128-B line (returning-atomic polls)
//   S    P polled with sc1 loads instead of returning atomics (a stale line would time out: the
//        abort word reports it)
//   A    the resident pass's publication and look-back (round 5): after the barrier every wave
//        stores its 4-granule A (sc1), wave 0 stores its workgroup's 5-granule G and adds to an
//        arrival counter, reads every lower G once with sc1 loads and re-reads only the untagged
//        granules by returning atomics, napping s_sleep(8) x {1, 2, 2, ...} with an abort-word
//        load and a clock read per nap
//   B    A without the per-wave A stores
//   C    A with the nap reduced to s_sleep(2) and the abort word read every 16th nap only
//   D    B, re-polling the missing granules with sc1 loads (no atomics), s_sleep(4), the abort
//        word every 16th poll
//   E    D with each workgroup's 5 granules stored and read as 16 + 16 + 8 B (dwordx4 sc1)
//   F    E with the per-wave A stores issued after the look-back (behind the second barrier)
//   N    E without the arrival counter
//   Q    P with 5 granules per workgroup (5 sc1 stores; each poll reads all 5 by returning atomics)
//   T    B with ONE granule per workgroup (the product's polling: sc1 once, then returning-atomic
//        re-reads of the missing lanes, s_sleep(8) naps, an abort-word load per nap)
//   G    grid-stride tile order (wave w: tiles w, w + W, ...), rows after each tile: the memory
//        pattern of a pipelined pass that works through the capture in time order
// The row width W is a run-time argument (32 = the npr_flow row; 16 and 8 = compact encodings;
// 0 = no rows).  Every launch reads one of 4 capture copies (320 MB > the 256 MiB Infinity Cache)
// and writes the same table, as bench.py does.  HIP events over S back-to-back launches (us per
// launch, launch gaps included, like bench.py's kernel_ms); run under rocprofv3 --kernel-trace
// --stats for kernel durations.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/microbench/rw_floor.hip -o scripts/microbench/rw_floor
// Usage: rw_floor [S] [sweep|lookback|all|floor] [capture bytes (default 80000024)]
//   floor: R, L and P at W = 32 only (e.g. the per-record convert's bytes: 88 or 120 MB read)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef __attribute__((address_space(3))) void *lds_ptr_t;
typedef unsigned int u32x4 __attribute__((__vector_size__(16)));

constexpr uint32_t kTile = 4096, kWg = 16, kRing = 2, kSlotW = kTile / 4 + 64;
constexpr uint32_t kRowsPerTile = 51;
constexpr uint32_t kLine64 = 16;  // 8-B words per 128-B line

struct Args {
  const uint8_t *buf;
  uint64_t len;
  uint8_t *out;
  uint32_t ntiles, nwaves;
  uint32_t wbytes;  // row bytes per record (0, 8, 16, 32)
  uint32_t *ctr;    // H: arrival counter (monotonic over launches); A/B/C: the pacing counter
  uint32_t *flags;  // K: one word per workgroup (the launch tag)
  uint64_t *gran;   // P/S/A/B/C: one 128-B line per workgroup (granules {tag:16 | value:48})
  uint64_t *agr;    // A/C: one 128-B line per wave (4 granules)
  uint32_t target;  // H: counter value once every workgroup of this launch arrived; else the launch tag
  uint32_t *abort_; // set when a bounded wait gives up (never expected)
};

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void dma_tile(const Args &a, uint64_t lo, uint32_t *dst) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t avail = a.len > lo ? a.len - lo : 0;
  const uint32_t nb = avail < (uint64_t)(kTile + 128) ? (uint32_t)avail : kTile + 128;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void *)(a.buf + lo), 0, (int)((nb + 15u) & ~15u), 0x00020000);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + i * 256), 16, (lane + 64u * i) * 16u, 0, 0, 2);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + 1024), 4, kTile + lane * 4u, 0, 0, 2);
}
__device__ __forceinline__ void res_range(const Args &a, uint32_t v, uint32_t &c0, uint32_t &c1) {
  const uint32_t q = a.ntiles / a.nwaves, r = a.ntiles % a.nwaves;
  c0 = v * q + (v < r ? v : r);
  c1 = c0 + q + (v < r ? 1u : 0u);
}
// the rows of tile t: one block of 51 x W bytes, stored as whole-line 16-B chunks written through
// (sc1) through a buffer resource over exactly the block (its range check drops the chunks past it)
__device__ __forceinline__ void put_block(const Args &a, uint32_t t, uint32_t v) {
  const uint32_t nb = kRowsPerTile * a.wbytes;
  if (nb == 0) return;
  const uint32_t lane = threadIdx.x & 63u;
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + (uint64_t)t * nb), 0, (int)nb, 0x00020000);
  const u32x4 x{v, lane, v ^ lane, t};
  __builtin_amdgcn_raw_buffer_store_b128(x, rr, (int)(lane * 16u), 0, 16);
  if (nb > 1024u) __builtin_amdgcn_raw_buffer_store_b128(x, rr, (int)((lane + 64u) * 16u), 0, 16);
}
__device__ __forceinline__ bool timed_out(const Args &a, uint64_t t0) {
  if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s at 100 MHz
    __hip_atomic_store(a.abort_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return __hip_atomic_load(a.abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
__device__ __forceinline__ uint64_t ld_atomic(uint64_t *p) {
  return __hip_atomic_fetch_add(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// two granules in one 16-B write-through (sc1) store (R2: observed untorn on gfx950 for 16-B sc1 halves)
__device__ __forceinline__ void st16(uint64_t *p, uint64_t x, uint64_t y) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)p, 0, 16, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)}, rs, 0,
                                         0, 16);
}
__device__ __forceinline__ bool tg(uint64_t w, uint32_t tag);
// a workgroup's 5 granules: 8-B sc1 loads or returning atomics, or (WIDE) 16 + 16 + 8-B sc1 loads
template <bool WIDE, bool ATOMIC, int NG = 5>
__device__ __forceinline__ bool load5(uint64_t *g, uint32_t tag) {
  if (NG == 1) return tg(ATOMIC ? __hip_atomic_fetch_add(g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), tag);
  uint64_t x[5];
  if (ATOMIC) {
#pragma unroll
    for (int k = 0; k < 5; ++k) x[k] = __hip_atomic_fetch_add(g + k, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (WIDE) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)g, 0, 40, 0x00020000);
    const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rs, 0, 0, 16), v1 = __builtin_amdgcn_raw_buffer_load_b128(rs, 16, 0, 16);
    x[0] = ((uint64_t)v0[1] << 32) | v0[0], x[1] = ((uint64_t)v0[3] << 32) | v0[2];
    x[2] = ((uint64_t)v1[1] << 32) | v1[0], x[3] = ((uint64_t)v1[3] << 32) | v1[2];
    x[4] = __hip_atomic_load(g + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
#pragma unroll
    for (int k = 0; k < 5; ++k) x[k] = __hip_atomic_load(g + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return tg(x[0], tag) && tg(x[1], tag) && tg(x[2], tag) && tg(x[3], tag) && tg(x[4], tag);
}
__device__ __forceinline__ uint64_t gr(uint32_t tag, uint64_t v) { return ((uint64_t)tag << 48) | (v & ((1ull << 48) - 1)); }
__device__ __forceinline__ bool tg(uint64_t w, uint32_t tag) { return (uint32_t)(w >> 48) == (tag & 0xffffu); }

// MODE: see the header
template <char MODE>
__global__ __launch_bounds__(kWg * 64) void k_rw(Args a) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[kWg][kRing][kSlotW];
  __shared__ uint32_t fail;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t v = blockIdx.x * kWg + wid;
  uint32_t acc = lane;
  if (MODE == 'W') {
    uint32_t c0, c1;
    res_range(a, v, c0, c1);
    for (uint32_t t = c0; t < c1; ++t) put_block(a, t, acc);
    return;
  }
  if (MODE == 'G') {  // grid-stride over tiles, rows after each tile
    const uint32_t W = a.nwaves;
    uint32_t t = v, k = 0;
    if (t < a.ntiles) dma_tile(a, (uint64_t)t * kTile, ring[wid][0]);
    for (; t < a.ntiles; t += W, ++k) {
      if (t + W < a.ntiles) {
        dma_tile(a, (uint64_t)(t + W) * kTile, ring[wid][(k + 1) & 1]);
        __builtin_amdgcn_s_waitcnt(0x0F70 | 5);
      } else {
        __builtin_amdgcn_s_waitcnt(0x0F70);
      }
      wsync();
      acc += ring[wid][k & 1][lane * 16];
      put_block(a, t, acc);
      wsync();
    }
    return;
  }
  uint32_t c0, c1;
  res_range(a, v, c0, c1);
  if (c0 < c1) dma_tile(a, (uint64_t)c0 * kTile, ring[wid][0]);
  for (uint32_t t = c0, k = 0; t < c1; ++t, ++k) {
    if (t + 1 < c1) {
      dma_tile(a, (uint64_t)(t + 1) * kTile, ring[wid][(k + 1) & 1]);
      // vmcnt(5) retires the current tile (I: its stores are older than the next DMA too)
      __builtin_amdgcn_s_waitcnt(0x0F70 | 5);
    } else {
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    wsync();
    acc += ring[wid][k & 1][lane * 16];
    if (MODE == 'I') put_block(a, t, acc);
    wsync();
  }
  if (MODE == 'R') {
    if (acc == 0x12345678u) a.out[v] = (uint8_t)acc;
    return;
  }
  if (MODE == 'L') {
    for (uint32_t t = c0; t < c1; ++t) put_block(a, t, acc);
    return;
  }
  if (threadIdx.x == 0) fail = 0;
  __syncthreads();
  const uint32_t b = blockIdx.x, tag = a.target & 0xffffu;
  constexpr bool kLook = MODE == 'A' || MODE == 'B' || MODE == 'C' || MODE == 'D' || MODE == 'E' || MODE == 'F' ||
                        MODE == 'N' || MODE == 'T';
  constexpr int kNg = MODE == 'T' ? 1 : 5;  // granules per workgroup aggregate
  constexpr bool kSc1Poll = MODE == 'D' || MODE == 'E' || MODE == 'F' || MODE == 'N';
  constexpr bool kWide = MODE == 'E' || MODE == 'F' || MODE == 'N';
  if (MODE == 'A' || MODE == 'C') {  // every wave's A after the barrier (the product's order)
    if (lane == 0) {
      uint64_t *p = a.agr + (uint64_t)v * kLine64;
#pragma unroll
      for (int k = 0; k < 4; ++k) st_sc1(p + k, gr(tag, c0 + k));
    }
  }
  if (wid == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (MODE == 'H') {
      if (lane == 0) __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (;;) {
        const uint32_t c = __hip_atomic_fetch_add(a.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int32_t)(c - a.target) >= 0) break;
        if (timed_out(a, t0)) {
          fail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    } else if (MODE == 'K') {  // publish this workgroup's flag, wait for every lower workgroup's
      if (lane == 0) __hip_atomic_store(a.flags + blockIdx.x, a.target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (;;) {
        bool miss = false;
        for (uint32_t w0 = 0; w0 < b; w0 += 64) {
          const uint32_t i = w0 + lane;
          const uint32_t f = i < b ? __hip_atomic_fetch_add(a.flags + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                   : a.target;
          miss = miss || __ballot(f != a.target) != 0ull;
        }
        if (!miss) break;
        if (timed_out(a, t0)) {
          fail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    } else if (MODE == 'P' || MODE == 'S' || MODE == 'Q') {  // one (Q: five) 8-B granule(s) per workgroup, one line each
      if (lane == 0) {
        st_sc1(a.gran + (uint64_t)b * kLine64, gr(tag, b));
        if (MODE == 'Q')
#pragma unroll
          for (int k = 1; k < 5; ++k) st_sc1(a.gran + (uint64_t)b * kLine64 + k, gr(tag, b + k));
      }
      for (;;) {
        bool miss = false;
        for (uint32_t w0 = 0; w0 < b; w0 += 64) {
          const uint32_t i = w0 + lane;
          uint64_t *p = a.gran + (uint64_t)i * kLine64;
          bool got = true;
          if (i < b) {
            if (MODE == 'Q') {
              const uint64_t x0 = ld_atomic(p), x1 = ld_atomic(p + 1), x2 = ld_atomic(p + 2), x3 = ld_atomic(p + 3),
                             x4 = ld_atomic(p + 4);
              got = tg(x0, tag) && tg(x1, tag) && tg(x2, tag) && tg(x3, tag) && tg(x4, tag);
            } else {
              got = tg(MODE == 'P' ? ld_atomic(p) : ld_sc1(p), tag);
            }
          }
          miss = miss || __ballot(!got) != 0ull;
        }
        if (!miss) break;
        if (timed_out(a, t0)) {
          fail = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    } else if (kLook) {  // A ... N: the resident pass's G publication and look-back
      if (lane == 0) {
        uint64_t *g = a.gran + (uint64_t)b * kLine64;
        if (kWide) {
          st16(g, gr(tag, b), gr(tag, b + 1));
          st16(g + 2, gr(tag, b + 2), gr(tag, b + 3));
          st_sc1(g + 4, gr(tag, b + 4));
        } else {
#pragma unroll
          for (int k = 0; k < kNg; ++k) st_sc1(g + k, gr(tag, b + k));
        }
        if (MODE != 'N') (void)__hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      constexpr int kWin = 4;
      bool have[kWin];
#pragma unroll
      for (int w = 0; w < kWin; ++w) {  // every window once, sc1
        const uint32_t i = 64u * w + lane;
        have[w] = true;
        if (i < b) have[w] = load5<kWide, false, kNg>(a.gran + (uint64_t)i * kLine64, tag);
      }
      uint32_t nap = 1;
      for (int tries = 0;; ++tries) {
        bool miss = false;
#pragma unroll
        for (int w = 0; w < kWin; ++w) miss = miss || __ballot(!have[w]) != 0ull;
        if (!miss) break;
        if (tries) {
          if (kSc1Poll) {
            __builtin_amdgcn_s_sleep(4);
            if ((tries & 15) == 0 && timed_out(a, t0)) {
              fail = 1;
              break;
            }
          } else if (MODE == 'C') {
            __builtin_amdgcn_s_sleep(2);
            if ((tries & 15) == 0 && timed_out(a, t0)) {
              fail = 1;
              break;
            }
          } else {
            for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(8);
            nap = nap < 2u ? nap * 2u : 2u;
            if (timed_out(a, t0)) {
              fail = 1;
              break;
            }
          }
        }
#pragma unroll
        for (int w = 0; w < kWin; ++w) {
          const uint32_t i = 64u * w + lane;
          if (__ballot(!have[w])) {
            if (!have[w]) have[w] = load5<kWide, !kSc1Poll, kNg>(a.gran + (uint64_t)i * kLine64, tag);
          }
        }
      }
    }
  }
  __syncthreads();
  if (fail) return;
  if (MODE == 'F' && lane == 0) {  // the per-wave A stores, deferred past the look-back
    uint64_t *p = a.agr + (uint64_t)v * kLine64;
#pragma unroll
    for (int k = 0; k < 4; ++k) st_sc1(p + k, gr(tag, c0 + k));
  }
  for (uint32_t t = c0; t < c1; ++t) put_block(a, t, acc);
}

template <class F>
float timeit(F launch, int steps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 10; ++i) launch(i);
  CK(hipEventRecord(e0));
  for (int i = 0; i < steps; ++i) launch(10 + i);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / steps;  // us per launch
}

int main(int argc, char **argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 200;
  const char *what = argc > 2 ? argv[2] : "all";
  const bool sweep = !strcmp(what, "sweep") || !strcmp(what, "all");
  const bool look = !strcmp(what, "lookback") || !strcmp(what, "all");
  const bool floor_only = !strcmp(what, "floor");
  const uint64_t len = argc > 3 ? strtoull(argv[3], nullptr, 10) : 80000024ull;
  const uint32_t ntiles = (uint32_t)((len + kTile - 1) / kTile);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_rw<'A'>, kWg * 64, 0));
  const uint32_t nwg = (uint32_t)prop.multiProcessorCount;  // one per CU, all co-resident
  if (occ < 1 || nwg > 256) {
    fprintf(stderr, "occupancy %d, %u CUs: the grid cannot be co-resident / exceeds the windows\n", occ, nwg);
    return 1;
  }
  const uint32_t nwaves = nwg * kWg;
  uint8_t *bufs[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&bufs[i], len + 8192));
    CK(hipMemset(bufs[i], 0x11 * (i + 1), len + 8192));
  }
  uint8_t *out;
  CK(hipMalloc(&out, (size_t)ntiles * kRowsPerTile * 32 + 4096));
  uint32_t *ctl;  // [0] counter, [1] abort, [64..] flags
  CK(hipMalloc(&ctl, 4096 * 4));
  CK(hipMemset(ctl, 0, 4096 * 4));
  uint64_t *gran, *agr;
  CK(hipMalloc(&gran, (size_t)nwg * 128));
  CK(hipMemset(gran, 0, (size_t)nwg * 128));
  CK(hipMalloc(&agr, (size_t)nwaves * 128));
  CK(hipMemset(agr, 0, (size_t)nwaves * 128));
  CK(hipDeviceSynchronize());
  printf("rw_floor: %u CUs, occupancy %d WG/CU, %u waves, %u tiles, read %.1f MB\n", nwg, occ, nwaves, ntiles,
         len / 1e6);
  uint32_t launches = 0, h_launches = 0;
  char mode_now = 0;
  uint32_t wb_now = 32;
  auto arg = [&](int i) {
    Args x{};
    x.buf = bufs[i & 3];
    x.len = len;
    x.out = out;
    x.ntiles = ntiles;
    x.nwaves = nwaves;
    x.wbytes = wb_now;
    x.ctr = ctl;
    x.abort_ = ctl + 1;
    x.flags = ctl + 64;
    x.gran = gran;
    x.agr = agr;
    ++launches;
    if (mode_now == 'H') ++h_launches;
    // H: the counter after this launch's arrivals (only H launches add to it); else a fresh tag
    // (16-bit granule tags: never 0, which the zero-filled slots hold)
    x.target = mode_now == 'H' ? h_launches * nwg : (launches % 65535u) + 1u;
    return x;
  };
  const double rb = (double)len;
  auto rep = [&](const char *name, uint32_t wbytes, float us, double r) {
    const double w = (double)ntiles * kRowsPerTile * wbytes;
    printf("%-62s W=%2u %7.2f us  read %6.0f GB/s (read-only frac %.3f)  total %6.0f GB/s  frac(read+32B rows) %.3f\n",
           name, wbytes, us, r / (us * 1e-6) / 1e9, r / (us * 1e-6) / 8e12, (r + w) / (us * 1e-6) / 1e9,
           (rb + (double)ntiles * kRowsPerTile * 32) / (us * 1e-6) / 8e12);
  };
#define RUN(M, WB, name, r)                                                                                  \
  mode_now = M;                                                                                              \
  wb_now = WB;                                                                                               \
  rep(name, WB, timeit([&](int i) { hipLaunchKernelGGL(k_rw<M>, dim3(nwg), dim3(kWg * 64), 0, 0, arg(i)); }, S), r)
  for (int round = 0; round < 3; ++round) {
    printf("-- round %d\n", round);
    if (floor_only) {
      RUN('R', 0, "R read only", rb);
      RUN('L', 32, "L rows after the wave's own range (others still read)", rb);
      RUN('P', 32, "P 8-B granule per line, atomic polls", rb);
    }
    if (sweep) {
      RUN('R', 0, "R read only", rb);
      for (uint32_t wb : {32u, 16u, 8u}) {
        RUN('W', wb, "W write only", 0);
        RUN('I', wb, "I rows after each tile (independent of the reads)", rb);
        RUN('L', wb, "L rows after the wave's own range (others still read)", rb);
        RUN('K', wb, "K wait for lower workgroups only, then rows", rb);
        RUN('G', wb, "G grid-stride tiles, rows after each tile", rb);
      }
      RUN('K', 0, "K wait for lower workgroups only, no rows", rb);
      RUN('H', 32, "H one grid-wide hand-off, then rows", rb);
    }
    if (look) {
      RUN('K', 32, "K 4-B flags packed, atomic polls", rb);
      RUN('P', 32, "P 8-B granule per line, atomic polls", rb);
      RUN('S', 32, "S 8-B granule per line, sc1-load polls", rb);
      RUN('A', 32, "A resident pass's publication + look-back", rb);
      RUN('B', 32, "B = A without the per-wave A stores", rb);
      RUN('C', 32, "C = A with short naps, abort word every 16th", rb);
      RUN('D', 32, "D = B with sc1 re-polls, s_sleep(4)", rb);
      RUN('E', 32, "E = D with 16-B granule pairs", rb);
      RUN('F', 32, "F = E with the A stores after the look-back", rb);
      RUN('N', 32, "N = E without the arrival counter", rb);
      RUN('Q', 32, "Q = P with 5 granules per workgroup", rb);
      RUN('T', 32, "T = B with one granule per workgroup", rb);
      for (uint32_t wb : {16u, 8u, 0u}) {
        RUN('P', wb, "P 8-B granule per line, atomic polls", rb);
      }
    }
  }
#undef RUN
  uint32_t ab = 0;
  CK(hipMemcpy(&ab, ctl + 1, 4, hipMemcpyDeviceToHost));
  printf("abort word %u (0 = every bounded wait completed)\n", ab);
  return ab == 0 ? 0 : 3;
}
