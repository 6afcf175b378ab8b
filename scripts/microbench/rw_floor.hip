// rw_floor — the combined read + write floor of the C2 launch on this MI355X:
// read the 80 MB capture and write the 32 MB flow table in ONE kernel, in the resident pass's
// geometry (256 workgroups x 16 waves, one per CU; each wave a contiguous range of 4 KiB tiles
// through a two-slot LDS-DMA ring, nt loads; rows stored as whole-line sc1 blocks of 51 rows x 32 B
// per tile, the resident pass's phase-B store).  Nothing is parsed: this is the memory system alone.
//   R    read only
//   W    write only (the 32 MB, each wave its ranges' blocks)
//   I    writes independent of the reads: each tile's rows are stored right after it lands
//   L    each wave stores its range's rows after its own last tile (other waves still read)
//   H    one grid-wide hand-off (every workgroup arrives on one counter after its reads, wave 0
//        polls it by returning atomics + s_sleep), then the rows
//   K    the look-back's dependency without the fold: workgroup b waits for workgroups 0..b-1
//        only (a flag per workgroup, a window read by wave 0), then its rows
//   G    grid-stride tile order (wave w: tiles w, w + W, ...), rows after each tile: the memory
//        pattern of a pipelined pass that works through the capture in time order
// Every launch reads one of 4 capture copies (320 MB > the 256 MiB Infinity Cache) and writes the
// same 32 MB table, as bench.py does.  HIP events over S back-to-back launches (us per launch,
// launch gaps included, like bench.py's kernel_ms); run under rocprofv3 --kernel-trace --stats for
// kernel durations.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/microbench/rw_floor.hip -o scripts/microbench/rw_floor
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
constexpr uint32_t kRowsPerTile = 51, kRowBytes = 32, kBlock = kRowsPerTile * kRowBytes;  // 1632 B

struct Args {
  const uint8_t *buf;
  uint64_t len;
  uint8_t *out;
  uint32_t ntiles, nwaves;
  uint32_t *ctr;    // H: arrival counter (monotonic over launches)
  uint32_t *flags;  // K: one word per workgroup (the launch index + 1 once published)
  uint32_t target;  // H: counter value once every workgroup of this launch arrived; K: the launch tag
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
// the rows of tile t: one 1632-B block, stored as whole-line 16-B chunks written through (sc1)
__device__ __forceinline__ void put_block(const Args &a, uint32_t t, uint32_t v) {
  const uint32_t lane = threadIdx.x & 63u;
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc((void *)(a.out + (uint64_t)t * kBlock), 0, (int)kBlock, 0x00020000);
  const u32x4 x{v, lane, v ^ lane, t};
  __builtin_amdgcn_raw_buffer_store_b128(x, rr, (int)(lane * 16u), 0, 16);
  __builtin_amdgcn_raw_buffer_store_b128(x, rr, (int)((lane + 64u) * 16u), 0, 16);
}
__device__ __forceinline__ bool timed_out(const Args &a, uint64_t t0) {
  if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s at 100 MHz
    __hip_atomic_store(a.abort_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  return __hip_atomic_load(a.abort_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// MODE: 'R', 'W', 'I', 'L', 'H', 'K', 'G'
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
      // vmcnt(5) retires the current tile (I: its two stores are older than the next DMA too)
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
  if (MODE == 'H' || MODE == 'K') {
    if (threadIdx.x == 0) fail = 0;
    __syncthreads();
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
      } else {  // K: publish this workgroup's flag, wait for every lower workgroup's
        if (lane == 0) __hip_atomic_store(a.flags + blockIdx.x, a.target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t b = blockIdx.x;
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
      }
    }
    __syncthreads();
    if (fail) return;
    for (uint32_t t = c0; t < c1; ++t) put_block(a, t, acc);
  }
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
  const uint64_t len = 80000024;
  const uint32_t ntiles = (uint32_t)((len + kTile - 1) / kTile);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_rw<'H'>, kWg * 64, 0));
  const uint32_t nwg = (uint32_t)prop.multiProcessorCount;  // one per CU, all co-resident
  if (occ < 1) {
    fprintf(stderr, "occupancy %d: the grid cannot be co-resident\n", occ);
    return 1;
  }
  const uint32_t nwaves = nwg * kWg;
  uint8_t *bufs[4];
  for (int i = 0; i < 4; ++i) {
    CK(hipMalloc(&bufs[i], len + 8192));
    CK(hipMemset(bufs[i], 0x11 * (i + 1), len + 8192));
  }
  uint8_t *out;
  CK(hipMalloc(&out, (size_t)ntiles * kBlock + 4096));
  uint32_t *ctl;  // [0] counter, [1] abort, [64..] flags
  CK(hipMalloc(&ctl, 4096 * 4));
  CK(hipMemset(ctl, 0, 4096 * 4));
  CK(hipDeviceSynchronize());
  printf("rw_floor: %u CUs, occupancy %d WG/CU, %u waves, %u tiles, read %.1f MB, write %.1f MB\n", nwg, occ, nwaves,
         ntiles, len / 1e6, (double)ntiles * kBlock / 1e6);
  uint32_t launches = 0, h_launches = 0;
  char mode_now = 0;
  auto arg = [&](int i) {
    Args x{};
    x.buf = bufs[i & 3];
    x.len = len;
    x.out = out;
    x.ntiles = ntiles;
    x.nwaves = nwaves;
    x.ctr = ctl;
    x.abort_ = ctl + 1;
    x.flags = ctl + 64;
    ++launches;
    if (mode_now == 'H') ++h_launches;
    // H: the counter after this launch's arrivals (only H launches add to it); K: a fresh tag
    x.target = mode_now == 'H' ? h_launches * nwg : launches;
    return x;
  };
  const double rb = (double)len, wb = (double)ntiles * kBlock;
  auto rep = [&](const char *name, float us, double r, double w) {
    printf("%-58s %7.2f us  read %6.0f GB/s  total %6.0f GB/s  frac(112MB) %.3f\n", name, us, r / (us * 1e-6) / 1e9,
           (r + w) / (us * 1e-6) / 1e9, 112000024.0 / (us * 1e-6) / 8e12);
  };
  for (int round = 0; round < 3; ++round) {
    printf("-- round %d\n", round);
#define RUN(M, name, r, w) \
  mode_now = M;            \
  rep(name, timeit([&](int i) { hipLaunchKernelGGL(k_rw<M>, dim3(nwg), dim3(kWg * 64), 0, 0, arg(i)); }, S), r, w)
    RUN('R', "R read only", rb, 0);
    RUN('W', "W write only", 0, wb);
    RUN('I', "I rows after each tile (independent of the reads)", rb, wb);
    RUN('L', "L rows after the wave's own range (others still read)", rb, wb);
    RUN('H', "H one grid-wide hand-off, then rows", rb, wb);
    RUN('K', "K wait for lower workgroups only, then rows", rb, wb);
    RUN('G', "G grid-stride tiles, rows after each tile", rb, wb);
#undef RUN
  }
  uint32_t ab = 0;
  CK(hipMemcpy(&ab, ctl + 1, 4, hipMemcpyDeviceToHost));
  printf("abort word %u (0 = every bounded wait completed)\n", ab);
  return 0;
}
