// Microbenchmark of the parse kernels' skeleton: persistent one-wave workgroups, each owning a
// contiguous run of 4 KiB tiles, 2-deep register prefetch (16-B buffer loads), LDS commit.
// MODE 0: commit only; 1: + one LDS read per lane per tile (checksum); 2: + 17-word window
// reads per lane (the decode_fast window).  Prints GB/s per mode for 80 MB (and 4 rotating copies).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef unsigned int u32x4 __attribute__((__vector_size__(16)));
constexpr int kTile = 4096, kStage = 4224, kChunks = (kStage / 16 + 63) / 64;

__device__ __forceinline__ void issue(const uint8_t *buf, uint64_t len, uint64_t lo, u32x4 (&q)[kChunks]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t avail = len > lo ? len - lo : 0;
  const uint32_t nb = avail < (uint64_t)kStage ? (uint32_t)avail : (uint32_t)kStage;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(buf + lo), 0, (int)((nb + 15u) & ~15u), 0x00020000);
#pragma unroll
  for (int i = 0; i < kChunks; ++i) q[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((lane + 64u * i) * 16u), 0, 0);
}
__device__ __forceinline__ void commit(uint32_t *d, const u32x4 (&q)[kChunks]) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int i = 0; i < kChunks; ++i) {
    const uint32_t c = lane + 64u * i;
    if (c < kStage / 16) *reinterpret_cast<u32x4 *>(&d[c * 4]) = q[i];
  }
}

template <int MODE>
__global__ __launch_bounds__(64) void k_stream(const uint8_t *buf, uint64_t len, uint32_t nt, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint32_t d[kStage / 4 + 32];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t c0 = (uint64_t)blockIdx.x * nt / gridDim.x, c1 = (uint64_t)(blockIdx.x + 1) * nt / gridDim.x;
  if (c0 >= c1) return;
  u32x4 qa[kChunks], qb[kChunks];
  issue(buf, len, (uint64_t)c0 * kTile, qa);
  if (c0 + 1 < c1) issue(buf, len, (uint64_t)(c0 + 1) * kTile, qb);
  uint32_t acc = 0;
  auto step = [&](uint32_t t, u32x4 (&q)[kChunks]) {
    commit(d, q);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (t + 2 < c1) issue(buf, len, (uint64_t)(t + 2) * kTile, q);
    if (MODE >= 1) acc += d[lane * 16];
    if (MODE >= 2) {
      const uint32_t rel = lane * 80u + 16u;
      const uint32_t *p = d + (rel >> 2);
#pragma unroll
      for (int k = 0; k < 17; ++k) acc ^= __builtin_amdgcn_alignbyte(p[k + 1], p[k], rel & 3u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  for (uint32_t t = c0; t < c1; t += 2) {
    step(t, qa);
    if (t + 1 < c1) step(t + 1, qb);
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int MODE>
float run(uint8_t **bufs, int nb, uint64_t len, int grid, uint32_t *out) {
  const uint32_t nt = (uint32_t)((len + kTile - 1) / kTile);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_stream<MODE>, dim3(grid), dim3(64), 0, 0, bufs[i % nb], len, nt, out);
  hipEventRecord(a);
  const int steps = 50;
  for (int i = 0; i < steps; ++i) hipLaunchKernelGGL(k_stream<MODE>, dim3(grid), dim3(64), 0, 0, bufs[i % nb], len, nt, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / steps;
}

int main() {
  const uint64_t len = 80000024;
  uint8_t *bufs[4];
  for (int i = 0; i < 4; ++i) {
    hipMalloc(&bufs[i], len + 4096);
    hipMemset(bufs[i], i + 1, len + 4096);
  }
  uint32_t *out;
  hipMalloc(&out, 1 << 20);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  int per_cu[3];
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[0], k_stream<0>, 64, 0);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[1], k_stream<1>, 64, 0);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu[2], k_stream<2>, 64, 0);
  for (int waves : {4, 8, 12, 16, 24, 32}) {
    const int grid = prop.multiProcessorCount * waves;
    float t0 = run<0>(bufs, 4, len, grid, out), t1 = run<1>(bufs, 4, len, grid, out), t2 = run<2>(bufs, 4, len, grid, out);
    float s0 = run<0>(bufs, 1, len, grid, out);
    printf("waves/CU %2d (occ %d/%d/%d): commit %.1f us (%.0f GB/s) | +read %.1f us | +window %.1f us | same-buffer commit %.1f us (%.0f GB/s)\n",
           waves, per_cu[0], per_cu[1], per_cu[2], t0 * 1e3, len / (t0 * 1e-3) / 1e9, t1 * 1e3, t2 * 1e3, s0 * 1e3, len / (s0 * 1e-3) / 1e9);
  }
  return 0;
}
