// store_pattern — does the way k_parse_resident's phase B stores its 32-B flow rows cost write
// bandwidth?  Every variant writes the same bytes: 4096 persistent waves (256 workgroups x 16) each
// write their contiguous share of a buffer of 32-B rows, 64 rows per wave round.
//   rows   : lane l writes row l of the round as two dwordx4 stores (bytes 0-15, then 16-31): each
//            store instruction touches 64 half rows at a 32-B stride (the kernel's pattern)
//   contig : the same 2 KB per round as two fully contiguous 1 KB stores (lane i writes bytes
//            16 i .. 16 i + 15 of each half of the round)
//   lds    : rows staged through LDS and stored contiguously (what a transpose in the kernel costs)
//   rows_w / contig_w : rows / contig with s_waitcnt vmcnt(0) after each round (stores drained
//            before the next round issues)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/microbench/store_pattern.hip -o scripts/microbench/store_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(1024) void k_store(uint4 *out, uint64_t rows_per_wave, uint32_t seed) {
  __shared__ uint4 stage[16][128];
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * 16 + wid;
  uint4 *base = out + w * rows_per_wave * 2;  // 2 uint4 per row
  for (uint64_t r0 = 0; r0 < rows_per_wave; r0 += 64) {
    const uint32_t v = seed ^ (uint32_t)(r0 + lane);
    const uint4 a = make_uint4(v, v + 1, v + 2, v + 3), b = make_uint4(v + 4, v + 5, v + 6, v + 7);
    uint4 *blk = base + r0 * 2;
    if (MODE == 0 || MODE == 3) {
      blk[2 * lane] = a;
      blk[2 * lane + 1] = b;
      if (MODE == 3) __builtin_amdgcn_s_waitcnt(0x0F70);
    } else if (MODE == 1 || MODE == 4) {  // the same bytes land contiguously per instruction (values differ: timing only)
      blk[lane] = a;
      blk[64 + lane] = b;
      if (MODE == 4) __builtin_amdgcn_s_waitcnt(0x0F70);
    } else {
      stage[wid][2 * lane] = a;
      stage[wid][2 * lane + 1] = b;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint4 c = stage[wid][lane], d = stage[wid][64 + lane];
      blk[lane] = c;
      blk[64 + lane] = d;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  }
}

int main() {
  const uint64_t waves = 4096;
  for (uint64_t mb : {32ull, 320ull}) {
    const uint64_t bytes = mb << 20, rows = bytes / 32, per = (rows / waves + 63) / 64 * 64;
    uint4 *out;
    CK(hipMalloc(&out, waves * per * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 5; ++mode) {
      auto launch = [&](uint32_t s) {
        if (mode == 0) hipLaunchKernelGGL(k_store<0>, dim3(256), dim3(1024), 0, 0, out, per, s);
        else if (mode == 1) hipLaunchKernelGGL(k_store<1>, dim3(256), dim3(1024), 0, 0, out, per, s);
        else if (mode == 2) hipLaunchKernelGGL(k_store<2>, dim3(256), dim3(1024), 0, 0, out, per, s);
        else if (mode == 3) hipLaunchKernelGGL(k_store<3>, dim3(256), dim3(1024), 0, 0, out, per, s);
        else hipLaunchKernelGGL(k_store<4>, dim3(256), dim3(1024), 0, 0, out, per, s);
      };
      for (int i = 0; i < 3; ++i) launch(i);
      CK(hipDeviceSynchronize());
      const int reps = 20;
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) launch(100 + i);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / reps, tbps = waves * per * 32 / (us * 1e-6) / 1e12;
      printf("{\"MB\": %llu, \"mode\": \"%s\", \"us\": %.2f, \"TBps\": %.2f}\n", (unsigned long long)mb,
             mode == 0 ? "rows" : mode == 1 ? "contig" : mode == 2 ? "lds" : mode == 3 ? "rows_w" : "contig_w", us, tbps);
    }
    CK(hipFree(out));
  }
  return 0;
}
