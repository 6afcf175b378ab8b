// dma_ring — what streaming pattern reaches HBM bandwidth on this MI355X (no parsing at all).
// Every variant reads a 1 GiB buffer once; W persistent waves each own a contiguous range, as
// k_parse_resident's phase A does.  Prints GB/s per variant.
//   reg   : global_load_dwordx4 to registers, K loads per lane in flight
//   dma R : buffer_load_dwordx4 ... lds into an R-slot ring of 4 KiB tiles per wave (R-1 in flight)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/microbench/dma_ring.hip -o scripts/microbench/dma_ring
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef __attribute__((address_space(3))) void *lds_ptr_t;
constexpr int kTile = 4096;

template <int K>
__global__ __launch_bounds__(1024) void k_reg(const uint4 *buf, uint64_t n16, uint64_t per_wave, unsigned *sink) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const uint64_t lo = w * per_wave, hi = lo + per_wave < n16 ? lo + per_wave : n16;
  uint32_t acc = 0;
  for (uint64_t i = lo + lane; i < hi; i += 64 * K) {
    uint4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = i + 64 * k < hi ? buf[i + 64 * k] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < K; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int R, int AUX>
__global__ __launch_bounds__(1024) void k_dma(const uint8_t *buf, uint64_t len, uint64_t tiles_per_wave, unsigned *sink) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  uint32_t *ring = lds + wid * R * (kTile / 4);
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x / 64) + wid;
  const uint64_t t0 = w * tiles_per_wave;
  auto dma = [&](uint64_t t, uint32_t *dst) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(buf + t * kTile), 0, kTile, 0x00020000);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(dst + i * 256), 16, (lane + 64u * i) * 16u, 0, 0, AUX);
  };
  uint32_t acc = 0;
  const uint64_t nt = tiles_per_wave;
#pragma unroll
  for (int k = 0; k < R - 1; ++k)
    if ((uint64_t)k < nt) dma(t0 + k, ring + k * (kTile / 4));
  for (uint64_t k = 0; k < nt; ++k) {
    if (k + R - 1 < nt) dma(t0 + k + R - 1, ring + ((k + R - 1) % R) * (kTile / 4));
    // wait for tile k: the younger DMAs (up to R-1 tiles x 4 instructions) may stay in flight
    const uint64_t ahead = nt - 1 - k < (uint64_t)(R - 1) ? nt - 1 - k : (uint64_t)(R - 1);
    if (ahead == 0) __builtin_amdgcn_s_waitcnt(0x0F70);
    else if (ahead == 1) __builtin_amdgcn_s_waitcnt(0x0F70 | 4);
    else if (ahead == 2) __builtin_amdgcn_s_waitcnt(0x0F70 | 8);
    else __builtin_amdgcn_s_waitcnt(0x0F70 | 12);
    __builtin_amdgcn_wave_barrier();
    acc ^= ring[(k % R) * (kTile / 4) + lane];
    __builtin_amdgcn_wave_barrier();
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
  const uint64_t len = (argc > 1 ? strtoull(argv[1], 0, 10) : 1024ull) << 20;
  uint8_t *buf;
  unsigned *sink;
  CK(hipMalloc(&buf, len));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, len));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %8.1f GB/s  (%.3f ms per GiB pass)\n", name, len / (ms / reps * 1e-3) / 1e9, ms / reps);
    fflush(stdout);
  };
  const uint64_t n16 = len / 16;
  for (int wg : {256, 512, 1024}) {
    const uint64_t waves = (uint64_t)wg * 16;
    const uint64_t per = (n16 + waves - 1) / waves;
    char nm[64];
    snprintf(nm, sizeof nm, "reg K=4 waves=%llu", (unsigned long long)waves);
    timeit(nm, [&] { hipLaunchKernelGGL(k_reg<4>, dim3(wg), dim3(1024), 0, 0, (const uint4 *)buf, n16, per, sink); });
    snprintf(nm, sizeof nm, "reg K=8 waves=%llu", (unsigned long long)waves);
    timeit(nm, [&] { hipLaunchKernelGGL(k_reg<8>, dim3(wg), dim3(1024), 0, 0, (const uint4 *)buf, n16, per, sink); });
  }
  const uint64_t ntiles = len / kTile;
  auto dma_case = [&](auto kern, int R, int wpb, const char *tag) {
    const int wgs = 256;  // one workgroup of wpb waves per CU
    const uint64_t waves = (uint64_t)wgs * wpb;
    const uint64_t tpw = ntiles / waves;
    const size_t shm = (size_t)wpb * R * kTile;
    char nm[64];
    snprintf(nm, sizeof nm, "dma R=%d waves/CU=%d %s", R, wpb, tag);
    timeit(nm, [&] { hipLaunchKernelGGL(kern, dim3(wgs), dim3(wpb * 64), shm, 0, buf, len, tpw, sink); });
  };
  CK(hipFuncSetAttribute((const void *)k_dma<2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void *)k_dma<2, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void *)k_dma<3, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void *)k_dma<4, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  dma_case(k_dma<2, 2>, 2, 16, "nt");
  dma_case(k_dma<2, 0>, 2, 16, "plain");
  dma_case(k_dma<3, 2>, 3, 12, "nt");
  dma_case(k_dma<4, 2>, 4, 8, "nt");
  dma_case(k_dma<4, 2>, 4, 9, "nt");
  dma_case(k_dma<3, 2>, 3, 8, "nt");
  return 0;
}
