// req_size — which load forms make the L2 fetch less than a 128-B line from memory: 8M independent
// 16-B (or 4-B) loads at random positions (offset 0 or 64 of a random line) of a 2-GB buffer, one
// kernel per load form, timed by HIP events; run under rocprofv3 --pmc TCC_EA0_RDREQ_{32B,64B,128B}
// to see the request sizes.
//   D global_load_dwordx4 (default policy)     N nontemporal (nt)
//   S global_load_dwordx4 sc1                  U global_load_dwordx4 sc0 sc1
//   W global_load_dword (4 B per lane)
// Build: hipcc -O3 --offload-arch=gfx950 scripts/microbench/req_size.hip -o scripts/microbench/req_size
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kPer = 8;

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

template <char M>
__global__ __launch_bounds__(256) void k_req(const uint8_t *buf, uint64_t nlines, uint32_t *out, uint32_t salt) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t acc = 0, bad = 0;
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const uint64_t h = mix(t * kPer + j + ((uint64_t)salt << 40));
    const uint64_t p = (h % nlines) * 128 + ((h >> 62) & 1) * 64;
    const uint8_t *a = buf + p;
    if (M == 'D') {
      const u32x4 v = *(const __attribute__((address_space(1))) u32x4 *)(uintptr_t)a;
      acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    } else if (M == 'N') {
      const u32x4 v = __builtin_nontemporal_load((const u32x4 *)a);
      acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    } else if (M == 'S') {
      u32x4 v;
      asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(a) : "memory");
      acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    } else if (M == 'U') {
      u32x4 v;
      asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(a) : "memory");
      acc += v[0] ^ v[1] ^ v[2] ^ v[3];
    } else if (M == 'H') {  // 64 B at a random BYTE position: four unaligned dwordx4 loads
      const uint64_t pb = h % (nlines * 128 - 64);
      const __attribute__((address_space(1))) u32x4 *q = (const __attribute__((address_space(1))) u32x4 *)(uintptr_t)(buf + pb);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const u32x4 v = q[k];
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        if (k == 0) {  // the byte pattern buf[i] = i * 7 (mod 256): the first word must match it
          const uint32_t b0 = (uint32_t)(pb * 7), want = (b0 & 255) | ((b0 + 7) & 255) << 8 | ((b0 + 14) & 255) << 16 | ((b0 + 21) & 255) << 24;
          bad += v[0] != want;
        }
      }
    } else if (M == 'F' || M == 'G') {  // an 80-B (F) / 64-B (G) window at a random 16-B aligned position
      const uint8_t *w = buf + ((h % (nlines * 8 - 8)) * 16);
      const __attribute__((address_space(1))) u32x4 *q = (const __attribute__((address_space(1))) u32x4 *)(uintptr_t)w;
#pragma unroll
      for (int k = 0; k < (M == 'F' ? 5 : 4); ++k) {
        const u32x4 v = q[k];
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
      }
    } else {
      acc += *(const __attribute__((address_space(1))) uint32_t *)(uintptr_t)a;
    }
  }
  out[t] = M == 'H' ? (bad << 24) + (acc & 0xffffffu) : acc;
}

__global__ void k_fill(uint8_t *buf, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) buf[i] = (uint8_t)(i * 7);
}

template <char M>
float run(const uint8_t *buf, uint64_t nlines, uint32_t *out, uint32_t threads) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_req<M>, dim3(threads / 256), dim3(256), 0, 0, buf, nlines, out, 1u);
  CK(hipEventRecord(e0));
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k_req<M>, dim3(threads / 256), dim3(256), 0, 0, buf, nlines, out, 2u + i);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / 5;
}

int main(int argc, char **argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 2.0;  // buffer size in GiB (TLB reach: DESIGN.md §5.2)
  const uint64_t bytes = (uint64_t)(gb * (1ull << 30)) & ~127ull, nlines = bytes / 128;
  printf("buffer %.1f GiB\n", gb);
  const uint32_t threads = 1u << 20;
  uint8_t *buf;
  uint32_t *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, threads * 4ull));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, bytes);
  CK(hipDeviceSynchronize());
  const double loads = (double)threads * kPer;
  auto show = [&](const char *name, float us) {
    printf("%-28s %8.1f us  %6.2f G loads/s  %7.1f GB/s of 128-B lines\n", name, us, loads / us / 1e3,
           loads * 128 / us / 1e3);
  };
  show("D dwordx4", run<'D'>(buf, nlines, out, threads));
  {  // windows: lines touched = 1 + P(the window crosses a line end)
    const float f = run<'F'>(buf, nlines, out, threads), g = run<'G'>(buf, nlines, out, threads);
    const double lf = loads * (1.0 + 79.0 / 128.0 * 0 + (8.0 - 3.0) / 8.0), lg = loads * (1.0 + (8.0 - 4.0) / 8.0);
    printf("%-28s %8.1f us  %6.2f G windows/s %6.2f G lines/s\n", "F 80-B windows (5 x dwordx4)", f, loads / f / 1e3, lf / f / 1e3);
    printf("%-28s %8.1f us  %6.2f G windows/s %6.2f G lines/s\n", "G 64-B windows (4 x dwordx4)", g, loads / g / 1e3, lg / g / 1e3);
    const float hh = run<'H'>(buf, nlines, out, threads);
    uint32_t *ho = (uint32_t *)malloc(threads * 4ull);
    CK(hipMemcpy(ho, out, threads * 4ull, hipMemcpyDeviceToHost));
    uint64_t nbad = 0;
    for (uint32_t i = 0; i < threads; ++i) nbad += ho[i] >> 24;
    free(ho);
    printf("%-28s %8.1f us  %6.2f G windows/s %6.2f G lines/s  (%llu wrong words)\n", "H 64 B unaligned (4 x dwordx4)", hh,
           loads / hh / 1e3, loads * (1.0 + 63.0 / 128.0) / hh / 1e3, (unsigned long long)nbad);
  }
  if (argc > 2) {  // sizes sweep: the default form only
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
  }
  show("N dwordx4 nt", run<'N'>(buf, nlines, out, threads));
  show("S dwordx4 sc1", run<'S'>(buf, nlines, out, threads));
  show("U dwordx4 sc0 sc1", run<'U'>(buf, nlines, out, threads));
  show("W dword", run<'W'>(buf, nlines, out, threads));
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
