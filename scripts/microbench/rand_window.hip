// rand_window — the memory side of the sparse walk on this MI355X: 80-B windows
// ([p & ~15, +80), five dwordx4 loads into registers) at record-like positions of a 6.4-GB buffer.
//   chain C : every lane walks C interleaved chains of its byte range, hop = 16 + (a loaded word
//             mod 1441 + 64): the next window depends on the current one (the walk's shape; C = 1
//             is the product's one window in flight per lane)
//   indep B : the same hop lengths precomputed (no dependency): B windows in flight per lane
// Prints per variant: ms, windows, 128-B lines touched, lines/s and line-GB/s.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/microbench/rand_window.hip -o scripts/microbench/rand_window
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 *gv4_t;

__device__ __forceinline__ uint32_t win_sum(const uint8_t *buf, uint64_t p, uint32_t &w0) {
  const gv4_t s = (gv4_t)(uintptr_t)(buf + (p & ~15ull));
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const u32x4 v = s[k];
    if (k == 0) w0 = v[0] ^ v[2];
    acc += v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  return acc;
}
__device__ __forceinline__ uint32_t lines_of(uint64_t p) { return 1u + ((((p & ~15ull) & 127u) + 80u) > 128u); }

// C chains per lane: lane range [lo, lo + span) cut into C equal parts, walked together.
// ST: 0 no stores; 1 a 32-B slot per window as k_sparse_walk writes them (slot k of lane j: row
// (g cap + k) 64 + j, two 16-B stores at a 32-B stride); 2 the same bytes as whole 1-KiB blocks
// (lane j stores 16-B pieces j and 64 + j of the 2-KiB slot row)
template <int C, int ST = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_chain(const uint8_t *buf, uint64_t span,
                                                                                        uint64_t nlanes, unsigned long long *out) {
  const uint64_t l = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (l >= nlanes) return;
  const uint64_t part = span / C;
  uint64_t pos[C], hi[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    pos[c] = l * span + c * part;
    hi[c] = pos[c] + part;
  }
  uint32_t acc = 0, n = 0, lines = 0;
  bool live = true;
  while (live) {
    live = false;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (pos[c] < hi[c]) {
        uint32_t w0;
        acc += win_sum(buf, pos[c], w0);
        lines += lines_of(pos[c]);
        ++n;
        if (ST) {
          u32x4 *slots = reinterpret_cast<u32x4 *>(out + 4);
          const uint64_t g = l >> 6, j = l & 63u, k = n < 96u ? n - 1u : 95u;
          u32x4 *row = slots + (g * 96u + k) * 128u;
          const u32x4 x = u32x4{acc, w0, n, lines};
          if (ST == 1) {
            row[2 * j] = x;
            row[2 * j + 1] = x;
          } else {
            row[j] = x;
            row[64 + j] = x;
          }
        }
        pos[c] += 16u + 64u + (w0 % 1441u);
        live = true;
      }
    }
  }
  atomicAdd(out, (unsigned long long)n);
  atomicAdd(out + 1, (unsigned long long)lines);
  atomicAdd(out + 2, (unsigned long long)acc);
}

// B independent windows in flight per lane: positions from a per-lane hash walk (no data dependency)
template <int B>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_indep(const uint8_t *buf, uint64_t span,
                                                                                        uint64_t nlanes, unsigned long long *out) {
  const uint64_t l = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (l >= nlanes) return;
  const uint64_t part = span / B;
  uint64_t pos[B], hi[B];
  uint32_t h[B];
#pragma unroll
  for (int c = 0; c < B; ++c) {
    pos[c] = l * span + c * part;
    hi[c] = pos[c] + part;
    h[c] = (uint32_t)(l * 2654435761u) ^ (uint32_t)(c * 40503u);
  }
  uint32_t acc = 0, n = 0, lines = 0;
  bool live = true;
  while (live) {
    live = false;
#pragma unroll
    for (int c = 0; c < B; ++c) {
      if (pos[c] < hi[c]) {
        uint32_t w0;
        acc += win_sum(buf, pos[c], w0);
        lines += lines_of(pos[c]);
        ++n;
        h[c] = h[c] * 1664525u + 1013904223u;
        pos[c] += 16u + 64u + ((h[c] >> 8) % 1441u);
        live = true;
      }
    }
  }
  atomicAdd(out, (unsigned long long)n);
  atomicAdd(out + 1, (unsigned long long)lines);
  atomicAdd(out + 2, (unsigned long long)acc);
}

// Persistent waves over small lane ranges in address order: wave w takes groups w, w + W, ... (64
// lanes of `span` bytes each), so at any moment the waves work inside one band of W x 64 x span
// bytes of the buffer instead of across all of it (the walk's lanes all start at once, spread over
// the whole capture).  SPEC: each lane first loads three dependent windows (the walk's start
// speculation: a screening window and two chained headers) before its chain.
template <int SPEC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_band(const uint8_t *buf, uint64_t span,
                                                                                       uint64_t nlanes, unsigned long long *out) {
  const uint64_t nw = (uint64_t)gridDim.x * 4u, w = (uint64_t)blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t acc = 0, n = 0, lines = 0;
  for (uint64_t g = w; g * 64 < nlanes; g += nw) {
    const uint64_t l = g * 64 + lane;
    if (l >= nlanes) continue;
    uint64_t pos = l * span;
    const uint64_t hi = pos + span;
    if (SPEC) {
      uint32_t w0;
      acc += win_sum(buf, pos, w0);
      uint64_t q = pos + 16u + (w0 % 61u);
      acc += win_sum(buf, q, w0);
      q += 16u + 64u + (w0 % 1441u);
      acc += win_sum(buf, q, w0);
      lines += lines_of(pos) + 2;
      acc += (uint32_t)q;
    }
    while (pos < hi) {
      uint32_t w0;
      acc += win_sum(buf, pos, w0);
      lines += lines_of(pos);
      ++n;
      pos += 16u + 64u + (w0 % 1441u);
    }
  }
  atomicAdd(out, (unsigned long long)n);
  atomicAdd(out + 1, (unsigned long long)lines);
  atomicAdd(out + 2, (unsigned long long)acc);
}

int main(int argc, char **argv) {
  const uint64_t bytes = 6400ull << 20;
  const uint64_t nlanes = argc > 1 ? strtoull(argv[1], 0, 0) : 160000ull;
  const uint64_t span = (bytes - 4096) / nlanes;
  uint8_t *buf;
  unsigned long long *out;
  CK(hipMalloc(&buf, bytes));
  const uint64_t slot_bytes = ((nlanes + 63) / 64) * 96ull * 2048ull;
  CK(hipMalloc(&out, 32 + slot_bytes));
  // random contents (a cheap device fill: hipMemset of a pattern would make every hop the same)
  {
    std::vector<uint32_t> h(1 << 24);
    uint32_t x = 12345;
    for (auto &v : h) v = (x = x * 1664525u + 1013904223u);
    for (uint64_t o = 0; o < bytes; o += h.size() * 4)
      CK(hipMemcpy(buf + o, h.data(), (bytes - o) < h.size() * 4 ? bytes - o : h.size() * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid0((unsigned)((nlanes + 255) / 256));
  dim3 grid = grid0;
  uint64_t span_run = span, nl_run = nlanes;
  auto run = [&](const char *name, void (*k)(const uint8_t *, uint64_t, uint64_t, unsigned long long *)) {
    float best = 1e30f;
    unsigned long long r[3] = {0, 0, 0};
    for (int it = 0; it < 4; ++it) {
      CK(hipMemset(out, 0, sizeof(r)));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(k, grid, dim3(256), 0, 0, buf, span_run, nl_run, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0 && ms < best) best = ms;
      CK(hipMemcpy(r, out, sizeof(r), hipMemcpyDeviceToHost));
    }
    printf("%-9s lanes %llu  %.3f ms  windows %.2fM  lines %.2fM (%.2f/window)  %.1f G lines/s  %.2f TB/s of lines\n", name,
           (unsigned long long)nl_run, best, r[0] / 1e6, r[1] / 1e6, (double)r[1] / r[0], r[1] / (best * 1e-3) / 1e9,
           r[1] * 128.0 / (best * 1e-3) / 1e12);
    fflush(stdout);
  };
  if (argc > 2 && std::string(argv[2]) == "band") {
    // persistent workgroups of 4 waves (argv[3]: how many; 1024 = 4 per CU) over lanes of S bytes
    grid = dim3(argc > 3 ? (unsigned)strtoul(argv[3], 0, 0) : 1024u);
    printf("persistent workgroups: %u (%u waves)\n", grid.x, grid.x * 4u);
    for (uint64_t S : {4096ull, 8192ull, 16384ull, 40960ull}) {
      span_run = S;
      nl_run = (bytes - 4096) / S;
      char nm[64];
      snprintf(nm, sizeof nm, "band%llu", (unsigned long long)S);
      run(nm, k_band<0>);
      snprintf(nm, sizeof nm, "band%llu+spec", (unsigned long long)S);
      run(nm, k_band<1>);
    }
    grid = grid0;
    span_run = span;
    nl_run = nlanes;
    run("chain1", k_chain<1>);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
  }
  run("chain1", k_chain<1>);
  run("chain2", k_chain<2>);
  run("chain1+slots", k_chain<1, 1>);
  run("chain1+blocks", k_chain<1, 2>);
  run("indep1", k_indep<1>);
  run("indep2", k_indep<2>);
  run("indep4", k_indep<4>);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
