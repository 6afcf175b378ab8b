# k_parse_resident: the extra tiles of an uneven split dealt round-robin over the workgroups (wave w of
# every workgroup before wave w + 1 of any), so every CU gets the same number of tiles +-1 (C2: 76 or
# 77 per workgroup instead of 80 for the first 196 workgroups and 64 for the rest).  Full workgroups
# only (nwaves a multiple of the workgroup size); otherwise the plain split.
a = """__device__ __forceinline__ void res_range(const ParseParams &kp, uint32_t v, uint32_t &c0, uint32_t &c1) {
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves;
  c0 = v * q + (v < r ? v : r);
  c1 = c0 + q + (v < r ? 1u : 0u);
}
// the wave whose range holds tile m
__device__ __forceinline__ uint32_t res_wave_of(const ParseParams &kp, int64_t m) {
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves;
  const uint64_t big = (uint64_t)r * (q + 1);
  return (uint64_t)m < big ? (uint32_t)((uint64_t)m / (q + 1)) : (uint32_t)(r + ((uint64_t)m - big) / q);
}"""
assert s.count(a) == 1
s = s.replace(a, """__device__ __forceinline__ void res_range(const ParseParams &kp, uint32_t v, uint32_t &c0, uint32_t &c1) {
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves;
  if (kp.nwaves % kResWg == 0) {
    const uint32_t nwg = kp.nwaves / kResWg, R = r / nwg, s = r % nwg, b = v / kResWg, w = v % kResWg;
    const uint32_t e = R + (b < s ? 1u : 0u);  // waves of workgroup b with q + 1 tiles (its oldest)
    c0 = v * q + b * R + (b < s ? b : s) + (w < e ? w : e);
    c1 = c0 + q + (w < e ? 1u : 0u);
    return;
  }
  c0 = v * q + (v < r ? v : r);
  c1 = c0 + q + (v < r ? 1u : 0u);
}
// the wave whose range holds tile m
__device__ __forceinline__ uint32_t res_wave_of(const ParseParams &kp, int64_t m) {
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves;
  if (kp.nwaves % kResWg == 0) {
    const uint32_t nwg = kp.nwaves / kResWg, R = r / nwg, s = r % nwg;
    const uint64_t tw = (uint64_t)kResWg * q + R, big = (uint64_t)s * (tw + 1);
    const uint32_t b = (uint64_t)m < big ? (uint32_t)((uint64_t)m / (tw + 1)) : (uint32_t)(s + ((uint64_t)m - big) / tw);
    const uint64_t sb = (uint64_t)b * tw + (b < s ? b : s), l = (uint64_t)m - sb;
    const uint32_t e = R + (b < s ? 1u : 0u);
    const uint64_t bigw = (uint64_t)e * (q + 1);
    const uint32_t w = l < bigw ? (uint32_t)(l / (q + 1)) : (uint32_t)(e + (l - bigw) / q);
    return b * kResWg + w;
  }
  const uint64_t big = (uint64_t)r * (q + 1);
  return (uint64_t)m < big ? (uint32_t)((uint64_t)m / (q + 1)) : (uint32_t)(r + ((uint64_t)m - big) / q);
}""")
