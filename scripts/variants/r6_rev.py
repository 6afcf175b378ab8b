# k_parse_resident: the extra tiles of an uneven split go to the LAST ntiles % nwaves waves instead
# of the first, so the lower workgroups (whose aggregates every higher one waits for) finish their
# phase A first and write their rows while the higher ones still read
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
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves, s0 = kp.nwaves - r;  // waves >= s0: q + 1
  c0 = v * q + (v > s0 ? v - s0 : 0u);
  c1 = c0 + q + (v >= s0 ? 1u : 0u);
}
// the wave whose range holds tile m
__device__ __forceinline__ uint32_t res_wave_of(const ParseParams &kp, int64_t m) {
  const uint32_t q = kp.ntiles / kp.nwaves, r = kp.ntiles % kp.nwaves, s0 = kp.nwaves - r;
  const uint64_t small = (uint64_t)s0 * q;
  return (uint64_t)m < small ? (uint32_t)((uint64_t)m / q) : (uint32_t)(s0 + ((uint64_t)m - small) / (q + 1));
}""")
