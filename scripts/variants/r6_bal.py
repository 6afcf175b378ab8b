# k_parse_resident: tiles dealt per WORKGROUP first (every CU gets ntiles / nwg tiles, +1 for the
# first ntiles % nwg), then over the workgroup's 16 waves, when the waves fill whole workgroups;
# otherwise the per-wave split.  32-bit arithmetic only (round 5's res_bal variant did the inverse
# map in 64 bits and gained a 40-B private segment).  C2: CUs hold 76-77 tiles instead of 80 / 64.
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
s = s.replace(a, """// [c0, c1) = the n items of a split of `total` items over `parts` parts, part i: total / parts
// each, one more for the first total % parts
__device__ __forceinline__ void split_range(uint32_t total, uint32_t parts, uint32_t i, uint32_t &c0, uint32_t &c1) {
  const uint32_t q = total / parts, r = total % parts;
  c0 = i * q + (i < r ? i : r);
  c1 = c0 + q + (i < r ? 1u : 0u);
}
// the part of such a split that holds item m
__device__ __forceinline__ uint32_t split_of(uint32_t total, uint32_t parts, uint32_t m) {
  const uint32_t q = total / parts, r = total % parts, big = r * (q + 1u);
  return m < big ? m / (q + 1u) : r + (m - big) / q;
}
__device__ __forceinline__ void res_range(const ParseParams &kp, uint32_t v, uint32_t &c0, uint32_t &c1) {
  if ((kp.nwaves & (kResWg - 1u)) == 0) {  // whole workgroups: per workgroup, then per wave
    uint32_t g0, g1;
    split_range(kp.ntiles, kp.nwaves / kResWg, v / kResWg, g0, g1);
    split_range(g1 - g0, kResWg, v % kResWg, c0, c1);
    c0 += g0;
    c1 += g0;
    return;
  }
  split_range(kp.ntiles, kp.nwaves, v, c0, c1);
}
// the wave whose range holds tile m
__device__ __forceinline__ uint32_t res_wave_of(const ParseParams &kp, int64_t m) {
  if ((kp.nwaves & (kResWg - 1u)) == 0) {
    const uint32_t b = split_of(kp.ntiles, kp.nwaves / kResWg, (uint32_t)m);
    uint32_t g0, g1;
    split_range(kp.ntiles, kp.nwaves / kResWg, b, g0, g1);
    return b * kResWg + split_of(g1 - g0, kResWg, (uint32_t)m - g0);
  }
  return split_of(kp.ntiles, kp.nwaves, (uint32_t)m);
}""")
# a workgroup aggregate's tiles straight from the per-workgroup split (not two per-wave splits)
a = """  uint32_t c0, c1, d0, d1;
  const uint32_t v0 = lvl == 0 ? (uint32_t)idx : (uint32_t)idx * kResWg;
  const uint32_t v1 = lvl == 0 ? (uint32_t)idx : v0 + kResWg - 1u < kp.nwaves - 1 ? v0 + kResWg - 1u : kp.nwaves - 1;
  res_range(kp, v0, c0, c1);
  res_range(kp, v1, d0, d1);
  L.first = c0;
  L.last = (int64_t)d1 - 1;"""
assert s.count(a) == 1
s = s.replace(a, """  uint32_t c0, c1, d0, d1;
  if (lvl == 1 && (kp.nwaves & (kResWg - 1u)) == 0) {
    split_range(kp.ntiles, kp.nwaves / kResWg, (uint32_t)idx, c0, d1);
  } else {
    const uint32_t v0 = lvl == 0 ? (uint32_t)idx : (uint32_t)idx * kResWg;
    const uint32_t v1 = lvl == 0 ? (uint32_t)idx : v0 + kResWg - 1u < kp.nwaves - 1 ? v0 + kResWg - 1u : kp.nwaves - 1;
    res_range(kp, v0, c0, c1);
    res_range(kp, v1, d0, d1);
  }
  L.first = c0;
  L.last = (int64_t)d1 - 1;""")
