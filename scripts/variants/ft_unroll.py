# k_agg_insert: the row loop fully unrolled (the scratch-resident Key build of round 4 was)
a = "  for (int q = 0; q < kInsPer; ++q) {\n    const uint64_t i = (uint64_t)blockIdx.x * kInsRows"
assert s.count(a) == 1
s = s.replace(a, "#pragma unroll\n" + a)
