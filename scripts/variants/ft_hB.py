# bisect (round-4 flow table): round-4 Key and compare, unrolled hash (4 words + 6 more for IPv6)
s = open("/root/repo/scripts/variants/ft_head.hip").read()
a = "  for (uint32_t i = 0; i < k.nw; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);"
assert s.count(a) == 1
s = s.replace(a, """#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  if (k.nw == 10) {
#pragma unroll
    for (uint32_t i = 4; i < 10; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  }""")
