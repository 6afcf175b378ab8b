# k_agg_insert: workgroup-scope probe read (ft_wg) + the key hash as a rolled loop (4 or 10 trips)
# whose word is picked from the register-resident Key by a select chain (no dynamic indexing)
exec(open("/root/repo/scripts/variants/ft_wg.py").read())
a = """#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  if (k.v6) {
#pragma unroll
    for (uint32_t i = 4; i < 10; ++i) h = mix64(h ^ (uint64_t)k.w[i] * 0xff51afd7ed558ccdull + i);
  }"""
assert s.count(a) == 1
s = s.replace(a, """  const uint32_t nw = k.v6 ? 10u : 4u;
#pragma clang loop unroll(disable)
  for (uint32_t i = 0; i < nw; ++i) {
    uint32_t x = k.w[0];
#pragma unroll
    for (uint32_t j = 1; j < 10; ++j) x = i == j ? k.w[j] : x;
    h = mix64(h ^ (uint64_t)x * 0xff51afd7ed558ccdull + i);
  }""")
