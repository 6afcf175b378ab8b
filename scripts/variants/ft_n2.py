# k_agg_insert: the key hash as a rolled loop over the row's words in memory (4 or 10 words), the
# Key itself (for the compare) unrolled in registers
a = "    const uint64_t h = key_hash(k);"
assert s.count(a) == 1
s = s.replace(a, """    uint64_t h = 0x9e3779b97f4a7c15ull;
    {
      const uint32_t *v6r = flows_v6 ? flows_v6 + i * 8 : nullptr;
      const uint32_t nw = k.v6 ? 10u : 4u;
      for (uint32_t j = 0; j < nw; ++j) {
        const uint32_t wj = j == 0 ? k.w[0] : j == 1 ? k.w[1] : k.v6 ? (v6r ? v6r[j - 2] : 0u) : row[(j - 2) & 1];
        h = mix64(h ^ (uint64_t)wj * 0xff51afd7ed558ccdull + j);
      }
    }""")
