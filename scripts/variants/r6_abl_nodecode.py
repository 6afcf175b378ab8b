# Timing-only ablation (wrong results): the sparse walk's per-record decode replaced by copying
# window words into the flow (no parse), to size the decode's share of the walk.
s = s.replace("""  uint32_t st = decode_fast_core<true, true>(a, incl, f, true);""", """  uint32_t st = 0u;  // (ablation)
#pragma unroll
  for (int k = 0; k < 7; ++k) f.d[k] = a[k + 2];
  if (incl == 0x7fffffffu) st = decode_fast_core<true, true>(a, incl, f, true);""")
