# Sparse walk as persistent waves: 1 workgroup(s) of 4 waves per CU (256 CUs) loop over the groups
# (wave w takes groups w, w + W, ...), instead of one wave per group with every group resident.
s = s.replace("""  const uint32_t g = blockIdx.x * (kSpBlock / 64) + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) *sp.ctl = 0;  // the rows kernel runs only after a new exact scan
  if (g >= sp.ngroups) return;  // (wave-uniform)
  const uint64_t li = (uint64_t)g * 64 + lane;
  const bool act = li < sp.nlanes;
  const SpecCtx sc = spec_ctx(kp, spec_ctx_load(kp));
  uint32_t *row = rows + threadIdx.x * kSpRow;
""", """  if (blockIdx.x == 0 && threadIdx.x == 0) *sp.ctl = 0;  // the rows kernel runs only after a new exact scan
  const SpecCtx sc = spec_ctx(kp, spec_ctx_load(kp));
  uint32_t *row = rows + threadIdx.x * kSpRow;
  for (uint32_t g = blockIdx.x * (kSpBlock / 64) + (threadIdx.x >> 6); g < sp.ngroups; g += gridDim.x * (kSpBlock / 64)) {
  const uint64_t li = (uint64_t)g * 64 + lane;
  const bool act = li < sp.nlanes;
""")
s = s.replace("""    sp.first_entry[g] = has ? rl64(entry, __builtin_ctzll(has)) : kNone;
  }
}
""", """    sp.first_entry[g] = has ? rl64(entry, __builtin_ctzll(has)) : kNone;
  }
  }
}
""")
s = s.replace("""    hipLaunchKernelGGL(k_sparse_walk, dim3((sp.ngroups + kSpBlock / 64 - 1) / (kSpBlock / 64)), dim3(kSpBlock), 0, s, sp);""",
"""    const uint32_t nwg = (sp.ngroups + kSpBlock / 64 - 1) / (kSpBlock / 64);
    hipLaunchKernelGGL(k_sparse_walk, dim3(nwg < 256u * 1 ? nwg : 256u * 1), dim3(kSpBlock), 0, s, sp);""")
