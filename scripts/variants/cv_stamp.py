# k_convert_records with per-workgroup s_memrealtime stamps (100 MHz) written to the IPv6 side
# table (C2 has no IPv6 flows, so nothing else writes it): start, decoded, prefix known, rows issued.
# Timing only: read by scripts/cvt_stamps.py.
a = "  const uint64_t j = blockIdx.x, nb = gridDim.x;\n  const int64_t lo"
assert s.count(a) == 1
s = s.replace(a, "  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();\n  __shared__ uint64_t ts3_sh;\n" + a)
b = "  __syncthreads();\n  uint32_t cnt = 0;\n"
assert s.count(b) == 1
s = s.replace(b, "  __syncthreads();\n  const uint64_t ts1 = __builtin_amdgcn_s_memrealtime();\n  uint32_t cnt = 0;\n")
c = "    excl_sh = ok ? acc : ~0ull;\n"
assert s.count(c) == 1
s = s.replace(c, "    ts3_sh = __builtin_amdgcn_s_memrealtime();\n" + c)
d = "    after += rc;\n  }\n}\n"
assert s.count(d) == 1
s = s.replace(d, "    after += rc;\n  }\n  if (threadIdx.x == 0) {\n    uint64_t *st = reinterpret_cast<uint64_t *>(out_v6) + j * 4;\n    st[0] = ts0; st[1] = ts1; st[2] = ts3_sh; st[3] = __builtin_amdgcn_s_memrealtime();\n  }\n}\n")
