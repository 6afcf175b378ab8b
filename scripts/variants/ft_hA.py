# bisect (round-4 flow table): round-4 Key (w[11], nw) zero-filled, round-4 hash loop, 10-word XOR compare
s = open("/root/repo/scripts/variants/ft_head.hip").read()
a = "    k.w[3] = row[1];\n    k.nw = 4;"
assert s.count(a) == 1
s = s.replace(a, a + "\n#pragma unroll\n    for (int i = 4; i < 11; ++i) k.w[i] = 0u;")
b = """  if (a.nw != b.nw) return false;
  for (uint32_t i = 0; i < a.nw; ++i)
    if (a.w[i] != b.w[i]) return false;
  return true;"""
assert s.count(b) == 1
s = s.replace(b, """  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) diff |= a.w[i] ^ b.w[i];
  return diff == 0;""")
