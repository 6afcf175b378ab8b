# TileReader::slow32 (the general decoder's bounds-checked read past the staged window) inlined:
# the resident kernel then makes no calls at all (42 call sites of the cold path)
a = """  static __device__ __noinline__ uint32_t slow32(const uint8_t *g, uint64_t gavail, uint32_t q) {"""
assert s.count(a) == 1
s = s.replace(a, """  static __device__ __forceinline__ uint32_t slow32(const uint8_t *g, uint64_t gavail, uint32_t q) {""")
