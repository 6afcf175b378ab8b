# the sparse walk's tail_dword (the buffer's last bytes, dword by dword) inlined: k_sparse_walk /
# k_sparse_rows / k_sparse_scan then make no calls
a = """__device__ __noinline__ uint32_t tail_dword(const uint8_t *p, const uint8_t *end) {"""
assert s.count(a) == 1
s = s.replace(a, """__device__ __forceinline__ uint32_t tail_dword(const uint8_t *p, const uint8_t *end) {""")
