# k_sparse_walk / lane_walk: each record's window loaded at the header itself (four unaligned dwordx4
# loads, 64 B) instead of [header & ~15, +80) (five aligned loads); no per-lane byte selection.
a = """// lanes whose bit of m is set: a, the others: b"""
assert s.count(a) == 1
s = s.replace(a, """// chunks [K0, K1) of the bytes at p, any alignment (unaligned dwordx4 loads), into w[4 K0 .. 4 K1);
// dword by dword for the buffer's last bytes
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef const __attribute__((address_space(1))) u32x4_u *gv4u_t;
template <int K0, int K1>
__device__ __forceinline__ void load_at(const uint8_t *p, const uint8_t *end, uint32_t (&w)[kSpWords]) {
  if (p + 16 * K1 <= end) {
    const gv4u_t s = (gv4u_t)(uintptr_t)p;
#pragma unroll
    for (int k = K0; k < K1; ++k) {
      const u32x4 v = s[k];
#pragma unroll
      for (int e = 0; e < 4; ++e) w[4 * k + e] = v[e];
    }
  } else {
#pragma unroll
    for (int k = K0; k < K1; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) w[4 * k + e] = dword_at(p + 16 * k + 4 * e, end);
  }
}
""" + a)
b = """  uint32_t a[17];
  words_at<16, 12>(w, rel, a);
#pragma unroll
  for (int k = 12; k < 17; ++k) a[k] = 0u;
  const uint32_t etype = ((a[3] & 0xffu) << 8) | ((a[3] >> 8) & 0xffu);
  const bool six = etype == 0x86ddu;
  bool full = false;
  if (__ballot(six)) {
    if (six) {
      load_chunks<5, 7>(a16, end, w);
      words_at<16, 17>(w, rel, a);
      full = true;
    }
  }
  uint32_t st = decode_fast_core<true, true>(a, incl, f, true);
  if (__ballot(st == 0xffu)) {
    if (st == 0xffu) {
      if (!full) load_chunks<5, 7>(a16, end, w);
#pragma unroll
      for (int j = 0; j < kSpWords; ++j) row[j] = w[j];
      const SpRowReader r{row, rel + 16u, pp + 16, avail - 16};"""
assert s.count(b) == 1
s = s.replace(b, """  (void)rel, (void)a16;
  uint32_t a[17];
#pragma unroll
  for (int k = 0; k < 12; ++k) a[k] = w[4 + k];
#pragma unroll
  for (int k = 12; k < 17; ++k) a[k] = 0u;
  const uint32_t etype = ((a[3] & 0xffu) << 8) | ((a[3] >> 8) & 0xffu);
  const bool six = etype == 0x86ddu;
  bool full = false;
  if (__ballot(six)) {
    if (six) {
      load_at<4, 6>(pp, end, w);
#pragma unroll
      for (int k = 12; k < 17; ++k) a[k] = w[4 + k];
      full = true;
    }
  }
  uint32_t st = decode_fast_core<true, true>(a, incl, f, true);
  if (__ballot(st == 0xffu)) {
    if (st == 0xffu) {
      if (!full) load_at<4, 7>(pp, end, w);
      else load_at<6, 7>(pp, end, w);
#pragma unroll
      for (int j = 0; j < kSpWords; ++j) row[j] = w[j];
      const SpRowReader r{row, 16u, pp + 16, avail - 16};""")
c = """  uint32_t w[kSpWords];
  load_chunks<0, 5>(align16(kp.buf + pos), end, w);
  for (;;) {
    const uint8_t *pp = kp.buf + pos;
    const uint32_t rel = (uint32_t)((uintptr_t)pp & 15u);
    uint32_t h[1];
    words_at<8, 1>(w, rel, h);  // incl_len
    const uint32_t incl = kp.big ? __builtin_bswap32(h[0]) : h[0];"""
assert s.count(c) == 1
s = s.replace(c, """  uint32_t w[kSpWords];
  load_at<0, 4>(kp.buf + pos, end, w);
  for (;;) {
    const uint8_t *pp = kp.buf + pos;
    const uint32_t rel = 0;
    const uint32_t incl = kp.big ? __builtin_bswap32(w[2]) : w[2];  // incl_len""")
d = """    if (more) load_chunks<0, 5>(align16(kp.buf + next), end, wn);
    FlowWords f{};
    const uint32_t st = rec_decode(kp, row, pp, avail, rel, incl, w, f);
    sink(pos, st == NPR_FLOW_OK, f);
    ++cnt;
    pos = next;
    if (!more) break;
#pragma unroll
    for (int j = 0; j < 20; ++j) w[j] = wn[j];"""
assert s.count(d) == 1
s = s.replace(d, """    if (more) load_at<0, 4>(kp.buf + next, end, wn);
    FlowWords f{};
    const uint32_t st = rec_decode(kp, row, pp, avail, rel, incl, w, f);
    sink(pos, st == NPR_FLOW_OK, f);
    ++cnt;
    pos = next;
    if (!more) break;
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = wn[j];""")
