# Sparse walk: each record's slot stores issued one record later, right after the next-but-one
# window's loads (software-pipelined), so the latch's vmcnt(0) wait does not wait on their acks.
s = s.replace("""  uint32_t cap, n, okn;
  uint64_t okmask, okmask2, ovf;
  __device__ __forceinline__ void operator()(uint64_t p, bool ok, const FlowWords &f) {
    if (n < cap) {
      if (slot_a) {
        u32x4 a;
        uint32_t b[3];
        slot_image(f, p, lo, a, b);
        slot_a[(uint64_t)n * 64u] = a;
        uint32_t *d = slot_b + (uint64_t)n * 192u;
        d[0] = b[0];
        d[1] = b[1];
        d[2] = b[2];
      }""", """  uint32_t cap, n, okn;
  uint64_t okmask, okmask2, ovf;
  u32x4 pa;          // the previous record's slot image, stored by flush()
  uint32_t pb[3], pn;
  __device__ __forceinline__ void flush() {
    if (pn != ~0u) {
      slot_a[(uint64_t)pn * 64u] = pa;
      uint32_t *d = slot_b + (uint64_t)pn * 192u;
      d[0] = pb[0];
      d[1] = pb[1];
      d[2] = pb[2];
      pn = ~0u;
    }
  }
  __device__ __forceinline__ void operator()(uint64_t p, bool ok, const FlowWords &f) {
    if (n < cap) {
      if (slot_a) {
        slot_image(f, p, lo, pa, pb);
        pn = n;
      }""")
s = s.replace("""                  lane_lo(sp, g * 64u + lane), sp.cap, 0u, 0u, 0ull, 0ull, kNone};""",
              """                  lane_lo(sp, g * 64u + lane), sp.cap, 0u, 0u, 0ull, 0ull, kNone, u32x4{}, {0u, 0u, 0u}, ~0u};""")
s = s.replace("""  uint64_t base;  // the lane's first Ok flow's convert_records index
  uint32_t rank;
""", """  uint64_t base;  // the lane's first Ok flow's convert_records index
  uint32_t rank;
  __device__ __forceinline__ void flush() {}
""")
s = s.replace("""    if (more) load_chunks<0, 5>(align16(kp.buf + next), end, wn);
    FlowWords f{};""", """    if (more) load_chunks<0, 5>(align16(kp.buf + next), end, wn);
    sink.flush();  // the previous record's slot, behind this one's loads
    FlowWords f{};""")
s = s.replace("""    pos = next;
    if (!more) break;
#pragma unroll
    for (int j = 0; j < 20; ++j) w[j] = wn[j];
  }
  return pos;""", """    pos = next;
    if (!more) break;
#pragma unroll
    for (int j = 0; j < 20; ++j) w[j] = wn[j];
  }
  sink.flush();
  return pos;""")
