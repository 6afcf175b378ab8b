# The look-back's fold E(b) = E ⊕ G(0) ⊕ ... ⊕ G(b-1) in one pass over every window when every
# link is consistent (each aggregate's entry is its predecessor's exit, the first one E's, none
# ends the chain, all valid): the windows' counts summed lane-wise, then ONE pair of wave sums,
# instead of a fold_window (two wave sums each) and a combine per window; anything else takes the
# per-window fold as before
a = """#pragma unroll
    for (int w = 0; w < kTopWin; ++w) {
      const uint32_t w0 = 64u * (uint32_t)w;
      if (w0 >= b || !okw) break;
      E = combine(kp, E, fold_window(kp, G[w], (int)(b - w0 < 64u ? b - w0 : 64u) - 1));
    }"""
assert s.count(a) == 1
s = s.replace(a, """    bool lean = okw && b > 0 && E.valid && E.exit >= tile_end(kp, E.last);
    if (lean) {
      bool bad = false;
      uint32_t c = 0, o = 0;
#pragma unroll
      for (int w = 0; w < kTopWin; ++w) {
        const uint32_t w0 = 64u * (uint32_t)w, sz = b > w0 ? (b - w0 < 64u ? b - w0 : 64u) : 0u;
        const bool in = (uint32_t)lane < sz;
        // predecessor: lane + 1 of this window, or (its first element) the last element of the
        // window below (lane 0 there), or E
        const uint64_t nxt = shfl_down64(G[w].exit);
        const uint64_t below = w == 0 ? E.exit : rl64(G[w > 0 ? w - 1 : 0].exit, 0);
        const uint64_t prev = (uint32_t)lane + 1u < sz ? nxt : below;
        bad = bad || (in && (!G[w].valid || G[w].entry != prev || G[w].exit < tile_end(kp, G[w].last)));
        c += in ? (uint32_t)G[w].cnt : 0u;
        o += in ? (uint32_t)G[w].ok : 0u;
      }
      lean = __ballot(bad) == 0ull;
      if (lean) {
        const int wl = (int)((b - 1u) >> 6);  // the window of G(b-1): its lane 0
        uint64_t ex = 0;
        int64_t la = 0;
#pragma unroll
        for (int w = 0; w < kTopWin; ++w)
          if (w == wl) {
            ex = rl64(G[w].exit, 0);
            la = (int64_t)rl64((uint64_t)G[w].last, 0);
          }
        E.cnt += __ockl_wfred_add_u32(c);
        E.ok += __ockl_wfred_add_u32(o);
        E.exit = ex;
        E.last = la;
      }
    }
    if (!lean) {
#pragma unroll
      for (int w = 0; w < kTopWin; ++w) {
        const uint32_t w0 = 64u * (uint32_t)w;
        if (w0 >= b || !okw) break;
        E = combine(kp, E, fold_window(kp, G[w], (int)(b - w0 < 64u ? b - w0 : 64u) - 1));
      }
    }""")
