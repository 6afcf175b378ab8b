# Fast prefix: tile 1's DMA issued only once tile 0 has landed (the launch's opening burst is one
# tile per wave, 16 MB, instead of two), later tiles double-buffered as before.
old = """      if (t + 1 < c1) {  // the successor tile's DMA (dma_tile's rows, offsets into the range)
        uint32_t *dst = sh.w[wid].data[(slot + 1) % kResRing];"""
assert s.count(old) == 1
s = s.replace(old, """      if (Q == 0) res_wait<0>(0u);  // (variant: tile 0 first)
      if (t + 1 < c1) {  // the successor tile's DMA (dma_tile's rows, offsets into the range)
        uint32_t *dst = sh.w[wid].data[(slot + 1) % kResRing];""")
