# k_parse_resident: the one-length fast prefix as a rolled loop (one copy of the tile body and its
# decode_fast; the flows go to kept round Q by a uniform select, as in the general loop) instead of
# six unrolled copies: tests whether the unrolled prefix's code size (+23 KB) costs instruction fetch.
a = "#pragma unroll\n    for (uint32_t Q = 0; Q < (uint32_t)kResSlots; ++Q) {  // (unrolled: kept round Q is a register block)"
assert s.count(a) == 1
s = s.replace(a, "#pragma clang loop unroll(disable)\n    for (uint32_t Q = 0; Q < (uint32_t)kResSlots; ++Q) {")
b = """      fl[Q][0] = (f.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) ? f.v6off : f.d[0];
#pragma unroll
      for (int j = 1; j < 7; ++j) fl[Q][j] = f.d[j];
      fl[Q][7] = lo_r + rr;  // record offset - base
"""
assert s.count(b) == 1
s = s.replace(b, """      {
        const uint32_t sw[8] = {(f.d[6] & (NPR_FLOW_KIND_IPV6 << 16)) ? f.v6off : f.d[0], f.d[1], f.d[2], f.d[3],
                                f.d[4], f.d[5], f.d[6], lo_r + rr};
        const uint32_t qu = __builtin_amdgcn_readfirstlane(Q);
#pragma unroll
        for (int qq = 0; qq < kResSlots; ++qq)
          if ((uint32_t)qq == qu) {
#pragma unroll
            for (int j = 0; j < 8; ++j) fl[qq][j] = sw[j];
          }
      }
""")
