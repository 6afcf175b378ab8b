# k_convert_records with PFD payload windows in flight per lane (the product: 1).  PFD is set by the
# wrapper file that execs this one.
a = """  bool fnext = window_fits(buf, len, rc[0]);
  RowWin Wn;
  win_load(rc[0], fnext, Wn);
#pragma unroll
  for (int r = 0; r < kCvtPer; ++r) {
    const bool f = fnext;
    const RowWin W = Wn;
    if (r + 1 < kCvtPer) {
      fnext = window_fits(buf, len, rc[r + 1]);
      win_load(rc[r + 1], fnext, Wn);
    }
    if (f) window_store(W, rows[0] + threadIdx.x * kRowWords);
"""
b = """  constexpr int kPF = %d;
  bool fq[kCvtPer];
  RowWin Wq[kCvtPer];
#pragma unroll
  for (int r = 0; r < kPF && r < kCvtPer; ++r) {
    fq[r] = window_fits(buf, len, rc[r]);
    win_load(rc[r], fq[r], Wq[r]);
  }
#pragma unroll
  for (int r = 0; r < kCvtPer; ++r) {
    if (r + kPF < kCvtPer) {
      fq[r + kPF] = window_fits(buf, len, rc[r + kPF]);
      win_load(rc[r + kPF], fq[r + kPF], Wq[r + kPF]);
    }
    const bool f = fq[r];
    if (f) window_store(Wq[r], rows[0] + threadIdx.x * kRowWords);
""" % PFD
assert s.count(a) == 1
s = s.replace(a, b)
