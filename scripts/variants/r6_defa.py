# k_parse_resident: the per-wave A stores (read only by the rare generic prefix of a mis-speculated
# range) issued after the look-back instead of right after the first barrier, where their 16 K
# write-through stores met the workgroup aggregates' publication (rw_floor A vs B: 21.4 vs 20.4 us)
a = """  // A in HBM, for the rare generic prefix of another range (its readers wait for the epoch tags).
  // Stored after the barrier: the barrier's release fence waits for every store issued before it,
  // and write-through stores held the workgroup's fold back by their round trip.
  if (active && lane == 0) {
    RangeSlot *rs = kp.rslots + v;
    st_agent(&rs->a[0], gran(ep, pos == kNone ? 0ull : pos));
    st_agent(&rs->a[1], gran(ep, entry == kNone ? 0ull : entry + 1));
    st_agent(&rs->a[2], gran(ep, cnt));
    st_agent(&rs->a[3], gran(ep, okc));
  }
"""
assert s.count(a) == 1
s = s.replace(a, "")
b = """  __syncthreads();
  if (sh.fail) return false;
  if (!active) return true;
"""
assert s.count(b) == 1
s = s.replace(b, b + """  // A in HBM, for the rare generic prefix of another range (its readers wait for the epoch tags),
  // stored once the look-back is done
  if (lane == 0) {
    RangeSlot *rs = kp.rslots + v;
    st_agent(&rs->a[0], gran(ep, pos == kNone ? 0ull : pos));
    st_agent(&rs->a[1], gran(ep, entry == kNone ? 0ull : entry + 1));
    st_agent(&rs->a[2], gran(ep, cnt));
    st_agent(&rs->a[3], gran(ep, okc));
  }
""")
