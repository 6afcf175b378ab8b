# k_parse_resident look-back: re-poll an unpublished aggregate by its LAST granule only (one
# returning atomic per lane instead of five), then read all five once that one is this launch's.
a = """        const bool need = (uint32_t)lane < sz && !G[w].present;
        if (__ballot(need)) {
          const LaneSeg N = load_res(kp, 1, (int64_t)w0 + sz - 1 - lane, need);
          if (need) G[w] = N;
        }"""
assert s.count(a) == 1
s = s.replace(a, """        const bool need = (uint32_t)lane < sz && !G[w].present;
        if (__ballot(need)) {
          const int64_t gi = (int64_t)w0 + sz - 1 - lane;
          const bool pub = need && tagged(ld_res(&kp.rgroups[need ? gi : 0].g[4]), kp.epoch);
          if (__ballot(pub)) {
            const LaneSeg N = load_res(kp, 1, gi, pub);
            if (pub) G[w] = N;
          }
        }""")
