# DIAG only: wave 0 of each workgroup stamps [10] right after the publication barrier and [11]
# right after the workgroup fold (before put_agg), instead of its deferred-tile count / fast flag.
s = s.replace("""  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
""", """  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  if (DIAG && wid == 0) stamp_at(st, 10);
""")
s = s.replace("""    res_fold_lanes(kp, L, (int)nw, e, agg);
    // G(b), then the arrival.""", """    res_fold_lanes(kp, L, (int)nw, e, agg);
    if (DIAG) stamp_at(st, 11);
    // G(b), then the arrival.""")
s = s.replace("""    st.v[10] = c1 - tdef;
    st.v[11] = (entry != kNone && xe == pos) ? 1 : 0;""", """    if (wid != 0) {
      st.v[10] = c1 - tdef;
      st.v[11] = (entry != kNone && xe == pos) ? 1 : 0;
    }""")
