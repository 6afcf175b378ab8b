# Short ranges: a wave's priority set once from its age rank on its SIMD (wave w of a workgroup:
# rank w / 4; the arbiter favours older waves, so younger ones get the higher priority) instead of
# stepping every wave down over its first three tiles.
old_a = """        if (Q == 0) __builtin_amdgcn_s_setprio(2);
        else if (Q == 1) __builtin_amdgcn_s_setprio(1);
        else if (Q == 2) __builtin_amdgcn_s_setprio(0);"""
assert s.count(old_a) == 1
s = s.replace(old_a, """        (void)0;""")
old_b = """      if (k == 0) __builtin_amdgcn_s_setprio(2);
      else if (k == 1) __builtin_amdgcn_s_setprio(1);
      else if (k == 2) __builtin_amdgcn_s_setprio(0);"""
assert s.count(old_b) == 1
s = s.replace(old_b, """      (void)0;""")
old_c = """  __builtin_amdgcn_s_setprio(3);  // lowered by one per tile parsed (below)"""
assert s.count(old_c) == 1
s = s.replace(old_c, """  if (wid < 4) __builtin_amdgcn_s_setprio(0);
  else if (wid < 8) __builtin_amdgcn_s_setprio(1);
  else if (wid < 12) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(3);""")
