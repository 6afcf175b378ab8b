# Short ranges: no priority steps (every wave stays at the kernel's starting priority 3).
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
