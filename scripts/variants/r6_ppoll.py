# the look-back's polling in rw_floor's P style: every poll re-reads the missing aggregates by
# returning atomics, s_sleep(4) between polls, the abort word and the clock checked on every poll
# (no backed-off naps)
a = """      if (tries && !res_nap(kp, t0, nap)) {
        okw = false;
        break;
      }"""
assert s.count(a) == 1
s = s.replace(a, """      if (tries) {
        if (__hip_atomic_load(kp.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kp.epoch ||
            __builtin_amdgcn_s_memrealtime() - t0 > kp.timeout_ticks) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > kp.timeout_ticks)
            __hip_atomic_store(kp.abort_word, kp.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          okw = false;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }""")
