# k_agg_insert: the probe's slot read at workgroup scope (an L1-cacheable load, not an L2 round trip
# per lane): a claimed slot never changes, and a stale 0 is corrected by the agent-scope CAS
a = "      uint64_t w = __hip_atomic_load(slot_word + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);"
assert s.count(a) == 1
s = s.replace(a, "      uint64_t w = __hip_atomic_load(slot_word + pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);")
