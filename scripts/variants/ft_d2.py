# k_agg_insert (workgroup hash dedupe): 512 rows per workgroup (24-KB LDS tables, 6 workgroups per CU)
a = "constexpr int kInsPer = 4, kInsRows"
assert s.count(a) == 1
s = s.replace(a, "constexpr int kInsPer = 2, kInsRows")
