# convert_shape: rpb = ceil(n / CUs) rounded up to a multiple of 256 records
a = "  uint64_t rpb = (n + c - 1) / c;\n"
assert s.count(a) == 1
s = s.replace(a, "  uint64_t rpb = (n + c - 1) / c;\n  rpb = (rpb + 255) / 256 * 256;\n")
