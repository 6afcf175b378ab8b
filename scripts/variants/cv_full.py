# convert_shape: whole lanes (rpb = per x 1024, per = ceil(n / (CUs x 1024))) instead of ceil(n / CUs)
a = "  uint64_t rpb = (n + c - 1) / c;\n"
assert s.count(a) == 1
s = s.replace(a, "  uint64_t rpb = (n + c - 1) / c;\n  rpb = (rpb + kCvtBlock - 1) / kCvtBlock * kCvtBlock;\n")
