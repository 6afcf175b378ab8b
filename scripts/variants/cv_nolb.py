# k_convert_records without the look-back wait: every block starts its rows at j x 1024 (C2: every
# record Ok), the same write pattern with no dependency.  Timing only (wrong rows on other inputs).
a = "    for (;;) {\n      const bool s_miss"
assert s.count(a) == 1
s = s.replace(a, "    for (;false;) {\n      const bool s_miss")
b = "      acc = x;\n"
assert s.count(b) == 1
s = s.replace(b, "      acc = x * 0 + j * (uint64_t)kCvtRecs;\n")
