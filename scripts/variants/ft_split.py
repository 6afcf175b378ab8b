# k_agg_insert: the Key's IPv6 words read without the per-word null test (one test for the row)
a = "    for (int i = 0; i < 8; ++i) k.w[2 + i] = v6row ? v6row[i] : 0u;"
assert s.count(a) == 1
s = s.replace(a, "    for (int i = 0; i < 8; ++i) k.w[2 + i] = v6row[i];")
s = s.replace("  k.v6 = (kind & NPR_FLOW_KIND_IPV6) != 0;\n  if (k.v6) {", "  k.v6 = (kind & NPR_FLOW_KIND_IPV6) != 0;\n  if (k.v6 && v6row) {")
