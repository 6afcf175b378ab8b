# C3 lane sizing: at most 32 mean records per lane when the range fills the chip (product: 64), so
# the walk runs more workgroups per CU (C3: 8M records -> k = ceil(8M / (256 CUs x 256 lanes x 32))).
s = s.replace("constexpr uint64_t kSparseLaneRecords = 64;", "constexpr uint64_t kSparseLaneRecords = 32;")
