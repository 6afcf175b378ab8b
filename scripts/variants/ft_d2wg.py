exec(open("/root/repo/scripts/variants/ft_d2.py").read())
exec(open("/root/repo/scripts/variants/ft_wg.py").read().replace("      uint64_t w = __hip_atomic_load", "    uint64_t w = __hip_atomic_load"))
