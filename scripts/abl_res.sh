#!/bin/bash
# A/B of resident-kernel builds (lib/libnpr_*.so; "" = lib/libnpr.so): C2 kernel time, then one
# --stats run per variant whose per-wave stamps go through scripts/res_stamps.py.
set -e
mkdir -p gpurun_out
for v in "$@"; do
  lib=net-parser-rs_amd/lib/libnpr${v:+_$v}.so
  for rep in 1 2; do
    NPR_LIB=$lib timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu > gpurun_out/abl.json 2>/dev/null
    echo "${v:-base} rep$rep $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abl.json)"
  done
  NPR_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --stats > gpurun_out/abl.json 2>/dev/null
  cp gpurun_out/stamps_rank0.npy gpurun_out/st_${v:-base}.npy
done
