#!/bin/bash
# interleaved A/B of timing-only ablation builds (C2 kernel time, results unchecked):
# bash scripts/abl_ab_nogate.sh ROUNDS VARIANT...
set -e
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    if [ -z "$v" ] || [ "$v" = base ]; then lib=""; else lib=$PWD/net-parser-rs_amd/lib/libnpr_$v.so; fi
    NPR_LIB=$lib timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu --no-gate > gpurun_out/abl.json 2>/dev/null
    echo "${v:-base} r$r $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abl.json)"
  done
done
