#!/bin/bash
# interleaved A/B of lib variants on C3 (ms per capture): bash scripts/ab_c3.sh ROUNDS VARIANT...
set -e
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    if [ -z "$v" ] || [ "$v" = base ]; then lib=""; else lib=$PWD/net-parser-rs_amd/lib/libnpr_$v.so; fi
    NPR_LIB=$lib timeout -k 10 200 python bench.py --config c3 --steps 6 --warmup 1 --no-cpu > gpurun_out/abl_c3.json 2>/dev/null
    echo "${v:-base} r$r c3 $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abl_c3.json)"
  done
done
