#!/bin/bash
# C2 kernel time under environment variants: bash scripts/abl_env.sh "ENV=.. ENV2=.." ...
set -e
mkdir -p gpurun_out
for e in "$@"; do
  env $e timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu > gpurun_out/abl.json 2>/dev/null
  echo "[$e] $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/abl.json)"
done
