#!/bin/bash
# Interleaved C2 timing of the round-6 lattice-rows experiment build (scripts/variants/r6_lattice_rows.diff
# applied; NPR_NO_LATTICE=1 switched it off there -- the product has no such switch), on and off:
# ROUNDS x each, bench.py --steps 200 (HIP-event kernel time printed).  Usage: ab_lattice.sh TAG ROUNDS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG="$1"; ROUNDS="$2"
for r in $(seq 1 "$ROUNDS"); do
  for v in lattice off; do
    if [ "$v" = off ]; then export NPR_NO_LATTICE=1; else unset NPR_NO_LATTICE; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > "gpurun_out/${TAG}_${v}_$r.json" 2>> "gpurun_out/${TAG}.err" || exit $?
    python -c "import json; d=json.load(open('gpurun_out/${TAG}_${v}_$r.json')); print('$v $r', d['roofline']['kernel_ms'], d['value'])"
  done
done
unset NPR_NO_LATTICE
exit 0
