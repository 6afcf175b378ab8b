#!/bin/bash
# C3 (8M variable-length records, 6.4 GB) through the sparse record walk, on the GPU box.
#   check TAG              the sparse parity tests, the C3 bit-exact test, the C3 bench line and its
#                          FETCH_SIZE / WRITE_SIZE PMC passes (-> gpurun_out/TAG_pmc_c3.json)
#   span TAG ROUNDS SPAN.. interleaved C3 bench lines with the walk forced at each lane span (bytes)
#   prof TAG SPAN..        rocprofv3 --kernel-trace --stats of the C3 bench at each lane span
# Usage: gpu_c3.sh MODE ARGS...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
MODE="$1"; TAG="$2"; shift 2
case "$MODE" in
check)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sparse" --timeout 120 --timeout-method thread -p no:cacheprovider > "gpurun_out/${TAG}_sparse_tests.log" 2>&1 || exit $?
  timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -k "c3 or adversarial_300mb" --timeout 250 --timeout-method thread -p no:cacheprovider > "gpurun_out/${TAG}_c3.log" 2>&1 || exit $?
  timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > "gpurun_out/${TAG}_bench_c3.json" 2> "gpurun_out/${TAG}_bench_c3.err" || exit $?
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_${TAG}_c3/p$i" -o run \
        -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_${TAG}_c3_$grp.log" 2>&1) || exit $?
  done
  python scripts/pmc_json.py "${TAG}_c3" "gpurun_out/${TAG}_pmc_c3.json" c3 || exit $?
  ;;
span)
  ROUNDS="$1"; shift
  for r in $(seq 1 "$ROUNDS"); do
    for sp in "$@"; do
      timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 2 --no-cpu --sparse-span "$sp" > "gpurun_out/${TAG}_s${sp}_$r.json" 2> "gpurun_out/${TAG}_s${sp}_$r.err" || exit $?
      python -c "import json; d=json.load(open('gpurun_out/${TAG}_s${sp}_$r.json')); print('$sp $r', d['roofline']['kernel_ms'])"
    done
  done
  ;;
prof)
  for sp in "$@"; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_s$sp" -o run --output-format csv \
       -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu --sparse-span "$sp" > "$R/gpurun_out/${TAG}_s$sp.json" 2> "$R/gpurun_out/${TAG}_s$sp.err") || exit $?
    grep -E "k_sparse" "gpurun_out/${TAG}_s$sp/run_kernel_stats.csv" | cut -d, -f1-4 | sed "s/^/$sp /"
  done
  ;;
*) echo "unknown mode $MODE"; exit 2 ;;
esac
exit 0
