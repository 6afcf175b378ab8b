#!/bin/bash
# C3 sparse-path check: the sparse parity tests, the C3 bit-exact test, the C3 bench line and the
# FETCH_SIZE / WRITE_SIZE PMC passes of it.  Usage: gpu_c3_check.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="${1:-r04}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "sparse" --timeout 120 --timeout-method thread -p no:cacheprovider > "gpurun_out/${TAG}_sparse_tests.log" 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -k c3 --timeout 250 --timeout-method thread -p no:cacheprovider > "gpurun_out/${TAG}_c3.log" 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu > "gpurun_out/${TAG}_bench_c3.json" 2> "gpurun_out/${TAG}_bench_c3.err" || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_${TAG}_c3/p$i" -o run \
      -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_${TAG}_c3_$grp.log" 2>&1 || exit $?
done
cd "$R" && python scripts/pmc_json.py "${TAG}_c3" "gpurun_out/${TAG}_pmc_c3.json" c3 || exit $?
exit 0
