#!/bin/bash
# C3 lane-span sweep: for each span (bytes per lane), the C3 bench line (sparse forced at that span)
# and the FETCH_SIZE / WRITE_SIZE PMC passes.  Usage: gpu_c3_span.sh TAG SPAN...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG="$1"; shift
for sp in "$@"; do
  timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu --sparse-span "$sp" > "gpurun_out/${TAG}_s${sp}_bench.json" 2> "gpurun_out/${TAG}_s${sp}_bench.err" || exit $?
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$R/gpurun_out/pmc_${TAG}_s${sp}/p$i" -o run \
        -- python3 "$R/bench.py" --config c3 --steps 2 --warmup 1 --no-cpu --sparse-span "$sp" > "$R/gpurun_out/pmc_${TAG}_s${sp}_p$i.log" 2>&1) || exit $?
  done
  python scripts/pmc_json.py "${TAG}_s${sp}" "gpurun_out/${TAG}_s${sp}_pmc.json" c3 > /dev/null || exit $?
done
exit 0
