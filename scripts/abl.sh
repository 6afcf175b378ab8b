#!/bin/bash
# rocprofv3 kernel-trace stats of scripts/launch_only.py for each library variant given.
# Usage: bash scripts/abl.sh TAG lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; R=$(pwd); mkdir -p gpurun_out
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  b=$(basename "$L" .so)
  NPR_LIB="$R/$L" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/abl_${TAG}_$b" -o run \
      --output-format csv -- python3 "$R/scripts/launch_only.py" > "$R/gpurun_out/abl_${TAG}_$b.log" 2>&1 || exit $?
done
exit 0
