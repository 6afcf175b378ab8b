set -e -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./scripts/microbench/rw_floor 200 > gpurun_out/${TAG:-r05b}_rw_floor.txt 2>&1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05b}_prof -o rw -- $GRAFT_REPO_ROOT/scripts/microbench/rw_floor 50 > $GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05b}_rw_floor_prof.txt 2>&1
