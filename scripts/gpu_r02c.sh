set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_stream.py tests/test_c_harness.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests_r02c.log 2>&1 || exit $?
timeout -k 10 300 python scripts/pcie_rate.py --config c2 --reps 3 > gpurun_out/pcie_c2_r02c.log 2>&1 || exit $?
timeout -k 10 300 python scripts/pcie_rate.py --config c3 --reps 3 > gpurun_out/pcie_c3_r02c.log 2>&1 || exit $?
