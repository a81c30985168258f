set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
# data-parallel GPU tests after the readiness fix, the loader tests, then 3
# more world-1 vs world-2 comparisons
timeout -k 10 900 python -u -m pytest tests/gpu/test_dp_gpu.py tests/gpu/test_loader_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/dp_tests3.log 2>&1 &&
ZK_TEST_STEPS=4 DIAG_REPS=3 DIAG_BRIEF=1 timeout -k 10 300 python -u scripts/diag_dp.py /tmp/dpd8 1 > gpurun_out/dp_diag8.log 2>&1
