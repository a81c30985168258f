set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
# world-1 vs world-2 (side stream, deterministic, 2 steps) with the bucketer's
# event-readiness log
ZK_COMM_DEBUG_EVENTS=1 ZK_TEST_STEPS=2 DIAG_REPS=2 timeout -k 10 300 python -u scripts/diag_dp.py /tmp/dpd5 1 > gpurun_out/dp_diag5.log 2>&1
