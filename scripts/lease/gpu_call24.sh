# comm_backend auto (native RCCL communicator, collective fallback): DP and
# native-communicator GPU tests, then forced 1-rank DP bench vs plain
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 700 python -u -m pytest tests/gpu/test_dp_gpu.py tests/gpu/test_native_comm.py tests/gpu/test_trainer_hip.py -q --timeout 300 --timeout-method thread > gpurun_out/auto_tests.log 2>&1 || exit $?
AB_STEPS=30 AB_ROUNDS=1 bash scripts/ab.sh - --force-dp --force-dp,--rt,comm_backend=torch
