# BN apply + shortcut pool fusion: bit-identity + binary-block + DP tests,
# then E18 A/B (bn_pool_fuse on / off)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 600 python -u -m pytest tests/gpu/test_binary_block.py tests/gpu/test_dp_gpu.py tests/gpu/test_models_gpu.py -q --timeout 300 --timeout-method thread > gpurun_out/pool_tests.log 2>&1 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,bn_pool_fuse=False
