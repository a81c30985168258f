# wgrad_rows lab (+ its tests, BN / binary-block tests)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/gpu/test_wgrad_rows.py tests/gpu/test_binary_block.py tests/gpu/test_norm_pool.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t15.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/wgrad_lab.py --shapes 56,64,64/28,128,128 --rounds 2 --out gpurun_out/wlab15.jsonl > gpurun_out/wlab15.log 2>&1
