# pooled BN apply with the quad's loads issued up front: tests, E18 A/B,
# kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 600 python -u -m pytest tests/gpu/test_binary_block.py tests/gpu/test_norm_pool.py tests/gpu/test_determinism.py -q --timeout 300 --timeout-method thread > gpurun_out/pool2_tests.log 2>&1 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,bn_pool_fuse=False || exit $?
bash scripts/gpu.sh prof:BinaryResNetE18:1536
