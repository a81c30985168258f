set -o pipefail
for u in 1 2 4; do
  ZK_BN_UNROLL=$u timeout -k 10 200 python -u tools/bn_lab.py --tag ur$u --json gpurun_out/bn_lab_ur.jsonl > gpurun_out/bn_lab_ur$u.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_norm_pool.py tests/gpu/test_binary_block.py tests/gpu/test_bn_fusion.py tests/gpu/test_determinism.py tests/gpu/test_models_gpu.py > gpurun_out/bn_tests.log 2>&1 || { tail -30 gpurun_out/bn_tests.log; exit 1; }
tail -3 gpurun_out/bn_tests.log
