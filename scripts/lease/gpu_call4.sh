# BN-fusion tests; ResNet-50 A/B: fused BN backward sums, deep-gemm kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 400 python -u -m pytest tests/gpu/test_bn_fusion.py tests/gpu/test_norm_pool.py tests/gpu/test_pointwise.py tests/gpu/test_determinism.py tests/gpu/test_loader_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t17.log 2>&1 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh --model,ResNet50,--batch,1024 --model,ResNet50,--batch,1024,--rt,bn_bwd_fuse=False --model,ResNet50,--batch,1024,--rt,dgrad_deep=False,--rt,wgrad_deep=False
