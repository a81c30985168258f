# BN-fusion tests; ResNet-50 A/B of the fused BN backward sums
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 400 python -u -m pytest tests/gpu/test_bn_fusion.py tests/gpu/test_determinism.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t18.log 2>&1 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh --model,ResNet50,--batch,1024 --model,ResNet50,--batch,1024,--rt,bn_bwd_fuse=False
