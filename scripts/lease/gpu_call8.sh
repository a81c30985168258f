# same-box A/B of the round-5 ResNet changes
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_bn_fusion.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t20.log 2>&1 || exit $?
R="--model,ResNet50,--batch,1024"
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh $R $R,--rt,bn_bwd_fuse=False $R,--rt,bn_bwd_fuse=False,--rt,epilogue_prefetch=False $R,--rt,bn_bwd_fuse=False,--rt,bn_masked_handoff=False $R,--rt,bn_bwd_fuse=False,--rt,bn_masked_handoff=False,--rt,epilogue_prefetch=False
