# ResNet-50 kernel profiles with and without the fused BN backward sums
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu.sh "profargs:--model,ResNet50,--batch,1024,--steps,12,--warmup,6,--graph,0" "profargs:--model,ResNet50,--batch,1024,--steps,12,--warmup,6,--graph,0,--rt,bn_bwd_fuse=False"
