# round-5 profiles: ResNet-50 b1024 and E18 b1536 at the current defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu.sh "profargs:--model,ResNet50,--batch,1024,--steps,12,--warmup,6,--graph,0" prof:BinaryResNetE18:1536
