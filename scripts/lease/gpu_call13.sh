# round-5 final-state profiles: E18 b1536, ResNet-50 b1024, QuickNet-Large b1024
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu.sh prof:BinaryResNetE18:1536 "profargs:--model,ResNet50,--batch,1024,--steps,12,--warmup,6,--graph,0" prof:QuickNetLarge:1024 tests:float_wgrad
