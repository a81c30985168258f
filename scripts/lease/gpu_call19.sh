# ResNet-50 b1024: the tile_huge 48 default against 16 (the register-epilogue
# 3x3 256x256 dgrad rule also reaches its strided 3x3 convs)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=30 AB_ROUNDS=2 bash scripts/ab.sh --model,ResNet50,--batch,1024 --model,ResNet50,--batch,1024,--rt,tile_huge=16
