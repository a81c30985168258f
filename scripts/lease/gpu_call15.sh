# 3x3 256x256 dgrad epilogue: LDS (tile_huge 16, default) vs register (48),
# E18 b1536 and QuickNet-Large b1024, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,tile_huge=48 --model,QuickNetLarge,--batch,1024 --model,QuickNetLarge,--batch,1024,--rt,tile_huge=48
