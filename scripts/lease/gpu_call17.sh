# final-state E18 profile (kernel trace) + QuickNet-Large / E18 tile_huge
# wgrad-bit A/B at the current defaults
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
bash scripts/gpu.sh prof:BinaryResNetE18:1536 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh --model,QuickNetLarge,--batch,1024 --model,QuickNetLarge,--batch,1024,--rt,tile_huge=50 --model,QuickNetLarge,--batch,1024,--rt,tile_huge=52
