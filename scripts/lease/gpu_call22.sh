# round-5 final defaults, same box: E18 b1536, QuickNet-Large b1024, ResNet-50 b1024
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=50 AB_ROUNDS=2 bash scripts/ab.sh - --model,QuickNetLarge,--batch,1024 --model,ResNet50,--batch,1024
