# high-priority compute stream A/B (E18, ResNet-50)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
R="--model,ResNet50,--batch,1024"
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,compute_high_priority=True $R $R,--rt,compute_high_priority=True
