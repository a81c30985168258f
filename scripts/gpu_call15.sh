# row-streaming weight-gradient grid size A/B (E18 b1536, side stream)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,wgrad_rows_blocks=128 --rt,wgrad_rows_blocks=192 --rt,wgrad_rows_blocks=384
