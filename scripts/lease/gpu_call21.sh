# E18 wgrad_slab_mb 32 vs 64, three interleaved rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=40 AB_ROUNDS=3 bash scripts/ab.sh - --rt,wgrad_slab_mb=64
