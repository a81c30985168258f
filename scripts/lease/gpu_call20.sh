# final-state ResNet-50 profile; E18 wgrad_slab_mb 32 / 48 / 64 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
bash scripts/gpu.sh "profargs:--model,ResNet50,--batch,1024,--steps,12,--warmup,6,--graph,0" || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,wgrad_slab_mb=48 --rt,wgrad_slab_mb=64
