#!/bin/bash
# The bench contract with no flags, plus the other models at the default batch.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-def}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 400 gpurun_out/${TAG}_e18.log python bench.py
gpu_step 300 gpurun_out/${TAG}_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/${TAG}_r50.log python bench.py --model ResNet50 --steps 10 --warmup 3
echo done >> gpurun_out/progress.txt
