#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/r1ae_test.log python -m pytest tests/gpu -x -q -m gpu
gpu_step 300 gpurun_out/r1ae_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/r1ae_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/r1ae_r50.log python bench.py --model ResNet50 --steps 20 --warmup 5
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
