#!/bin/bash
# Baseline of HEAD on a fresh box: GPU tests, E18 / QuickNetLarge / ResNet-50 bench, E18 profile.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/r1ag_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
gpu_step 300 gpurun_out/r1ag_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/r1ag_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/r1ag_r50.log python bench.py --model ResNet50 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1ag_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1ag_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
