#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/r1af_test.log python -m pytest tests/gpu -x -q -m gpu
gpu_step 300 gpurun_out/r1af_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/r1af_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1af_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1af_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
