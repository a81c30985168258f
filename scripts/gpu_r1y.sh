#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/r1y_pytest_gpu.log python -m pytest tests/gpu -q -x
gpu_step 300 gpurun_out/r1y_bench_e18.log python bench.py --steps 30 --warmup 10
gpu_step 300 gpurun_out/r1y_bench_qnl.log python bench.py --model QuickNetLarge --steps 10 --warmup 5
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
