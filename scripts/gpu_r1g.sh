#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 400 gpurun_out/r1g_pytest_gpu.log python -m pytest tests -m gpu -q
gpu_step 900 gpurun_out/tune_bconv2.log python tools/tune_bconv.py --out gpurun_out/tune_bconv2.json
gpu_step 600 gpurun_out/r1g_bench_hip.log python bench.py --backend hip --steps 20 --warmup 5
echo done >> gpurun_out/progress.txt
