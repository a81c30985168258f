#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1x_test.log python -m pytest tests/gpu/test_bconv_bwd_kernels.py -q -x
gpu_step 600 gpurun_out/r1x_tune.log python tools/tune_bconv.py --only igf,igemm --reps 10 --out gpurun_out/r1x_tune.json
gpu_step 300 gpurun_out/r1x_bench_e18.log python bench.py --steps 30 --warmup 10
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
