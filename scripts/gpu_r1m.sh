#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1m_test.log python -m pytest tests/gpu/test_bconv_bwd_kernels.py tests/gpu/test_binary_block.py -q -x
gpu_step 500 gpurun_out/r1m_tune.log python tools/tune_bconv.py --only igw --reps 10 --out gpurun_out/r1m_tune.json
echo done >> gpurun_out/progress.txt
