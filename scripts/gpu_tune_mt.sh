#!/bin/bash
# Multi-tile conv3 variants: numerics of every dgrad / FP4-forward tile, then tile timings.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-mt}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/${TAG}_kern.log python -u -m pytest tests/gpu/test_fp4_forward.py tests/gpu/test_bconv_bwd_kernels.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_kern.log && ! grep -q " failed\| error" gpurun_out/${TAG}_kern.log || { echo "kernel tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 400 gpurun_out/${TAG}_tune.log python tools/tune_bconv.py --only igemm,igf4 --reps 10
echo done >> gpurun_out/progress.txt
