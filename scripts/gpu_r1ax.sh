#!/bin/bash
# Whole GPU suite after the DP-test tolerance fix (update-relative error).
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1ax_dp.log python -u -m pytest tests/gpu/test_dp_gpu.py -x -v --timeout 300 --timeout-method thread
gpu_step 900 gpurun_out/r1ax_test.log python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
echo done >> gpurun_out/progress.txt
