#!/bin/bash
# Two ranks on the box's GPU over gloo: the GPU data-parallel path.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start dp $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/dp_test.log python -u -m pytest tests/gpu/test_dp_gpu.py -x -v --timeout 300 --timeout-method thread
echo done >> gpurun_out/progress.txt
