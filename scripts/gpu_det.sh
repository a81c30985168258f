#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-det}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/${TAG}_test.log python -u -m pytest tests/gpu/test_determinism.py -x -v --timeout 120 --timeout-method thread
echo done >> gpurun_out/progress.txt
