#!/bin/bash
# dgrad epilogue with the residual gradient: numerics, then single-kernel timings.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-dres}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
export PYTHONPATH=.
gpu_step 400 gpurun_out/${TAG}_test.log python -u -m pytest tests/gpu/test_bconv_bwd_kernels.py tests/gpu/test_binary_block.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_test.log && ! grep -q " failed\| error" gpurun_out/${TAG}_test.log || { echo "tests failed" >> gpurun_out/progress.txt; exit 1; }
for spec in "56,56,64,64,1 27" "56,56,64,64,1 20" "28,28,128,128,1 23" "28,28,128,128,1 27" "14,14,256,256,1 14" "7,7,512,512,1 24" "56,56,64,128,2 7" "28,28,128,256,2 0"; do
  set -- $spec
  gpu_step 60 gpurun_out/${TAG}_t.log python tools/one_conv.py --op dgrad --shape $1 --variant $2 --reps 50
  cat gpurun_out/${TAG}_t.log >> gpurun_out/${TAG}_times.log
done
echo done >> gpurun_out/progress.txt
