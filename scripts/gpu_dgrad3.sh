#!/bin/bash
# conv3 dgrad variants: numerics (all variants) then tuning on the E18 shapes.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-dg3}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
export PYTHONPATH=.
gpu_step 400 gpurun_out/${TAG}_test.log python -u -m pytest tests/gpu/test_bconv_bwd_kernels.py tests/gpu/test_fp4_forward.py -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_test.log && ! grep -q " failed\| error" gpurun_out/${TAG}_test.log || { echo "tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 600 gpurun_out/${TAG}_tune.log python -u tools/tune_bconv.py --only igemm --out gpurun_out/${TAG}_tune.json
echo done >> gpurun_out/progress.txt
