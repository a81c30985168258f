#!/bin/bash
# conv3 weight-gradient kernel: numerics (all variants) then tuning vs the current kernels.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-wg3}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
export PYTHONPATH=.
gpu_step 400 gpurun_out/${TAG}_test.log python -u -m pytest tests/gpu/test_bconv_bwd_kernels.py -k igemm_wgrad -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_test.log && ! grep -q " failed\| error" gpurun_out/${TAG}_test.log || { echo "tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 600 gpurun_out/${TAG}_tune.log python -u tools/tune_bconv.py --only igw --igw 4,7,20,27,28,29,30,32,33,34 --tbs 256,384,512,768,1024,2048 --out gpurun_out/${TAG}_tune.json
echo done >> gpurun_out/progress.txt
