#!/bin/bash
# Side-stream weight gradients: GPU suite, then A/B bench (ZK_WGRAD_SIDE=0 / 1) and a profile.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-side}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/${TAG}_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_test.log && ! grep -q " failed\| error" gpurun_out/${TAG}_test.log || { echo "tests failed" >> gpurun_out/progress.txt; exit 1; }
ZK_WGRAD_SIDE=0 gpu_step 300 gpurun_out/${TAG}_off.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/${TAG}_on.log python bench.py --steps 30 --warmup 5
ZK_WGRAD_SIDE=0 gpu_step 300 gpurun_out/${TAG}_off2.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/${TAG}_on2.log python bench.py --steps 30 --warmup 5
ZK_WGRAD_SIDE=0 gpu_step 300 gpurun_out/${TAG}_qoff.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/${TAG}_qon.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
echo done >> gpurun_out/progress.txt
