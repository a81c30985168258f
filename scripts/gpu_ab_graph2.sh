#!/bin/bash
# graph auto mode at batch 256 / 128 / 64, and graph replay with the side stream off.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-graph2}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/${TAG}_gtest.log python -u -m pytest tests/gpu/test_graph.py -x -v --timeout 200 --timeout-method thread
gpu_step 300 gpurun_out/${TAG}_auto256.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/${TAG}_auto128.log python bench.py --steps 30 --warmup 5 --batch 128
gpu_step 300 gpurun_out/${TAG}_eager128.log python bench.py --steps 30 --warmup 5 --batch 128 --graph 0
gpu_step 300 gpurun_out/${TAG}_auto64.log python bench.py --steps 30 --warmup 5 --batch 64
ZK_WGRAD_SIDE=0 gpu_step 300 gpurun_out/${TAG}_g1noside.log python bench.py --steps 30 --warmup 5 --graph 1
gpu_step 300 gpurun_out/${TAG}_qauto.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
echo done >> gpurun_out/progress.txt
