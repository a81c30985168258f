#!/bin/bash
# HIP-graph training step: graph test first, then the GPU suite and A/B bench (--graph 0 / 1) at batch 256 and 64.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-graph}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/${TAG}_gtest.log python -u -m pytest tests/gpu/test_graph.py -x -v --timeout 200 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_gtest.log && ! grep -q " failed\| error" gpurun_out/${TAG}_gtest.log || { echo "graph test failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 600 gpurun_out/${TAG}_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
gpu_step 300 gpurun_out/${TAG}_g0.log python bench.py --steps 30 --warmup 5 --graph 0
gpu_step 300 gpurun_out/${TAG}_g1.log python bench.py --steps 30 --warmup 5 --graph 1
gpu_step 300 gpurun_out/${TAG}_b64g0.log python bench.py --steps 30 --warmup 5 --graph 0 --batch 64
gpu_step 300 gpurun_out/${TAG}_b64g1.log python bench.py --steps 30 --warmup 5 --graph 1 --batch 64
gpu_step 300 gpurun_out/${TAG}_qg1.log python bench.py --model QuickNetLarge --steps 20 --warmup 5 --graph 1
echo done >> gpurun_out/progress.txt
