#!/bin/bash
# Batch-512 tile defaults: numerics, whole GPU suite, E18 / QuickNetLarge / ResNet-50 bench.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1av_tiles.log python -u -m pytest tests/gpu/test_tile_defaults.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r1av_tiles.log && ! grep -q "failed\|error" gpurun_out/r1av_tiles.log || { echo "tile tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 600 gpurun_out/r1av_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
gpu_step 300 gpurun_out/r1av_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/r1av_e18_256.log python bench.py --steps 30 --warmup 5 --batch 256
gpu_step 300 gpurun_out/r1av_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/r1av_r50.log python bench.py --model ResNet50 --steps 10 --warmup 3
echo done >> gpurun_out/progress.txt
