#!/bin/bash
# Rehearse the driver's multi-rank bench launch (torch.distributed.run, 2 ranks)
# on the box's one GPU over gloo: bench.py's DP path end to end with the HIP kernels.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
export ZK_DIST_BACKEND=gloo
gpu_step 400 gpurun_out/r1ay_dp2.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 10 --warmup 3 --batch 128
unset ZK_DIST_BACKEND
gpu_step 300 gpurun_out/r1ay_dp1.log python bench.py --gpus 1 --steps 10 --warmup 3 --batch 128
echo done >> gpurun_out/progress.txt
