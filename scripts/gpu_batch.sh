#!/bin/bash
# E18 throughput vs per-GPU batch.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-batch}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
for b in 256 384 512 768; do
  gpu_step 300 gpurun_out/${TAG}_b$b.log python bench.py --steps 20 --warmup 5 --batch $b
done
echo done >> gpurun_out/progress.txt
