#!/bin/bash
# Re-tune the binary-conv tile variants at the default per-GPU batch (512).
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 500 gpurun_out/t512_tune.log python -u tools/tune_bconv.py --batch 512 --reps 10 --only igemm,igw,igf4 --tbs 512,1024,2048,4096 --out gpurun_out/t512_tune.json
echo done >> gpurun_out/progress.txt
