#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 900 gpurun_out/tune_bconv2.log python tools/tune_bconv.py --out gpurun_out/tune_bconv2.json
echo done >> gpurun_out/progress.txt
