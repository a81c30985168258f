#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-gdiag}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
export PYTHONPATH=.
ZK_WGRAD_SIDE=0 gpu_step 200 gpurun_out/${TAG}_noside.log python -u tools/graph_diag.py
gpu_step 200 gpurun_out/${TAG}_side.log python -u tools/graph_diag.py
echo done >> gpurun_out/progress.txt
