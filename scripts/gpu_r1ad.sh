#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
export ZK_PW_GEMM=0
gpu_step 300 gpurun_out/r1ad_qnl_nopw.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
unset ZK_PW_GEMM
gpu_step 300 gpurun_out/r1ad_qnl_pw.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1ad_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1ad_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --model QuickNetLarge --steps 10 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
