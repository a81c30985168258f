#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 400 gpurun_out/r1j_pytest_gpu.log python -m pytest tests/gpu/test_trainer_hip.py -q
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1j_prof_qnl.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1j_prof_qnl" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --model QuickNetLarge --steps 3 --warmup 2
gpu_step 300 "$GRAFT_REPO_ROOT/gpurun_out/r1j_counters.log" rocprofv3 -L
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
