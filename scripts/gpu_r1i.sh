#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 400 gpurun_out/r1i_pytest_gpu.log python -m pytest tests -m gpu -q
gpu_step 600 gpurun_out/r1i_bench_hip.log python bench.py --backend hip --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1i_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1i_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --backend hip --steps 5 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
