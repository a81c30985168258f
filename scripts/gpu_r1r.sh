#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1r_test_stem.log python -m pytest tests/gpu/test_stem.py -q -x
gpu_step 300 gpurun_out/r1r_tune_stem.log python tools/tune_stem.py
gpu_step 300 gpurun_out/r1r_bench_e18.log python bench.py --steps 30 --warmup 10
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
