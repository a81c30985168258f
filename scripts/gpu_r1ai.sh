#!/bin/bash
# Striped BN statistics + tuned FP4 tiles: numerics, suite, tile timings, bench, profile.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1ai_fp4.log python -u -m pytest tests/gpu/test_fp4_forward.py tests/gpu/test_stem.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/r1ai_fp4.log && ! grep -q "failed\|error" gpurun_out/r1ai_fp4.log || { echo "fp4/stem tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 600 gpurun_out/r1ai_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
gpu_step 300 gpurun_out/r1ai_tune.log python tools/tune_bconv.py --only igf,igf4 --reps 10
gpu_step 300 gpurun_out/r1ai_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/r1ai_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1ai_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1ai_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
