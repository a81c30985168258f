#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1o_test.log python -m pytest tests/gpu/test_bconv_bwd_kernels.py -q -x -k "fwd"
gpu_step 600 gpurun_out/r1o_pytest_gpu.log python -m pytest tests/gpu -q -x
gpu_step 500 gpurun_out/r1o_tune.log python tools/tune_bconv.py --only igf,fwd --reps 10 --out gpurun_out/r1o_tune.json
gpu_step 300 gpurun_out/r1o_bench_e18.log python bench.py --steps 30 --warmup 10
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/r1o_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r1o_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
