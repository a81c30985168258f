#!/bin/bash
# gpu_iter.sh + the ResNet-50 bench:  bash scripts/gpu_iter2.sh TAG
TAG=${1:?tag}; shift
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 600 gpurun_out/${TAG}_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@"
grep -q " passed" gpurun_out/${TAG}_test.log && ! grep -q " failed\| error" gpurun_out/${TAG}_test.log || { echo "tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 300 gpurun_out/${TAG}_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/${TAG}_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/${TAG}_r50.log python bench.py --model ResNet50 --steps 10 --warmup 3
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
