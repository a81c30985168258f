#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-pq}
R=$GRAFT_REPO_ROOT
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$R/gpurun_out/${TAG}_qprof.log" rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_qprof" -o run --output-format csv -- python "$R/bench.py" --model QuickNetLarge --steps 8 --warmup 3
gpu_step 600 "$R/gpurun_out/${TAG}_eprof.log" rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_eprof" -o run --output-format csv -- python "$R/bench.py" --steps 8 --warmup 3
gzip -f $R/gpurun_out/${TAG}_*prof/run_kernel_trace.csv
echo done >> "$R/gpurun_out/progress.txt"
