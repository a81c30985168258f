#!/bin/bash
# Host-side cost of a training step: cProfile over bench.py (eager), plus QuickNetLarge graph A/B.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-host}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/${TAG}_cprof.log python -m cProfile -o gpurun_out/${TAG}.prof bench.py --steps 40 --warmup 5 --graph 0
python -c "import pstats; s=pstats.Stats('gpurun_out/${TAG}.prof'); s.sort_stats('tottime').print_stats(45); s.sort_stats('cumulative').print_stats(40)" > gpurun_out/${TAG}_pstats.txt 2>&1
gpu_step 300 gpurun_out/${TAG}_qg0.log python bench.py --model QuickNetLarge --steps 20 --warmup 5 --graph 0
gpu_step 300 gpurun_out/${TAG}_qg1.log python bench.py --model QuickNetLarge --steps 20 --warmup 5 --graph 1
ZK_WGRAD_SIDE=0 gpu_step 300 gpurun_out/${TAG}_qg1ns.log python bench.py --model QuickNetLarge --steps 20 --warmup 5 --graph 1
echo done >> gpurun_out/progress.txt
