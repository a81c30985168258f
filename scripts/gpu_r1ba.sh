#!/bin/bash
# Long timed windows (>= 50 steps, SURVEY §6 protocol) with clock snapshots.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
timeout -k 5 30 rocm-smi --showclocks --showtemp --showpower > gpurun_out/r1ba_smi_before.txt 2>&1 || true
gpu_step 400 gpurun_out/r1ba_e18.log python bench.py --steps 200 --warmup 10
timeout -k 5 30 rocm-smi --showclocks --showtemp --showpower > gpurun_out/r1ba_smi_after_e18.txt 2>&1 || true
gpu_step 400 gpurun_out/r1ba_qnl.log python bench.py --model QuickNetLarge --steps 100 --warmup 10
gpu_step 400 gpurun_out/r1ba_r50.log python bench.py --model ResNet50 --steps 50 --warmup 5
gpu_step 400 gpurun_out/r1ba_e18_b256.log python bench.py --steps 100 --warmup 10 --batch 256
echo done >> gpurun_out/progress.txt
