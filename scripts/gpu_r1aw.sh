#!/bin/bash
# Re-entry check after container rebuild: smoke, whole GPU suite, default bench + kernel stats.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1aw_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
gpu_step 900 gpurun_out/r1aw_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
gpu_step 300 gpurun_out/r1aw_e18.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/r1aw_qnl.log python bench.py --model QuickNetLarge --steps 20 --warmup 5
gpu_step 300 gpurun_out/r1aw_r50.log python bench.py --model ResNet50 --steps 10 --warmup 3
echo done >> gpurun_out/progress.txt
