#!/bin/bash
# Final check at the round's HEAD: what the driver runs (GPU suite, smoke, default bench).
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 900 gpurun_out/r1bb_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
gpu_step 300 gpurun_out/r1bb_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')"
gpu_step 300 gpurun_out/r1bb_bench.log python bench.py
echo done >> gpurun_out/progress.txt
