#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/r1q_test_stem.log python -m pytest tests/gpu/test_stem.py -q -x
gpu_step 300 gpurun_out/r1q_tune_stem.log python tools/tune_stem.py
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
gpu_step 400 "$R/gpurun_out/r1q_pmc.log" rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d "$R/gpurun_out/r1q_pmc" -o run --output-format csv -- python "$R/tools/tune_stem.py" --reps 2
echo done >> "$R/gpurun_out/progress.txt"
