#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
gpu_step 400 "$R/gpurun_out/pmc5.log" rocprofv3 --pmc FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_WAVES -d "$R/gpurun_out/pmc5" -o run --output-format csv -- python "$R/tools/tune_stem.py" --reps 2
gpu_step 400 "$R/gpurun_out/pmc6.log" rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES -d "$R/gpurun_out/pmc6" -o run --output-format csv -- python "$R/tools/tune_stem.py" --reps 2
echo done >> "$R/gpurun_out/progress.txt"
