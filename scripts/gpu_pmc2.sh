#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
gpu_step 400 "$R/gpurun_out/pmc3.log" rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TA_BUSY_avr SQ_INSTS_VALU SQ_INSTS_MFMA -d "$R/gpurun_out/pmc3" -o run --output-format csv -- python "$R/tools/tune_bconv.py" --only igf --reps 2
gpu_step 400 "$R/gpurun_out/pmc4.log" rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES -d "$R/gpurun_out/pmc4" -o run --output-format csv -- python "$R/tools/tune_bconv.py" --only igf --reps 2
echo done >> "$R/gpurun_out/progress.txt"
