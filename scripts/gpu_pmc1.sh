#!/bin/bash
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
gpu_step 400 "$R/gpurun_out/pmc1.log" rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d "$R/gpurun_out/pmc1" -o run --output-format csv -- python "$R/tools/tune_bconv.py" --reps 2
gpu_step 400 "$R/gpurun_out/pmc2.log" rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD -d "$R/gpurun_out/pmc2" -o run --output-format csv -- python "$R/tools/tune_bconv.py" --reps 2
echo done >> "$R/gpurun_out/progress.txt"
