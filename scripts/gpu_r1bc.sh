#!/bin/bash
# PMC passes over an E18 training step (batch 256): MFMA busy / LDS conflicts, HBM fetch, HBM write.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
gpu_step 150 "$R/gpurun_out/r1bc_pmc1.log" timeout -s KILL 140 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d "$R/gpurun_out/r1bc_pmc1" -o run --output-format csv -- python "$R/bench.py" --steps 2 --warmup 2 --batch 256 --graph 0
gpu_step 150 "$R/gpurun_out/r1bc_pmc2.log" timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/r1bc_pmc2" -o run --output-format csv -- python "$R/bench.py" --steps 2 --warmup 2 --batch 256 --graph 0
gpu_step 150 "$R/gpurun_out/r1bc_pmc3.log" timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/r1bc_pmc3" -o run --output-format csv -- python "$R/bench.py" --steps 2 --warmup 2 --batch 256 --graph 0
echo done >> "$R/gpurun_out/progress.txt"
