#!/bin/bash
# PMC passes (one counter group per run) on single binary-conv kernels.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-pmc}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
export PYTHONPATH=$GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
for spec in "dgrad 56,56,64,64,1" "dgrad 28,28,128,128,1" "fwd4 56,56,64,64,1" "wgrad 56,56,64,64,1"; do
  set -- $spec
  op=$1; shape=$2; nm=${op}_${shape//,/_}
  gpu_step 120 gpurun_out/${TAG}_${nm}_time.log python tools/one_conv.py --op $op --shape $shape --reps 50
  cd /tmp && export TMPDIR=/tmp
  gpu_step 90 $R/gpurun_out/${TAG}_${nm}_p1.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/${TAG}_${nm}_p1 -o run --output-format csv -- python $R/tools/one_conv.py --op $op --shape $shape --reps 5
  gpu_step 90 $R/gpurun_out/${TAG}_${nm}_p2.log timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/${TAG}_${nm}_p2 -o run --output-format csv -- python $R/tools/one_conv.py --op $op --shape $shape --reps 5
  gpu_step 90 $R/gpurun_out/${TAG}_${nm}_p3.log timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/${TAG}_${nm}_p3 -o run --output-format csv -- python $R/tools/one_conv.py --op $op --shape $shape --reps 5
  cd $R
done
echo done >> gpurun_out/progress.txt
