#!/bin/bash
# Build (on the CPU host) and run the GEMM lab binaries on the GPU box:
#   gpurun -- bash tools/gemm_lab/run.sh <binary> [<binary> ...]
# Each binary runs the dense 8192^3 case and the E18 GEMM shapes as dense
# equivalents (stage-3 / stage-4 data gradient: M = pixels, N = Cin, K = 9 Cout).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
for b in "$@"; do
  for shape in "8192 8192 8192 10" "4096 4096 4096 20" "200704 256 2304 10" "50176 512 4608 10" \
               "802816 128 1152 5"; do
    timeout -k 5 60 "tools/gemm_lab/$b" $shape >> "$OUT/gemm_lab.log" 2>&1
    rc=$?
    echo "[$b $shape] rc=$rc" >> "$OUT/gemm_lab.log"
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
# PMC passes: ZK_LAB_PMC="<binary> <args>" runs three counter groups over it
if [ -n "${ZK_LAB_PMC:-}" ]; then
  R="$(pwd)"
  i=0
  for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
              "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE GRBM_COUNT" \
              "FETCH_SIZE TCC_HIT_sum"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $pass -d "$R/$OUT/labpmc_$i" -o run --output-format csv \
      -- "$R/tools/gemm_lab/"$ZK_LAB_PMC > "$R/$OUT/labpmc_$i.log" 2>&1) || exit $?
  done
fi
