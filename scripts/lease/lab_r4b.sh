#!/bin/bash
# Round-4 deep-GEMM check: numerics of the phased kernels, then standalone
# timings against the previous defaults at batch 1536.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
P="$OUT/progress.txt"
echo "r4b start $(date +%T)" >> "$P"
timeout -k 10 400 python -u -m pytest tests/gpu/test_bconv_bwd_kernels.py -x -q --timeout 120 \
  --timeout-method thread -k "igemm_dgrad_matches or igemm_wgrad_matches or dgrad_wgrad" \
  > "$OUT/r4b_tests.log" 2>&1 || { echo "tests failed $?" >> "$P"; exit 1; }
echo "tests ok $(date +%T)" >> "$P"
SH="14+14+256+256+1/7+7+512+512+1"
timeout -k 10 300 python -u tools/gemm_roofline.py --batch 1536 --ops dgrad --shapes "$SH/28+28+128+128+1" \
  --dvariants=60+45+27 > "$OUT/r4b_dgrad.log" 2>&1 || exit $?
echo "dgrad done $(date +%T)" >> "$P"
timeout -k 10 300 python -u tools/gemm_roofline.py --batch 1536 --ops wgrad --shapes "$SH" \
  --wvariants=60+8+12 > "$OUT/r4b_wgrad_atomic.log" 2>&1 || exit $?
echo "wgrad atomic done $(date +%T)" >> "$P"
timeout -k 10 300 python -u tools/gemm_roofline.py --batch 1536 --ops wgrad --shapes "$SH" \
  --wgrad-mode slab --wvariants=60+8+12 > "$OUT/r4b_wgrad_slab.log" 2>&1 || exit $?
echo "wgrad slab done $(date +%T)" >> "$P"
