#!/bin/bash
# Round-4 baseline lab: dense GEMM lab on the E18 deep shapes + per-layer
# roofline at batch 1536 in both split-K modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
OUT=gpurun_out
mkdir -p "$OUT"
echo "lab start $(date +%T)" >> "$OUT/progress.txt"
bash tools/gemm_lab/run.sh g8 || exit $?
echo "lab done $(date +%T)" >> "$OUT/progress.txt"
timeout -k 10 300 python -u tools/gemm_roofline.py --batch 1536 --ops dgrad,wgrad \
  --json "$OUT/roof_b1536_atomic.json" > "$OUT/roof_b1536_atomic.log" 2>&1 || exit $?
echo "roof atomic done $(date +%T)" >> "$OUT/progress.txt"
timeout -k 10 300 python -u tools/gemm_roofline.py --batch 1536 --ops wgrad --wgrad-mode slab \
  --json "$OUT/roof_b1536_slab.json" > "$OUT/roof_b1536_slab.log" 2>&1 || exit $?
echo "roof slab done $(date +%T)" >> "$OUT/progress.txt"
