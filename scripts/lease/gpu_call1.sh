# One GPU call: wgrad_rows + binary-block tests, the standalone lab under a
# kernel trace, in-step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/gpu/test_wgrad_rows.py tests/gpu/test_binary_block.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t13.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wl13 -o wl -- python -u tools/wgrad_lab.py --shapes 56,64,64/28,128,128 --rounds 2 --out gpurun_out/wlab13.jsonl > gpurun_out/wlab13.log 2>&1 || exit $?
AB_STEPS=60 AB_ROUNDS=2 bash scripts/ab.sh - --rt,wgrad_fp4=False --rt,wgrad_rows=False
