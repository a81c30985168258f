# wgrad_rows lab only (+ its tests)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/gpu/test_wgrad_rows.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t14.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/wgrad_lab.py --shapes 56,64,64/28,128,128 --rounds 2 --out gpurun_out/wlab14.jsonl > gpurun_out/wlab14.log 2>&1
