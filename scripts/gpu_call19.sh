# two-row BN apply: bit-identity test, then E18 A/B (bn_apply_unroll 1 / 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_binary_block.py -q -k "unrolled or shortcut_pool" --timeout 120 --timeout-method thread > gpurun_out/unroll_tests.log 2>&1 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh - --rt,bn_apply_unroll=2
