# held-back side-stream weight gradients: bit-identity test, then E18 A/B
# (off / stage 1 held / stages 1-2 held)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_determinism.py -v -k held --timeout 120 --timeout-method thread > gpurun_out/hold_tests.log 2>&1 || exit $?
AB_STEPS=60 AB_ROUNDS=2 bash scripts/ab.sh - --rt,wgrad_hold_hw=3136 --rt,wgrad_hold_hw=784
