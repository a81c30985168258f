# loader-stream preprocessing (+ fused stem pack): tests, then an interleaved
# E18 A/B against runtime.loader_preprocess=False, 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_stem.py tests/gpu/test_loader_gpu.py tests/gpu/test_kernels_elementwise.py -v --timeout 120 --timeout-method thread > gpurun_out/prep_tests.log 2>&1 || exit $?
AB_STEPS=60 AB_ROUNDS=2 bash scripts/ab.sh - --rt,loader_preprocess=False
