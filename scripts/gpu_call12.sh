# pipelined stem F2: bit-identity tests, E18 A/B (stem_pool_pp on / off),
# then a kernel-trace profile of the default E18 step
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_stem.py -v --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 || exit $?
AB_STEPS=60 AB_ROUNDS=2 bash scripts/ab.sh - --rt,stem_pool_pp=False || exit $?
bash scripts/gpu.sh prof:BinaryResNetE18:1536
