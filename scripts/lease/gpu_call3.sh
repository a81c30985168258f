# in-step A/B of the deep-gemm kernels, E18 kernel profile, ResNet-50 /
# QuickNet-Large benches
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_wgrad_rows.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t16.log 2>&1 || exit $?
AB_STEPS=60 AB_ROUNDS=2 bash scripts/ab.sh - --rt,dgrad_deep=False --rt,wgrad_deep=False || exit $?
bash scripts/gpu.sh prof:BinaryResNetE18:1536 bench:ResNet50:1024:60 bench:QuickNetLarge:1024:60
