# float-conv weight gradients on the side stream: bit-identity test, then
# ResNet-50 b1024 A/B and an E18 check
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_determinism.py -v -k "float_wgrad or resnet" --timeout 120 --timeout-method thread > gpurun_out/fside_tests.log 2>&1 || exit $?
AB_STEPS=30 AB_ROUNDS=2 bash scripts/ab.sh --model,ResNet50,--batch,1024 --model,ResNet50,--batch,1024,--rt,float_wgrad_side_stream=False - --rt,float_wgrad_side_stream=False
