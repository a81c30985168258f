# Round 6: 1x1 GEMM default tile (41 instead of 45 for N % 256 == 0, K < 1024):
# tools/tune_pw.py defaults at batch 1024, the GEMM / model GPU tests, and
# ResNet-50 b1024 benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tune_pw.py --batch 1024 --reps 10 --variants 41-43 > gpurun_out/pw_new_b1024.log 2>&1 || exit $?
grep "==" gpurun_out/pw_new_b1024.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_pointwise.py tests/gpu/test_bn_fusion.py tests/gpu/test_models_gpu.py tests/gpu/test_determinism.py tests/gpu/test_conv_family.py > gpurun_out/pw_tests.log 2>&1 || { tail -30 gpurun_out/pw_tests.log; exit 1; }
tail -1 gpurun_out/pw_tests.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model ResNet50 --batch 1024 --steps 20 > gpurun_out/pw_r50_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/pw_r50_$i.log | cut -c1-160
done
timeout -k 10 400 python -u bench.py --model QuickNetLarge --batch 1024 --steps 30 > gpurun_out/pw_qnl.log 2>&1 || exit $?
tail -1 gpurun_out/pw_qnl.log | cut -c1-160
