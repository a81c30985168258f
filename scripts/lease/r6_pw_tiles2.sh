# Round 6: 1x1 GEMM default tile, second step (43 for N % 256 == 0 and K <= 128):
# full GPU suite, smoke, default E18 bench, ResNet-50 x2 and QuickNet-Large b1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
tail -1 gpurun_out/full_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-200
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model ResNet50 --batch 1024 --steps 20 > gpurun_out/pw2_r50_$i.log 2>&1 || exit $?
  tail -1 gpurun_out/pw2_r50_$i.log | cut -c1-160
done
timeout -k 10 400 python -u bench.py --model QuickNetLarge --batch 1024 --steps 30 > gpurun_out/pw2_qnl.log 2>&1 || exit $?
tail -1 gpurun_out/pw2_qnl.log | cut -c1-160
