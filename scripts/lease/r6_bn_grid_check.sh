# Round 6: the BN grid caps in the defaults -- full GPU suite, smoke, default
# E18 bench, ResNet-50 and QuickNet-Large b1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -30 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log
timeout -k 10 400 python -u bench.py --model ResNet50 --batch 1024 --steps 20 > gpurun_out/bench_r50.log 2>&1 || exit $?
tail -1 gpurun_out/bench_r50.log
timeout -k 10 400 python -u bench.py --model QuickNetLarge --batch 1024 --steps 30 > gpurun_out/bench_qnl.log 2>&1 || exit $?
tail -1 gpurun_out/bench_qnl.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default2.log
