# Round 6: 32-lane-group f64 BN finalize -- full GPU suite, smoke, default E18
# bench, ResNet-50 b1024 bench and kernel-trace profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -40 gpurun_out/full_tests.log; exit 1; }
tail -1 gpurun_out/full_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_default.log | cut -c1-220
timeout -k 10 400 python -u bench.py --model ResNet50 --batch 1024 --steps 20 > gpurun_out/fin_r50.log 2>&1 || exit $?
tail -1 gpurun_out/fin_r50.log | cut -c1-200
rm -rf gpurun_out/prof_r50
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run --output-format csv -- python3 bench.py --model ResNet50 --batch 1024 --steps 12 --warmup 6 --graph 0 > gpurun_out/prof_r50.log 2>&1 || exit $?
echo prof done
