# Round 6: max-pool forward and backward with the window size at compile time (all taps
# loaded before the comparisons) vs the runtime-k loop (ZK_MAXPOOL_RT, temporary
# knob): tools/pool_lab.py, the pooling / QuickNet GPU tests, QuickNet-Large A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
ZK_MAXPOOL_RT=1 timeout -k 10 200 python -u tools/pool_lab.py --tag old > gpurun_out/pool_old.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/pool_lab.py --tag new > gpurun_out/pool_new.log 2>&1 || exit $?
grep -h maxpool gpurun_out/pool_old.log gpurun_out/pool_new.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_norm_pool.py tests/gpu/test_models_gpu.py tests/gpu/test_determinism.py > gpurun_out/pool_tests.log 2>&1 || { tail -30 gpurun_out/pool_tests.log; exit 1; }
tail -1 gpurun_out/pool_tests.log
run() {
  if [ "$2" = old ]; then export ZK_MAXPOOL_RT=1; else unset ZK_MAXPOOL_RT; fi
  timeout -k 10 400 python -u bench.py --model QuickNetLarge --batch 1024 --steps 30 > gpurun_out/pool_$1.log 2>&1 || exit $?
  echo "$1 $(tail -1 gpurun_out/pool_$1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run qnl_old1 old
run qnl_new1 new
run qnl_old2 old
run qnl_new2 new
