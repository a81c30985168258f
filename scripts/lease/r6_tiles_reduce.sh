# Round 6: coalesced bn_bwd_tiles_reduce -- its bit-exact test and the BN / model
# GPU tests, tools/bn_lab.py, ResNet-50 b1024 bench and kernel-trace profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/gpu/test_norm_pool.py tests/gpu/test_bn_fusion.py tests/gpu/test_models_gpu.py tests/gpu/test_determinism.py tests/gpu/test_pointwise.py > gpurun_out/tr_tests.log 2>&1 || { tail -30 gpurun_out/tr_tests.log; exit 1; }
tail -1 gpurun_out/tr_tests.log
timeout -k 10 200 python -u tools/bn_lab.py --tag tr --json gpurun_out/bn_lab_tr.jsonl > gpurun_out/bn_lab_tr.log 2>&1 || exit $?
grep tiles gpurun_out/bn_lab_tr.log
timeout -k 10 400 python -u bench.py --model ResNet50 --batch 1024 --steps 20 > gpurun_out/tr_r50.log 2>&1 || exit $?
tail -1 gpurun_out/tr_r50.log | cut -c1-200
rm -rf gpurun_out/prof_r50
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run --output-format csv -- python3 bench.py --model ResNet50 --batch 1024 --steps 12 --warmup 6 --graph 0 > gpurun_out/prof_r50.log 2>&1 || exit $?
echo prof done
