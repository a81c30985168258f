# deep data gradient for the binary convs too (dgrad_deep=2): QuickNet-Large
# b1024 and E18 b1536, interleaved A/B; the deep-dgrad numerics tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
timeout -k 10 300 python -u -m pytest tests/gpu/test_bconv_bwd_kernels.py -q -k "igemm_dgrad_matches_reference" --timeout 120 --timeout-method thread > gpurun_out/deep_tests.log 2>&1 || exit $?
AB_STEPS=40 AB_ROUNDS=2 bash scripts/ab.sh --model,QuickNetLarge,--batch,1024 --model,QuickNetLarge,--batch,1024,--rt,dgrad_deep=2 - --rt,dgrad_deep=2
