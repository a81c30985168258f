# forced 1-rank RCCL data parallelism overhead: plain vs --force-dp, with comm
# timing off, with CPU affinity off
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=30 AB_ROUNDS=1 bash scripts/ab.sh - --force-dp --force-dp,--rt,comm_timing=False --force-dp,--rt,cpu_affinity=False --force-dp,--rt,wgrad_side_stream=False
