# forced 1-rank data parallelism: ProcessGroupNCCL vs the in-tree RCCL
# communicator (comm_backend=native), against the plain run
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.jsonl gpurun_out/progress.txt
AB_STEPS=30 AB_ROUNDS=1 bash scripts/ab.sh - --force-dp --force-dp,--rt,comm_backend=native
