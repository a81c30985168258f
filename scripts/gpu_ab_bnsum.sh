source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; echo "start ab $(date +%T)" > gpurun_out/progress.txt
ZK_FUSE_BNSUM=0 gpu_step 300 gpurun_out/ab_nofuse.log python bench.py --steps 30 --warmup 5
gpu_step 300 gpurun_out/ab_fuse.log python bench.py --steps 30 --warmup 5
cd /tmp && export TMPDIR=/tmp
ZK_FUSE_BNSUM=0 gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/ab_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/ab_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3
