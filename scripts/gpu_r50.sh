#!/bin/bash
# ResNet-50: float 3x3 convs on the MFMA kernels vs MIOpen, numerics + A/B bench + profile.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r50}
echo "start $TAG $(date +%T)" > gpurun_out/progress.txt
gpu_step 300 gpurun_out/${TAG}_c3test.log python -u -m pytest tests/gpu/test_conv3x3.py -x -v --timeout 120 --timeout-method thread
grep -q " passed" gpurun_out/${TAG}_c3test.log && ! grep -q " failed\| error" gpurun_out/${TAG}_c3test.log || { echo "conv3x3 tests failed" >> gpurun_out/progress.txt; exit 1; }
gpu_step 600 gpurun_out/${TAG}_test.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
ZK_CONV3_MFMA=0 gpu_step 300 gpurun_out/${TAG}_miopen.log python bench.py --model ResNet50 --steps 20 --warmup 5
gpu_step 300 gpurun_out/${TAG}_mfma.log python bench.py --model ResNet50 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
gpu_step 600 "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log" rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --model ResNet50 --steps 6 --warmup 3
echo done >> "$GRAFT_REPO_ROOT/gpurun_out/progress.txt"
