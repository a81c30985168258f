#!/bin/bash
# A/B: side-stream weight gradients on/off and HIP stream priorities, E18 batch 512.
source "$GRAFT_REPO_ROOT/scripts/gpu_check.sh"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
echo "start $(date +%T)" > gpurun_out/progress.txt
python -c "import torch; print('prio range', torch.cuda.Stream.priority_range())" > gpurun_out/prio_range.log 2>&1
for cfg in "base1:" "side0:ZK_WGRAD_SIDE=0" "sidehi:ZK_WGRAD_PRIORITY=-1" "mainhi:ZK_MAIN_PRIORITY=-1" "base2:"; do
  tag=${cfg%%:*}; envs=${cfg#*:}
  gpu_step 300 gpurun_out/prio_$tag.log env $envs python bench.py --steps 40 --warmup 5
done
echo done >> gpurun_out/progress.txt
