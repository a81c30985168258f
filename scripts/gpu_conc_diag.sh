#!/bin/bash
# Is a rank's gradient corrupted when another process shares the GPU?  Run
# the world-size-1 worker alone twice, then two copies concurrently, and
# compare final parameters (per-layer maxima for the outliers).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/cd
export PYTHONPATH=$GRAFT_REPO_ROOT
for i in 1 2; do
  mkdir -p gpurun_out/cd/solo$i
  timeout -k 10 120 python tests/dp_gpu_worker.py same gpurun_out/cd/solo$i > gpurun_out/cd/solo$i.log 2>&1 || exit 1
done
for r in 1 2 3; do
  mkdir -p gpurun_out/cd/a$r gpurun_out/cd/b$r
  timeout -k 10 120 python tests/dp_gpu_worker.py same gpurun_out/cd/a$r > gpurun_out/cd/a$r.log 2>&1 &
  pa=$!
  timeout -k 10 120 python tests/dp_gpu_worker.py same gpurun_out/cd/b$r > gpurun_out/cd/b$r.log 2>&1 &
  pb=$!
  wait $pa || exit 1
  wait $pb || exit 1
done
python -c "
import torch
from zookeeper_amd.models.binary_resnet import BinaryResNetE
from zookeeper_amd.parallel.flat import FlatParams
fp = FlatParams(BinaryResNetE((64, 64, 3), 10, 18, backend='hip'), torch.device('cpu'))
ks = ['solo1', 'solo2', 'a1', 'b1', 'a2', 'b2', 'a3', 'b3']
d = {k: torch.load(f'gpurun_out/cd/{k}/same_w1_r0.pt', weights_only=True)['params'] for k in ks}
ref = d['solo1']
for k in ks[1:]:
    diffs = sorted(((d[k][s.offset:s.offset + s.numel] - ref[s.offset:s.offset + s.numel]).abs().max().item(), s.name) for s in fp.slots)[::-1][:4]
    print(k, ((d[k] - ref).norm() / ref.norm()).item(), [(n, round(v, 6)) for v, n in diffs])
" > gpurun_out/cd/result.txt 2>&1
rm -f gpurun_out/cd/*/*.pt
