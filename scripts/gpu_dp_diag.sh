#!/bin/bash
# Determinism diagnostics for the two-rank GPU DP test: world 1 twice,
# world 2 three times (same data); pairwise relative differences of the
# final parameters go to gpurun_out/dpd/result.txt.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/dpd
export PYTHONPATH=$GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 120 python tests/dp_gpu_worker.py same gpurun_out/dpd > gpurun_out/dpd/w1_$i.log 2>&1 && mv gpurun_out/dpd/same_w1_r0.pt gpurun_out/dpd/w1_$i.pt || exit 1
done
for i in 1 2 3; do
  timeout -k 10 180 python -c "
import sys; sys.path.insert(0,'.')
from zookeeper_amd.parallel.launch import spawn
sys.exit(spawn([sys.executable, 'tests/dp_gpu_worker.py', 'same', 'gpurun_out/dpd'], 2))" > gpurun_out/dpd/w2_$i.log 2>&1 && mv gpurun_out/dpd/same_w2_r0.pt gpurun_out/dpd/w2_$i.pt || exit 1
done
python -c "
import torch
ks = ['w1_1', 'w1_2', 'w2_1', 'w2_2', 'w2_3']
d = {k: torch.load(f'gpurun_out/dpd/{k}.pt', weights_only=True)['params'] for k in ks}
for i, a in enumerate(ks):
    for b in ks[i + 1:]:
        print(a, b, ((d[a] - d[b]).norm() / d[b].norm()).item(), (d[a] - d[b]).abs().max().item())
from zookeeper_amd.models.binary_resnet import BinaryResNetE
from zookeeper_amd.parallel.flat import FlatParams
fp = FlatParams(BinaryResNetE((64, 64, 3), 10, 18, backend='hip'), torch.device('cpu'))
for k in ks[2:]:
    diffs = sorted(((d[k][s.offset:s.offset + s.numel] - d['w1_1'][s.offset:s.offset + s.numel]).abs().max().item(), s.name) for s in fp.slots)[::-1][:8]
    print(k, [(n, round(v, 6)) for v, n in diffs])
" > gpurun_out/dpd/result.txt 2>&1
rm -f gpurun_out/dpd/*.pt
