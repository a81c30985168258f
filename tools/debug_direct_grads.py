"""Compare trainer (direct-grad) vs plain autograd gradients per parameter,
and check that nothing is written into the flat buffer's alignment padding."""
import copy
import torch
from zookeeper_amd.models.binary_resnet import BinaryResNetE
from zookeeper_amd.parallel.dist import DistInfo
from zookeeper_amd.core import configure
from zookeeper_amd.train import Adam, Trainer

torch.manual_seed(0)
base = BinaryResNetE((64, 64, 3), 10, backend="hip").cuda().to(memory_format=torch.channels_last)
x = torch.randn(8, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 10, (8,), device="cuda")
model = copy.deepcopy(base)
spec = Adam(); configure(spec, {"learning_rate": 1e-3})
tr = Trainer(model, "sparse_categorical_crossentropy", spec, DistInfo(device=torch.device("cuda")))
tr.flat.zero_grad()
loss, _ = tr.loss_fn(tr.model(x), y)
loss.backward()
torch.cuda.synchronize()
mask = torch.ones(tr.flat.total, dtype=torch.bool, device="cuda")
for s in tr.flat.slots:
    mask[s.offset:s.offset + s.numel] = False
pad = tr.flat.grad[mask]
print("padding nonzero:", int((pad != 0).sum()), "of", pad.numel())
gd = {s.name: s.param.grad.detach().float().clone() for s in tr.flat.slots}
plain = copy.deepcopy(base)
loss2, _ = tr.loss_fn(plain(x), y)
loss2.backward()
print("loss", loss.item(), loss2.item())
for name, p in plain.named_parameters():
    if name not in gd:
        continue
    a, b = gd[name], p.grad.float()
    rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
    print(f"{name:40s} rel={rel:.3e} |a|={a.norm().item():.3e} |b|={b.norm().item():.3e}")
