"""End to end on the GPU: the fused HIP training step of BinaryResNet-E18
(direct gradient accumulation into the flat buffer) produces the same
gradients as the pure-PyTorch fp32 oracle, and the full step runs."""

import copy

import pytest
import torch

from zookeeper_amd.models.binary_resnet import BinaryResNetE
from zookeeper_amd.parallel.dist import DistInfo

pytestmark = pytest.mark.gpu


def _grads(model, backend, x, y):
    from zookeeper_amd.core import configure
    from zookeeper_amd.train import Adam, Trainer

    model.set_backend(backend)
    spec = Adam()
    configure(spec, {"learning_rate": 1e-3})
    tr = Trainer(model, "sparse_categorical_crossentropy", spec,
                 DistInfo(device=torch.device("cuda")))
    tr.flat.zero_grad()
    if backend == "torch":
        tr.model.float()
        logits = tr.model(x.float())
    else:
        logits = tr.model(x)
    loss, _ = tr.loss_fn(logits, y)
    loss.backward()
    torch.cuda.synchronize()
    return tr, {s.name: s.param.grad.detach().float().clone() for s in tr.flat.slots}


def test_e18_gradients_match_oracle():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    torch.manual_seed(0)
    base = BinaryResNetE((64, 64, 3), 10).cuda()
    x = torch.randn(8, 3, 64, 64, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")
    _, gh = _grads(copy.deepcopy(base), "hip", x, y)
    _, gr = _grads(copy.deepcopy(base), "torch", x, y)
    bad = []
    for name, a in gh.items():
        b = gr[name]
        cos = torch.nn.functional.cosine_similarity(a.flatten(), b.flatten(), dim=0).item()
        if b.norm() > 1e-6 and cos < 0.98:
            bad.append((name, round(cos, 4)))
    assert not bad, bad


def test_e18_training_step_runs_and_decreases_loss():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd.core import configure
    from zookeeper_amd.train import Adam, Trainer

    torch.manual_seed(1)
    model = BinaryResNetE((64, 64, 3), 10, backend="hip")
    spec = Adam()
    configure(spec, {"learning_rate": 2e-3})
    tr = Trainer(model, "sparse_categorical_crossentropy", spec,
                 DistInfo(device=torch.device("cuda")))
    x = torch.randn(16, 3, 64, 64, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    losses = [tr.train_step(x, y)[0].item() for _ in range(15)]
    assert all(map(lambda v: v == v, losses))  # finite
    assert losses[-1] < losses[0]
    # weight_clip keeps the latent binary kernels in [-1, 1]
    for name, p in tr.model.named_parameters():
        if name.endswith("conv.weight") and "body" in name:
            assert p.abs().max().item() <= 1.0 + 1e-6
