"""Float BatchNorm backward sums reduced in the consuming 1x1 conv's data-
gradient epilogue (``runtime.bn_bwd_fuse``: ``zk_igemm_dgrad_bsums``,
``norm_pool.FloatBnSum``) and the 1-bit ReLU mask of the residual BN tail.

A ResNet-50 bottleneck (identity and downsampling forms) runs forward and
backward with the fusion on and off; every gradient must agree (the fused
sums add the same products in another order: relative differences at the
1e-3 level), the fused path must really have been taken for the BNs whose
output feeds only a 1x1 conv, and a repeat of the fused run is bit-identical
(per-tile partials summed in a fixed order, no atomics)."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _grads(blk, x, g):
    xx = x.clone().requires_grad_(True)
    out = blk(xx)
    out.backward(g)
    return [out.float(), xx.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]


@pytest.mark.parametrize("cin,width,stride", [(256, 64, 1), (64, 64, 1), (256, 128, 2)])
def test_fused_bn_backward_sums_match(monkeypatch, cin, width, stride):
    from zookeeper_amd.models.resnet import Bottleneck
    from zookeeper_amd.ops import norm_pool
    from zookeeper_amd.ops.options import OPTS

    torch.manual_seed(4)
    blk = Bottleneck(cin, width, stride).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blk.modules():
            if hasattr(m, "running_var"):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    x = _cl(torch.randn(4, cin, 14, 14, device="cuda")).to(torch.bfloat16)
    ho = 14 // stride
    g = _cl(torch.randn(4, width * 4, ho, ho, device="cuda")).to(torch.bfloat16)

    taken = []
    orig = norm_pool.FloatBnSum.reduced

    def spy(self, dout):
        ok = orig(self, dout)
        taken.append(ok)
        return ok

    monkeypatch.setattr(norm_pool.FloatBnSum, "reduced", spy)
    res = []
    for fuse in (True, False, True):
        monkeypatch.setattr(OPTS, "bn_bwd_fuse", fuse)
        res.append(_grads(copy.deepcopy(blk), x, g))
    for a, b in zip(res[0], res[2]):
        assert torch.equal(a, b)  # fused: bit-reproducible
    res = res[:2]
    # bn2 -> conv3 always fuses (a 1x1 conv computes bn2's whole gradient)
    assert any(taken), taken
    (o1, *g1), (o2, *g2) = res
    assert torch.equal(o1, o2)  # the forward is unchanged
    for a, b in zip(g1, g2):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 5e-3


def test_masked_residual_handoff_bit_identical(monkeypatch):
    """An identity bottleneck's tail hands its gradient and ReLU mask to
    conv1's data-gradient epilogue, which masks and adds it (no g * mask
    tensor): gradients bit-identical to the materialised hand-off."""
    from zookeeper_amd.models.resnet import Bottleneck
    from zookeeper_amd.ops.options import OPTS

    torch.manual_seed(6)
    blk = Bottleneck(256, 64, 1).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blk.modules():
            if hasattr(m, "running_var"):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    x = _cl(torch.randn(4, 256, 14, 14, device="cuda")).to(torch.bfloat16)
    g = _cl(torch.randn(4, 256, 14, 14, device="cuda")).to(torch.bfloat16)
    res = []
    for masked in (True, False):
        monkeypatch.setattr(OPTS, "bn_masked_handoff", masked)
        res.append(_grads(copy.deepcopy(blk), x, g))
    for a, b in zip(*res):
        assert torch.equal(a, b)
