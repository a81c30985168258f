"""Float BatchNorm backward sums reduced in the consuming 1x1 conv's data-
gradient epilogue (``runtime.bn_bwd_fuse``: ``zk_igemm_dgrad_bsums``,
``norm_pool.FloatBnSum``) and the 1-bit ReLU mask of the residual BN tail.

A ResNet-50 bottleneck (identity and downsampling forms) runs forward and
backward with the fusion on and off; every gradient must agree (the fused
sums use fp32 atomics in a different order: relative differences at the
1e-3 level), and the fused path must really have been taken for the BNs whose
output feeds only a 1x1 conv."""

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
    for fuse in (True, False):
        monkeypatch.setattr(OPTS, "bn_bwd_fuse", fuse)
        res.append(_grads(copy.deepcopy(blk), x, g))
    # bn2 -> conv3 always fuses (a 1x1 conv computes bn2's whole gradient)
    assert any(taken), taken
    (o1, *g1), (o2, *g2) = res
    assert torch.equal(o1, o2)  # the forward is unchanged
    for a, b in zip(g1, g2):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 5e-3
