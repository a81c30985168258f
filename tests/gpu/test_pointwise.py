"""1×1 convolution as MFMA implicit GEMMs (ops/pointwise.py) vs an fp32
``F.conv2d`` oracle: output, input gradient and weight gradient,
including accumulation into a pre-filled flat-gradient view."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("B,cin,cout,hw", [(4, 64, 128, 28), (2, 256, 512, 7), (3, 128, 64, 9)])
def test_conv1x1_matches_fp32(B, cin, cout, hw):
    from zookeeper_amd.ops.pointwise import conv1x1

    torch.manual_seed(0)
    x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = torch.randn(cout, cin, 1, 1, device="cuda", requires_grad=True)
    y = conv1x1(x, w)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(torch.bfloat16).float().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2


def test_conv1x1_accumulates_into_direct_grad():
    from zookeeper_amd.ops.pointwise import conv1x1

    torch.manual_seed(1)
    x = torch.randn(2, 64, 14, 14, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.randn(128, 64, 1, 1, device="cuda", requires_grad=True)
    w.grad = torch.full_like(w, 0.5)
    w._zk_direct_grad = True
    y = conv1x1(x, w)
    g = torch.randn_like(y)
    y.backward(g)
    ref = torch.einsum("bohw,bihw->oi", g.float(), x.float()).view(128, 64, 1, 1) + 0.5
    assert _rel(w.grad, ref) < 1e-2
