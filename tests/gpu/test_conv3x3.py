"""Float 3×3 stride-1 ``same`` convolution on the MFMA implicit-GEMM
kernels (ops/conv3x3.py: forward as a flipped-tap dgrad, dgrad, split-K
wgrad) against the fp32 PyTorch convolution: output, input gradient and
weight gradient."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("cin,cout,hw", [(64, 64, 14), (64, 128, 9), (128, 128, 7),
                                         (256, 256, 7), (512, 512, 5), (256, 64, 11)])
def test_conv3x3_matches_fp32(cin, cout, hw):
    from zookeeper_amd.ops import conv3x3

    torch.manual_seed(0)
    x = torch.randn(3, cin, hw, hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5))
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    assert conv3x3.supported(x, w, (1, 1), "same", 1)
    xx = x.clone().requires_grad_(True)
    y = conv3x3.conv3x3(xx, w)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    xr = x.float().clone().requires_grad_(True)
    wr = w.detach().float().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, padding=1)
    yr.backward(g.float())
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    assert _rel(xx.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2


def test_quantconv_dispatches_float_3x3_to_mfma():
    from zookeeper_amd.nn.layers import QuantConv2d

    torch.manual_seed(1)
    conv = QuantConv2d(64, 64, 3, 1, "same").cuda()
    x = torch.randn(2, 64, 8, 8, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = conv(x)
    assert y.grad_fn is not None and "Conv3x3" in type(y.grad_fn).__name__
    yr = F.conv2d(x.float(), conv.weight.float(), padding=1)
    assert _rel(y, yr) < 1e-2
