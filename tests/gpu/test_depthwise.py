"""Depthwise 3×3 HIP kernels (fwd / dgrad / wgrad) vs fp32 PyTorch."""

import pytest
import torch
import torch.nn.functional as F

from zookeeper_amd.nn.layers import pad_same_nhwc

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("C,H,W,s,padding", [(16, 17, 12, 2, "same"), (64, 14, 14, 2, "same"),
                                              (128, 9, 8, 1, "same"), (32, 10, 11, 1, "valid"),
                                              (256, 7, 7, 2, "same")])
def test_depthwise_matches_fp32(C, H, W, s, padding):
    from zookeeper_amd.ops.depthwise import depthwise_conv3x3

    torch.manual_seed(0)
    x = _cl(torch.randn(3, C, H, W, device="cuda")).to(torch.bfloat16)
    w = _cl(torch.randn(C, 1, 3, 3, device="cuda") * 0.3).requires_grad_(True)
    xh = x.clone().requires_grad_(True)
    y = depthwise_conv3x3(xh, w, s, padding)
    g = _cl(torch.randn_like(y.float())).to(torch.bfloat16)
    y.backward(g)
    xr = x.float().clone().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    xp = pad_same_nhwc(xr, (3, 3), (s, s)) if padding == "same" else xr
    yr = F.conv2d(xp, wr, None, s, 0, 1, C)
    yr.backward(g.float())
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(w.grad, wr.grad, atol=5e-2, rtol=1e-2)


def test_quicknet_uses_native_depthwise_and_trains():
    from zookeeper_amd.models.quicknet import QuickNetModule

    torch.manual_seed(0)
    m = QuickNetModule((64, 64, 3), 10, (1, 1, 1, 1), (64, 128, 256, 512), backend="hip")
    m = m.cuda().to(memory_format=torch.channels_last)
    x = _cl(torch.randn(4, 3, 64, 64, device="cuda")).to(torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=False):
        out = m(x)
    assert out.shape == (4, 10) and torch.isfinite(out).all()
    out.float().sum().backward()
    dw = m.stem[2].weight.grad
    assert dw is not None and torch.isfinite(dw).all() and dw.abs().sum() > 0
