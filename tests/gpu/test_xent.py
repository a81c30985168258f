"""Fused softmax cross-entropy kernel vs torch (fp32)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,eps", [(256, 1000, 0.0), (37, 10, 0.1), (8, 4097, 0.0)])
def test_softmax_xent_matches_torch(B, C, eps):
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd.ops import softmax_xent

    torch.manual_seed(0)
    x = (torch.randn(B, C, device="cuda") * 3).requires_grad_(True)
    y = torch.randint(0, C, (B,), device="cuda")
    loss, hits = softmax_xent(x, y, eps)
    (loss * 2.0).backward()
    xr = x.detach().clone().requires_grad_(True)
    ref = F.cross_entropy(xr, y, label_smoothing=eps)
    (ref * 2.0).backward()
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)
    assert int(hits) == int((xr.argmax(1) == y).sum())
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-6, rtol=1e-4)
