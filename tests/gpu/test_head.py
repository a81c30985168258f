"""Native classifier head (``csrc/kernels/head.hip``) against a plain PyTorch
fp32 reference: (ReLU) + global average pool + fp32 dense layer, forward and
all three gradients, and the bf16 global-average-pool alone."""

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


def _ref(x, w, b, relu):
    xf = x.detach().float().requires_grad_(True)
    wf = w.detach().clone().requires_grad_(True)
    bf = b.detach().clone().requires_grad_(True)
    a = F.relu(xf) if relu else xf
    out = F.linear(a.mean(dim=(2, 3)), wf, bf)
    return out, xf, wf, bf


@pytest.mark.parametrize("B,C,HW,N,relu", [
    (64, 512, 7, 1000, True),      # E18 / QuickNet ImageNet head
    (32, 2048, 7, 1000, False),    # ResNet-50 head
    (10, 256, 4, 10, True),        # CIFAR-sized, ragged tiles
    (3, 24, 3, 70, False),         # ragged everything
])
def test_head_matches_fp32(B, C, HW, N, relu):
    from zookeeper_amd.ops.head import classifier_head, head_supported

    torch.manual_seed(0)
    x = torch.randn(B, C, HW, HW, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(N, C, device="cuda") / C ** 0.5).requires_grad_(True)
    b = torch.randn(N, device="cuda").requires_grad_(True)
    assert head_supported(x, w)
    out = classifier_head(x, w, b, relu)
    ref, xf, wf, bf = _ref(x, w, b, relu)
    assert out.dtype == torch.float32 and out.shape == (B, N)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)
    g = torch.randn(B, N, device="cuda")
    out.backward(g)
    ref.backward(g)
    torch.testing.assert_close(w.grad, wf.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(b.grad, bf.grad, rtol=1e-4, atol=1e-4)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    # dx is bf16: one rounding of the fp32 value
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=1e-2, atol=1e-5)


def test_head_accumulates_into_direct_grad():
    """A parameter with a flat-buffer gradient gets dW/db added in place and
    the autograd result for it is None (FlatParams contract)."""
    from zookeeper_amd.ops.head import classifier_head

    torch.manual_seed(1)
    B, C, N = 16, 64, 40
    x = torch.randn(B, C, 5, 5, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w = torch.nn.Parameter(torch.randn(N, C, device="cuda") * 0.1)
    b = torch.nn.Parameter(torch.randn(N, device="cuda"))
    prior_w, prior_b = torch.randn(N, C, device="cuda"), torch.randn(N, device="cuda")
    w.grad, b.grad = prior_w.clone(), prior_b.clone()
    ready = []
    for p, tag in ((w, "w"), (b, "b")):
        p._zk_direct_grad = True
        p._zk_grad_ready = (lambda t=tag: ready.append(t))
    out = classifier_head(x, w, b, True)
    g = torch.randn(B, N, device="cuda")
    out.backward(g)
    ref, _, wf, bf = _ref(x, w, b, True)
    ref.backward(g)
    torch.testing.assert_close(w.grad, prior_w + wf.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(b.grad, prior_b + bf.grad, rtol=1e-4, atol=1e-4)
    assert sorted(ready) == ["b", "w"]


def test_global_avg_pool_matches_fp32():
    from zookeeper_amd.nn.layers import GlobalAvgPool

    torch.manual_seed(2)
    x = torch.randn(8, 136, 6, 6, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = GlobalAvgPool()(x)
    xf = x.detach().float().requires_grad_(True)
    yr = xf.mean(dim=(2, 3))
    assert y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), yr, rtol=8e-3, atol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    torch.testing.assert_close(x.grad.float(), xf.grad, rtol=1e-2, atol=1e-5)


def test_models_use_native_head():
    """The E18 forward ends in the native head (no F.linear on the GPU)."""
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.ops import head as head_mod

    calls = []
    real = head_mod._HeadFn.apply

    def spy(*a):
        calls.append(a[0].shape)
        return real(*a)

    head_mod._HeadFn.apply = spy
    try:
        m = BinaryResNetE((32, 32, 3), 10, 18, backend="hip").cuda()
        for p in m.parameters():
            if p.dim() == 4:
                p.data = p.data.contiguous(memory_format=torch.channels_last)
        x = torch.randn(4, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        out = m(x)
    finally:
        head_mod._HeadFn.apply = real
    assert out.dtype == torch.float32 and out.shape == (4, 10)
    assert calls, "native head not used"
