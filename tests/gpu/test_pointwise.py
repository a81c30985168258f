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


@pytest.mark.parametrize("B,cin,cout,hw,relu", [(4, 64, 128, 28, True), (2, 256, 512, 7, False),
                                                (3, 128, 64, 9, True), (2, 64, 256, 56, False)])
def test_conv1x1_epilogue_bn_statistics(B, cin, cout, hw, relu):
    """conv1x1(stats_for=bn): the BatchNorm's batch statistics summed in the
    GEMM epilogue over the stored bf16 outputs.  Running statistics and the
    normalised output match an fp64 oracle over the same bf16 y (the separate
    statistics pass computes exactly these sums), and the striped buffer is
    zero again afterwards (persistent accumulator)."""
    from zookeeper_amd.nn.layers import BatchNorm
    from zookeeper_amd.ops import norm_pool
    from zookeeper_amd.ops.pointwise import conv1x1

    torch.manual_seed(2)
    x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, 1, 1, device="cuda") * 0.1 + 0.02
    bn = BatchNorm(cout, 0.9, 1e-5).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    for step in range(2):  # the second step reuses the re-zeroed buffer
        y = conv1x1(x, w, stats_for=bn)
        assert "_zk_pending_fstats" in bn.__dict__
        rm0, rv0 = bn.running_mean.clone(), bn.running_var.clone()
        out = norm_pool.batch_norm(y, bn, relu)
        assert "_zk_pending_fstats" not in bn.__dict__
        yd = y.detach().double().permute(0, 2, 3, 1).reshape(-1, cout)
        n = yd.shape[0]
        mean, var = yd.mean(0), yd.var(0, unbiased=False)
        torch.testing.assert_close(bn.running_mean.double(), 0.9 * rm0.double() + 0.1 * mean,
                                   rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(bn.running_var.double(),
                                   0.9 * rv0.double() + 0.1 * var * n / (n - 1),
                                   rtol=1e-4, atol=1e-5)
        ref = (yd - mean) / torch.sqrt(var + 1e-5) * bn.weight.double() + bn.bias.double()
        if relu:
            ref = ref.clamp_min(0)
        got = out.detach().double().permute(0, 2, 3, 1).reshape(-1, cout)
        assert (got - ref).abs().max().item() < 3e-2 * max(1.0, ref.abs().max().item())
        assert bool((bn.__dict__["_zk_scratch"]["fstats"] == 0).all())


def test_conv1x1_epilogue_statistics_skipped_in_eval_and_deterministic():
    """No epilogue statistics where the BN would not consume them (eval mode)
    or where the fp64 atomics would break bit-reproducibility."""
    from zookeeper_amd.nn.layers import BatchNorm
    from zookeeper_amd.ops import options
    from zookeeper_amd.ops.pointwise import conv1x1

    x = torch.randn(2, 64, 8, 8, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 64, 1, 1, device="cuda")
    bn = BatchNorm(64, 0.9, 1e-5).cuda().eval()
    conv1x1(x, w, stats_for=bn)
    assert "_zk_pending_fstats" not in bn.__dict__
    bn.train()
    old = options.OPTS.deterministic
    try:
        options.set_options(deterministic=True)
        conv1x1(x, w, stats_for=bn)
        assert "_zk_pending_fstats" not in bn.__dict__
    finally:
        options.set_options(deterministic=old)


@pytest.mark.parametrize("cout,fused", [(256, True), (128, False)])
def test_conv3x3_epilogue_bn_statistics(cout, fused):
    """The 3x3 float forward with stats_for: 256 output channels run the
    LDS-epilogue tile (statistics fused), 128 a conv3 tile (statistics pass
    kept); the BN result is the same fp64-oracle BN either way."""
    from zookeeper_amd.nn.layers import BatchNorm
    from zookeeper_amd.ops import norm_pool
    from zookeeper_amd.ops.conv3x3 import conv3x3

    torch.manual_seed(3)
    x = torch.randn(2, 64, 14, 14, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, 64, 3, 3, device="cuda") * 0.05 + 0.01
    bn = BatchNorm(cout, 0.9, 1e-5).cuda()
    y = conv3x3(x, w, stats_for=bn)
    yr = F.conv2d(x.float(), w.to(torch.bfloat16).float(), padding=1)
    assert _rel(y, yr) < 1e-2
    assert ("_zk_pending_fstats" in bn.__dict__) == fused
    out = norm_pool.batch_norm(y, bn, True)
    yd = y.detach().double().permute(0, 2, 3, 1).reshape(-1, cout)
    mean, var = yd.mean(0), yd.var(0, unbiased=False)
    torch.testing.assert_close(bn.running_mean.double(), 0.1 * mean, rtol=1e-5, atol=1e-5)
    ref = ((yd - mean) / torch.sqrt(var + 1e-5)).clamp_min(0)
    got = out.detach().double().permute(0, 2, 3, 1).reshape(-1, cout)
    assert (got - ref).abs().max().item() < 3e-2 * max(1.0, ref.abs().max().item())
