"""bf16 NHWC BatchNorm(+ReLU) and pooling HIP kernels vs fp32 PyTorch."""

import copy

import pytest
import torch
import torch.nn.functional as F

from zookeeper_amd.nn.layers import AvgPool2d, BatchNorm, MaxPool2d

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("C,relu,affine", [(64, False, True), (128, True, True),
                                           (512, False, False), (2048, True, True)])
def test_batchnorm_train(C, relu, affine):
    torch.manual_seed(0)
    bn = BatchNorm(C, momentum=0.9, eps=1e-5, scale=affine, center=affine,
                   activation="relu" if relu else None).cuda()
    if affine:
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
    x = _cl(torch.randn(4, C, 6, 5, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    g = _cl(torch.randn(4, C, 6, 5, device="cuda")).to(torch.bfloat16)
    ref = copy.deepcopy(bn).float()
    xh = x.clone().requires_grad_(True)
    yh = bn(xh)
    yh.backward(g)
    xr = x.float().clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g.float())
    torch.testing.assert_close(yh.float(), yr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-4, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    if affine:
        torch.testing.assert_close(bn.weight.grad, ref.weight.grad, atol=5e-2, rtol=2e-2)
        torch.testing.assert_close(bn.bias.grad, ref.bias.grad, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("C,relu", [(256, True), (64, False), (2048, True)])
def test_batchnorm_residual_relu(C, relu):
    """relu(bn(x) + r) (a bottleneck tail, norm_pool.batch_norm): output and
    the gradients of x, r and the affine parameters against the fp32 oracle.
    The backward masks with the 1-bit ReLU mask the forward stored (not the
    bf16 output)."""
    from zookeeper_amd.ops import norm_pool

    torch.manual_seed(3)
    bn = BatchNorm(C, momentum=0.9, eps=1e-5).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = _cl(torch.randn(4, C, 6, 5, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    r = _cl(torch.randn(4, C, 6, 5, device="cuda")).to(torch.bfloat16)
    g = _cl(torch.randn(4, C, 6, 5, device="cuda")).to(torch.bfloat16)
    ref = copy.deepcopy(bn).float()
    xh, rh = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    yh = norm_pool.batch_norm(xh, bn, relu=relu, residual=rh)
    yh.backward(g)
    xr, rr = x.float().clone().requires_grad_(True), r.float().clone().requires_grad_(True)
    yr = ref(xr) + rr
    yr = torch.relu(yr) if relu else yr
    yr.backward(g.float())
    torch.testing.assert_close(yh.float(), yr, atol=3e-2, rtol=2e-2)
    # the mask decides exactly where the bf16 output is positive: compare the
    # residual gradient where the oracle's output is clearly nonzero
    live = (yr.abs() > 0.05) | (not relu)
    torch.testing.assert_close(rh.grad.float()[live], rr.grad[live], atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=5e-2, rtol=5e-2)
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, atol=5e-2, rtol=2e-2)


def test_batchnorm_eval_uses_running_stats():
    bn = BatchNorm(32, momentum=0.9, eps=1e-5).cuda()
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    bn.eval()
    x = _cl(torch.randn(2, 32, 4, 4, device="cuda")).to(torch.bfloat16)
    y = bn(x).float()
    ref = F.batch_norm(x.float(), bn.running_mean, bn.running_var, bn.weight, bn.bias, False, 0.0, 1e-5)
    torch.testing.assert_close(y, ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("k,s,padding,hw", [(3, 2, "same", 112), (3, 2, "same", 9),
                                            (2, 2, "valid", 8), (2, 1, "valid", 7)])
def test_maxpool(k, s, padding, hw):
    torch.manual_seed(1)
    x = _cl(torch.randn(2, 64, hw, hw, device="cuda")).to(torch.bfloat16)
    mp = MaxPool2d(k, s, padding)
    xh = x.clone().requires_grad_(True)
    yh = mp(xh)
    xr = x.float().clone().requires_grad_(True)
    yr = MaxPool2d(k, s, padding)(xr)
    torch.testing.assert_close(yh.float(), yr, atol=0, rtol=0)
    g = torch.randn_like(yr)
    yh.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("k,s,padding", [(2, 1, "valid"), (3, 2, "same")])
def test_maxpool_relu(k, s, padding):
    """relu(max_pool(x)) in one pass (QuickNet transitions): exact forward,
    and no gradient through outputs the ReLU clipped (window max <= 0)."""
    from zookeeper_amd.ops.norm_pool import max_pool

    torch.manual_seed(3)
    x = _cl(torch.randn(2, 64, 9, 9, device="cuda") - 0.7).to(torch.bfloat16)
    x[0, :, :4, :4] = 0  # windows whose max is exactly 0: clipped, no gradient
    xh = x.clone().requires_grad_(True)
    yh = max_pool(xh, k, s, padding, relu=True)
    xr = x.float().clone().requires_grad_(True)
    yr = F.relu(MaxPool2d(k, s, padding)(xr))
    torch.testing.assert_close(yh.float(), yr, atol=0, rtol=0)
    g = torch.randn_like(yr).to(torch.bfloat16)
    yh.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=2e-2, rtol=1e-2)
    assert (xh.grad[0, :, :3, :3] == 0).all()


def test_avgpool2():
    torch.manual_seed(2)
    x = _cl(torch.randn(2, 128, 14, 14, device="cuda")).to(torch.bfloat16)
    xh = x.clone().requires_grad_(True)
    yh = AvgPool2d(2, 2)(xh)
    xr = x.float().clone().requires_grad_(True)
    yr = F.avg_pool2d(xr, 2, 2)
    torch.testing.assert_close(yh.float(), yr, atol=2e-2, rtol=1e-2)
    g = torch.randn_like(yr).to(torch.bfloat16)
    yh.backward(g)
    yr.backward(g.float())
    torch.testing.assert_close(xh.grad.float(), xr.grad, atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("tiles,C", [(1, 64), (300, 200), (1568, 64), (5000, 1024), (513, 8)])
def test_bn_bwd_tiles_reduce_fixed_order(tiles, C):
    """zk_bn_bwd_tiles_reduce: copy b of value c = rows b, b + 512, ... of
    column c summed in that order (fp32, bit-exact against the same order in
    torch), written channel-major [2C][512]; every row re-zeroed."""
    from zookeeper_amd.ops._native import check, lib, stream_ptr

    L = lib()
    nparts = L.zk_bn_bwd_parts_max()
    rows = torch.randn(tiles, 2 * C, device="cuda")
    ref = torch.zeros(nparts, 2 * C, device="cuda")
    for k in range(0, tiles, nparts):
        blk = rows[k:k + nparts]
        ref[:blk.shape[0]] = ref[:blk.shape[0]] + blk
    out = torch.full((2 * C, nparts), float("nan"), device="cuda")
    check(L.zk_bn_bwd_tiles_reduce(rows.data_ptr(), tiles, C, out.data_ptr(), stream_ptr()),
          "zk_bn_bwd_tiles_reduce")
    torch.cuda.synchronize()
    assert torch.equal(out, ref.t().contiguous())
    assert torch.count_nonzero(rows).item() == 0
