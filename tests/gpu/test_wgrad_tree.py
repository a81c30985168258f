"""In-launch fixed-order split-K combine of the MFMA weight gradients
(``splitk_tree.h``: igemm.hip's igemm_wgrad_kernel, deep_gemm.hip's
wgrad_deep_kernel).  Shapes with one- and two-level trees: the result matches
the float64 ±1 weight gradient, repeated launches are bit-identical (the
arrival counters reset themselves: a stale counter would skip or double a
group), and the tree agrees with the slab + reduce-kernel path it replaces
(option 10 off) to fp32 summation-order noise."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

OPT_WGRAD_TREE = 10


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


# variant -1 picks wgrad_deep (60) for 256 -> 256 and an igemm_wgrad tile for
# the strided 128 -> 128 layer
@pytest.mark.parametrize("B,hw,cin,cout,stride,variant,target", [
    (64, 14, 256, 256, 1, 60, 512),   # deep, ~49 splits: two levels
    (16, 14, 256, 256, 1, 60, 512),   # deep, fewer splits: one level
    (32, 28, 128, 128, 2, -1, 1024),  # igemm_wgrad (strided), many splits
    (8, 14, 128, 256, 2, -1, 256),
])
def test_wgrad_tree(B, hw, cin, cout, stride, variant, target):
    from zookeeper_amd.nn.layers import pad_same_nhwc, same_padding
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(4)
    L, st = lib(), stream_ptr()
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1.2, 1.2)
    pt, pb = same_padding(hw, 3, stride)
    ho = (hw + pt + pb - 3) // stride + 1
    dy = torch.randn(B, ho, ho, cout, device="cuda").to(torch.bfloat16)
    nwords = x.numel() // 32
    sx = torch.empty_like(x)
    assert L.zk_sign_pack(x.data_ptr(), None, None, sx.data_ptr(), None, nwords, 1.0, st) == 0

    def run():
        nb = L.zk_igemm_wgrad_ws_bytes(B, cin, hw, hw, ho, ho, cout, 3, 3, stride, pt, pt, target,
                                       variant)
        ws = torch.empty(max(nb, 4) // 4, device="cuda")
        dw = torch.full((cout, 3, 3, cin), 0.25, device="cuda")
        assert L.zk_igemm_wgrad(dy.data_ptr(), sx.data_ptr(), w.data_ptr(), dw.data_ptr(), B, hw,
                                hw, cin, ho, ho, cout, 3, 3, stride, pt, pt, 0, 1.0, target,
                                variant, ws.data_ptr(), ws.numel() * 4, st) == 0
        torch.cuda.synchronize()
        return dw

    prev = L.zk_get_option(OPT_WGRAD_TREE)
    try:
        assert L.zk_set_option(OPT_WGRAD_TREE, 1) == 0
        runs = [run() for _ in range(3)]
        assert L.zk_set_option(OPT_WGRAD_TREE, 0) == 0
        old = run()
    finally:
        L.zk_set_option(OPT_WGRAD_TREE, prev)
    for r in runs[1:]:
        assert torch.equal(r, runs[0])
    xs = sign_pm1(x.double()).permute(0, 3, 1, 2)
    wsgn = sign_pm1(w.double()).permute(0, 3, 1, 2).requires_grad_(True)
    xp = pad_same_nhwc(xs, (3, 3), (stride, stride), 0.0)
    F.conv2d(xp, wsgn, stride=stride).backward(dy.double().permute(0, 3, 1, 2))
    ref = wsgn.grad.permute(0, 2, 3, 1) * (w.double().abs() <= 1.0) + 0.25
    scale = ref.abs().max().item()
    err = (runs[0].double() - ref).abs().max().item()
    assert err <= 1e-4 * scale + 1e-3, err
    assert (runs[0] - old).abs().max().item() <= 1e-5 * scale + 1e-4
