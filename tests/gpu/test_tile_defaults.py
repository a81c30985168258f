"""Default (variant -1) tile choices of the binary-conv kernels at the
per-GPU batches 512 and 1024 (the bench default), where the batch-aware rules in igemm.hip pick 256x256
tiles / larger split-K grids: data gradient, weight gradient and MX-FP4
forward must agree with an explicitly chosen variant that the per-variant
fp64 tests (test_bconv_bwd_kernels.py, test_fp4_forward.py) validate."""

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [  # H, W, Cin, Cout, stride (BinaryResNet-E18 / QuickNet 3x3 layers)
    (7, 7, 512, 512, 1),
    (14, 14, 256, 256, 1),
    (14, 14, 256, 512, 2),
    (28, 28, 128, 128, 1),
    (28, 28, 128, 256, 2),
]


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("B", [512, 1024])
@pytest.mark.parametrize("H,W,cin,cout,s", SHAPES)
def test_defaults_match_reference_variant(H, W, cin, cout, s, B):
    from zookeeper_amd.nn.layers import same_padding
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(3)
    L, st = lib(), stream_ptr()
    pt, pb = same_padding(H, 3, s)
    Ho = (H + pt + pb - 3) // s + 1
    x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1.2, 1.2)
    dy = torch.randn(B, Ho, Ho, cout, device="cuda").to(torch.bfloat16)
    nwords = x.numel() // 32
    mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    sx4 = torch.empty(B, H, W, cin // 2, dtype=torch.uint8, device="cuda")
    bits = torch.empty(nwords, dtype=torch.int32, device="cuda")
    assert L.zk_sign_pack(x.data_ptr(), bits.data_ptr(), mask.data_ptr(), sx.data_ptr(), None,
                          nwords, 1.0, st) == 0
    assert L.zk_sign_pack(x.data_ptr(), None, None, None, sx4.data_ptr(), nwords, 1.0, st) == 0
    wbits = torch.empty(cout * 9 * cin // 32, dtype=torch.int32, device="cuda")
    wpop = torch.empty(cout * 9, dtype=torch.int32, device="cuda")
    wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
    wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), wt.data_ptr(), None,
                            None, cout, 9, cin, st) == 0
    assert L.zk_weight_pack(w.data_ptr(), None, None, None, None, wf4.data_ptr(), cout, 9, cin,
                            st) == 0

    # data gradient: default vs the 128x128 tile (variant 0)
    dx = {}
    for v in (-1, 0):
        dx[v] = torch.full((B, H, W, cin), float("nan"), dtype=torch.bfloat16, device="cuda")
        assert L.zk_igemm_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), None,
                                dx[v].data_ptr(), B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, v,
                                st) == 0
    torch.cuda.synchronize()
    ref = dx[0].float()
    err = (dx[-1].float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err

    # weight gradient (slab split-K): default vs 128x128 tiles at 1024 blocks
    dw = {}
    for v, tb in ((-1, 0), (0, 1024)):
        nbytes = L.zk_igemm_wgrad_ws_bytes(B, cin, H, W, Ho, Ho, cout, 3, 3, s, pt, pt, tb, v)
        assert nbytes > 0
        ws = torch.empty(nbytes // 4, device="cuda")
        dw[v] = torch.zeros(cout, 3, 3, cin, device="cuda")
        assert L.zk_igemm_wgrad(dy.data_ptr(), sx.data_ptr(), w.data_ptr(), dw[v].data_ptr(), B, H,
                                W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, 0, 1.0, tb, v,
                                ws.data_ptr(), nbytes, st) == 0
    torch.cuda.synchronize()
    err = (dw[-1] - dw[0]).abs().max().item()
    assert err <= 1e-5 * dw[0].abs().max().item(), err

    # MX-FP4 forward: exact integer outputs and statistics, default vs variant 0
    y, stats = {}, {}
    for v in (-1, 0):
        y[v] = torch.empty(B, Ho, Ho, cout, dtype=torch.int16, device="cuda")
        stats[v] = torch.zeros(32, 2, cout, dtype=torch.int64, device="cuda")
        assert L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y[v].data_ptr(),
                                  stats[v].data_ptr(), B, H, W, cin, cout, 3, 3, s, pt, pt, Ho,
                                  Ho, 0, 0, v, 32, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(y[-1], y[0])
    assert torch.equal(stats[-1].sum(0), stats[0].sum(0))
