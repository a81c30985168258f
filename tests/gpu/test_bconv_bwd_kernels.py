"""MFMA dgrad / wgrad kernels of the binary conv vs fp64 references (the ±1
operand is exact; dy is bf16, so errors come only from fp32 accumulation)."""

import os
import sys

import pytest
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tile_support as ts  # noqa: E402

pytestmark = pytest.mark.gpu

# (variant, shape) pairs generated at collection: only those the launcher
# accepts (tests/test_tile_support.py pins the rule to the native queries)
DGRAD_SHAPES = [(64, 64, 1, 12), (64, 128, 2, 12), (128, 128, 1, 7), (256, 512, 2, 8),
                (128, 64, 1, 9), (128, 256, 2, 15), (64, 64, 1, 28), (256, 256, 1, 6),
                (64, 64, 1, 14), (256, 128, 1, 11), (512, 64, 1, 5)]
WGRAD_SHAPES = [(64, 64, 1, 12, 0), (64, 128, 2, 12, 0), (128, 128, 1, 7, 1), (256, 512, 2, 8, 0),
                (128, 64, 1, 9, 1), (64, 192, 1, 5, 1), (64, 64, 1, 28, 1), (128, 256, 1, 14, 0),
                (256, 256, 1, 6, 1), (512, 512, 1, 4, 0), (64, 64, 1, 56, 0),
                (256, 512, 1, 9, 1), (512, 256, 1, 7, 0)]
FWD_SHAPES = [(64, 64, 1, 12, 0, 0), (64, 128, 2, 12, 0, 1), (128, 128, 1, 7, 1, 1),
              (256, 512, 2, 8, 0, 0), (128, 64, 1, 9, 1, 0), (512, 128, 1, 5, 0, 1)]


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("cin,cout,stride,hw,pad_ones", [
    (64, 64, 1, 12, 0), (64, 128, 2, 12, 0), (128, 128, 1, 7, 1), (256, 512, 2, 8, 0),
    (128, 64, 1, 9, 0)])
def test_dgrad_wgrad(cin, cout, stride, hw, pad_ones):
    from zookeeper_amd.nn.layers import pad_same_nhwc, same_padding
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(0)
    L, st = lib(), stream_ptr()
    B = 3
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1.2, 1.2)
    pt, pb = same_padding(hw, 3, stride)
    ho = (hw + pt + pb - 3) // stride + 1
    dy = torch.randn(B, ho, ho, cout, device="cuda").to(torch.bfloat16)
    nwords = x.numel() // 32
    bits = torch.empty(nwords, dtype=torch.int32, device="cuda")
    mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    assert L.zk_sign_pack(x.data_ptr(), bits.data_ptr(), mask.data_ptr(), sx.data_ptr(), None, nwords,
                          1.0, st) == 0
    assert torch.equal(sx.float(), torch.where(x.float() >= 0, 1.0, -1.0))
    wbits = torch.empty(cout * 9 * cin // 32, dtype=torch.int32, device="cuda")
    wpop = torch.empty(cout * 9, dtype=torch.int32, device="cuda")
    wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), wt.data_ptr(), None, None,
                            cout, 9, cin, st) == 0
    dres = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    dx = torch.empty(B, hw, hw, cin, dtype=torch.bfloat16, device="cuda")
    assert L.zk_bconv_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), dres.data_ptr(),
                            dx.data_ptr(), B, hw, hw, cin, ho, ho, cout, 3, 3, stride, pt, pt,
                            -1, st) == 0
    dw = torch.zeros(cout, 3, 3, cin, device="cuda")
    assert L.zk_bconv_wgrad(dy.data_ptr(), bits.data_ptr(), w.data_ptr(), dw.data_ptr(), B, hw,
                            hw, cin, ho, ho, cout, 3, 3, stride, pt, pt, pad_ones, 1.0, 1024,
                            -1, st) == 0
    torch.cuda.synchronize()

    # fp64 reference through autograd of the ±1 convolution
    xs = sign_pm1(x.double()).permute(0, 3, 1, 2).requires_grad_(True)
    ws = sign_pm1(w.double()).permute(0, 3, 1, 2).requires_grad_(True)
    xp = pad_same_nhwc(xs, (3, 3), (stride, stride), 1.0 if pad_ones else 0.0)
    out = F.conv2d(xp, ws, stride=stride)
    out.backward(dy.double().permute(0, 3, 1, 2))
    ste_x = (x.double().abs() <= 1.0)
    ref_dx = xs.grad.permute(0, 2, 3, 1) * ste_x + dres.double()
    ref_dw = ws.grad.permute(0, 2, 3, 1) * (w.double().abs() <= 1.0)
    err_dx = (dx.double() - ref_dx).abs().max().item()
    assert err_dx <= 1e-2 * ref_dx.abs().max().item() + 1e-2, err_dx
    err_dw = (dw.double() - ref_dw).abs().max().item()
    assert err_dw <= 1e-4 * ref_dw.abs().max().item() + 1e-3, err_dw


@pytest.mark.parametrize("variant,cin,cout,stride,hw", ts.pairs(ts.dgrad_ok, ts.DGRAD, DGRAD_SHAPES))
def test_igemm_dgrad_matches_reference(variant, cin, cout, stride, hw):
    """LDS-DMA ring implicit-GEMM dgrad (igemm.hip), every tile variant, vs
    the fp64 ±1 conv gradient (STE mask + residual gradient fused)."""
    from zookeeper_amd.nn.layers import pad_same_nhwc, same_padding
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(1)
    L, st = lib(), stream_ptr()
    B = 3
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1.2, 1.2)
    pt, pb = same_padding(hw, 3, stride)
    ho = (hw + pt + pb - 3) // stride + 1
    dy = torch.randn(B, ho, ho, cout, device="cuda").to(torch.bfloat16)
    nwords = x.numel() // 32
    bits = torch.empty(nwords, dtype=torch.int32, device="cuda")
    mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    assert L.zk_sign_pack(x.data_ptr(), bits.data_ptr(), mask.data_ptr(), sx.data_ptr(), None, nwords,
                          1.0, st) == 0
    assert torch.equal(sx.float(), torch.where(x.float() >= 0, 1.0, -1.0))
    wbits = torch.empty(cout * 9 * cin // 32, dtype=torch.int32, device="cuda")
    wpop = torch.empty(cout * 9, dtype=torch.int32, device="cuda")
    wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), wt.data_ptr(), None, None,
                            cout, 9, cin, st) == 0
    dres = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    dx = torch.full((B, hw, hw, cin), float("nan"), dtype=torch.bfloat16, device="cuda")
    rc = L.zk_igemm_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), dres.data_ptr(),
                          dx.data_ptr(), B, hw, hw, cin, ho, ho, cout, 3, 3, stride, pt, pt,
                          variant, st)
    assert rc == 0, f"variant {variant} rejected a supported shape"
    torch.cuda.synchronize()
    xs = sign_pm1(x.double()).permute(0, 3, 1, 2).requires_grad_(True)
    ws = sign_pm1(w.double()).permute(0, 3, 1, 2)
    xp = pad_same_nhwc(xs, (3, 3), (stride, stride), 0.0)
    F.conv2d(xp, ws, stride=stride).backward(dy.double().permute(0, 3, 1, 2))
    ref = xs.grad.permute(0, 2, 3, 1) * (x.double().abs() <= 1.0) + dres.double()
    err = (dx.double() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("slab", [False, True])
@pytest.mark.parametrize("variant,cin,cout,stride,hw,pad_ones",
                         ts.pairs(ts.wgrad_ok, ts.WGRAD, WGRAD_SHAPES))
def test_igemm_wgrad_matches_reference(variant, cin, cout, stride, hw, pad_ones, slab):
    """LDS-DMA ring implicit-GEMM wgrad (igemm.hip) on the bf16 sign(x)
    image, every tile variant (20+: the conv3 kernel, all taps of a kernel
    row per block over halo-extended rows; 3x3 stride-1 only), split-K by
    fp32 atomics or through the workspace (the in-launch fixed-order tree, or
    slabs + reduce kernel), accumulating into dw, vs the fp64 ±1 conv weight
    gradient."""
    from zookeeper_amd.nn.layers import pad_same_nhwc, same_padding
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(2)
    L, st = lib(), stream_ptr()
    B = 3
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1.2, 1.2)
    pt, pb = same_padding(hw, 3, stride)
    ho = (hw + pt + pb - 3) // stride + 1
    dy = torch.randn(B, ho, ho, cout, device="cuda").to(torch.bfloat16)
    nwords = x.numel() // 32
    bits = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    assert L.zk_sign_pack(x.data_ptr(), bits.data_ptr(), None, sx.data_ptr(), None, nwords, 1.0,
                          st) == 0
    dw = torch.full((cout, 3, 3, cin), 0.25, device="cuda")  # accumulates into dw
    ws = None
    if slab:
        nbytes = L.zk_igemm_wgrad_ws_bytes(B, cin, hw, hw, ho, ho, cout, 3, 3, stride, pt, pt,
                                            256, variant)
        # 0: one split (the in-launch tree then writes dW directly, no slab)
        assert nbytes >= 0, f"variant {variant} rejected a supported shape"
        if nbytes > 0:
            ws = torch.empty(nbytes // 4, device="cuda")
    rc = L.zk_igemm_wgrad(dy.data_ptr(), sx.data_ptr(), w.data_ptr(), dw.data_ptr(), B, hw, hw,
                          cin, ho, ho, cout, 3, 3, stride, pt, pt, pad_ones, 1.0, 256, variant,
                          ws.data_ptr() if ws is not None else None,
                          ws.numel() * 4 if ws is not None else 0, st)
    assert rc == 0, f"variant {variant} rejected a supported shape"
    torch.cuda.synchronize()
    xs = sign_pm1(x.double()).permute(0, 3, 1, 2)
    wsgn = sign_pm1(w.double()).permute(0, 3, 1, 2).requires_grad_(True)
    xp = pad_same_nhwc(xs, (3, 3), (stride, stride), 1.0 if pad_ones else 0.0)
    F.conv2d(xp, wsgn, stride=stride).backward(dy.double().permute(0, 3, 1, 2))
    ref = wsgn.grad.permute(0, 2, 3, 1) * (w.double().abs() <= 1.0) + 0.25
    err = (dw.double() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("variant,cin,cout,stride,hw,pad_ones,relu",
                         ts.pairs(ts.fwd_ok, ts.FWD, FWD_SHAPES))
def test_igemm_fwd_matches_reference(variant, cin, cout, stride, hw, pad_ones, relu):
    """MFMA forward (igemm.hip) on the sign image: exact int16 output and
    exact int64 (sum, sum of squares) per channel, every tile variant."""
    from zookeeper_amd.nn.layers import pad_same_nhwc, same_padding
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(3)
    L, st = lib(), stream_ptr()
    B = 3
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, 3, 3, cin, device="cuda")
    pt, pb = same_padding(hw, 3, stride)
    ho = (hw + pt + pb - 3) // stride + 1
    nwords = x.numel() // 32
    mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    assert L.zk_sign_pack(x.data_ptr(), None, mask.data_ptr(), sx.data_ptr(), None, nwords, 1.0,
                          st) == 0
    wf = torch.empty(9, cout, cin, dtype=torch.bfloat16, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), None, None, None, wf.data_ptr(), None, cout, 9, cin, st) == 0
    y = torch.full((B, ho, ho, cout), -12345, dtype=torch.int16, device="cuda")
    stats = torch.zeros(2, cout, dtype=torch.int64, device="cuda")
    rc = L.zk_igemm_fwd(sx.data_ptr(), wf.data_ptr(), y.data_ptr(), stats.data_ptr(), B, hw, hw,
                        cin, cout, 3, 3, stride, pt, pt, ho, ho, pad_ones, relu, variant, 1, st)
    assert rc == 0, f"variant {variant} rejected a supported shape"
    torch.cuda.synchronize()
    xs = sign_pm1(x.double()).permute(0, 3, 1, 2)
    ws = sign_pm1(w.double()).permute(0, 3, 1, 2)
    xp = pad_same_nhwc(xs, (3, 3), (stride, stride), 1.0 if pad_ones else 0.0)
    ref = torch.nn.functional.conv2d(xp, ws, stride=stride).permute(0, 2, 3, 1)
    if relu:
        ref = ref.clamp_min(0)
    ref = ref.round().long()
    assert torch.equal(y.long(), ref)
    flat = ref.reshape(-1, cout)
    assert torch.equal(stats[0].cpu(), flat.sum(0).cpu())
    assert torch.equal(stats[1].cpu(), (flat * flat).sum(0).cpu())


@pytest.mark.parametrize("cout,taps,cin", [(64, 9, 64), (128, 9, 256), (512, 1, 256)])
def test_weight_pack_tiled_matches_per_word(cout, taps, cin):
    """The LDS-tiled packer (no bit outputs) writes the same wf / wt as the
    per-word kernel (which also produces the XNOR bits)."""
    from zookeeper_amd.ops._native import lib, stream_ptr

    L, st = lib(), stream_ptr()
    w = torch.randn(cout, taps, cin, device="cuda")
    w[0, 0, :8] = 0.0  # sign(0) = +1
    wf = torch.empty(taps, cout, cin, dtype=torch.bfloat16, device="cuda")
    wt = torch.empty(taps, cin, cout, dtype=torch.bfloat16, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), None, None, wt.data_ptr(), wf.data_ptr(), None, cout, taps,
                            cin, st) == 0
    wbits = torch.empty(cout * taps * cin // 32, dtype=torch.int32, device="cuda")
    wpop = torch.empty(cout * taps, dtype=torch.int32, device="cuda")
    wt2 = torch.empty_like(wt)
    wf2 = torch.empty_like(wf)
    assert L.zk_weight_pack(w.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), wt2.data_ptr(),
                            wf2.data_ptr(), None, cout, taps, cin, st) == 0
    torch.cuda.synchronize()
    ref = torch.where(w >= 0, 1.0, -1.0)
    assert torch.equal(wf.float(), ref.permute(1, 0, 2))
    assert torch.equal(wt.float(), ref.permute(1, 2, 0))
    assert torch.equal(wf, wf2) and torch.equal(wt, wt2)
