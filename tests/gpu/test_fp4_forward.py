"""Binary forward on MX-FP4 MFMA (``zk_igemm_fwd_fp4``, igemm.hip): e2m1 ±1
operands, exact integer outputs and BN statistics against the float64 ±1
convolution for every tile variant on E18 / QuickNet layer shapes (stride
1 and 2, zero and +1 padding, fused ReLU, tail tiles); the e2m1 sign images
of every producer (sign pack, weight pack, both BN epilogues) against their
bit-level definition; and the fused binary block giving the same forward
output on the FP4 and the bf16 MFMA paths."""

import copy

import pytest
import torch

from zookeeper_amd.ops.options import OPTS

pytestmark = pytest.mark.gpu

VARIANTS = [-1] + list(range(10)) + list(range(20, 29)) + [40]


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def fp4_ref(t: torch.Tensor) -> torch.Tensor:
    """sign(t) as e2m1 nibbles (+1 = 0x2, -1 = 0xA), two channels per byte
    along the last dim, the even channel in the low nibble."""
    nib = torch.where(t >= 0, 2, 10).to(torch.uint8)
    return nib[..., 0::2] | (nib[..., 1::2] << 4)


SHAPES = [
    # cin, cout, stride, hw, pad_ones, relu
    (64, 64, 1, 9, 0, 0),
    (64, 64, 1, 11, 1, 1),
    (64, 64, 1, 28, 0, 0),  # 10+ M tiles
    (64, 128, 2, 12, 0, 0),
    (128, 128, 1, 7, 0, 0),
    (128, 128, 1, 6, 1, 1),
    (128, 256, 2, 8, 0, 0),
    (256, 256, 1, 5, 0, 0),
    (256, 512, 2, 6, 0, 0),
    (512, 512, 1, 4, 0, 0),
    (128, 64, 1, 6, 0, 0),
]


@pytest.mark.parametrize("cin,cout,stride,hw,pad_ones,relu", SHAPES)
def test_igemm_fwd_fp4_exact(cin, cout, stride, hw, pad_ones, relu):
    from zookeeper_amd.nn.layers import pad_same_nhwc, same_padding
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(7)
    L, st = lib(), stream_ptr()
    B = 3
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, 3, 3, cin, device="cuda")
    nwords = x.numel() // 32
    sx4 = torch.empty(B, hw, hw, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_sign_pack(x.data_ptr(), None, None, None, sx4.data_ptr(), nwords, 1.0, st) == 0
    wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), None, None, None, None, wf4.data_ptr(), cout, 9, cin,
                            st) == 0
    torch.cuda.synchronize()
    assert torch.equal(sx4, fp4_ref(x.float()))
    assert torch.equal(wf4, fp4_ref(w.reshape(cout, 9, cin).permute(1, 0, 2)))

    pt, pb = same_padding(hw, 3, stride)
    ho = (hw + pt + pb - 3) // stride + 1
    xs = sign_pm1(x.double()).permute(0, 3, 1, 2)
    ws = sign_pm1(w.double()).permute(0, 3, 1, 2)
    xp = pad_same_nhwc(xs, (3, 3), (stride, stride), 1.0 if pad_ones else 0.0)
    ref = torch.nn.functional.conv2d(xp, ws, stride=stride).permute(0, 2, 3, 1)
    if relu:
        ref = ref.clamp_min(0)
    ref = ref.round().long()
    flat = ref.reshape(-1, cout)
    ran = 0
    for v in VARIANTS:
        y = torch.full((B, ho, ho, cout), -12345, dtype=torch.int16, device="cuda")
        stats = torch.zeros(2, cout, dtype=torch.int64, device="cuda")
        rc = L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(),
                                B, hw, hw, cin, cout, 3, 3, stride, pt, pt, ho, ho, pad_ones,
                                relu, v, 1, st)
        if rc != 0:
            assert v != -1, "the default tile must cover every E18 / QuickNet shape"
            continue
        torch.cuda.synchronize()
        ran += 1
        assert torch.equal(y.long(), ref), (v, (y.long() - ref).abs().max().item())
        assert torch.equal(stats[0].cpu(), flat.sum(0).cpu()), v
        assert torch.equal(stats[1].cpu(), (flat * flat).sum(0).cpu()), v
    assert ran >= 2
    # striped statistics: block b adds into copy b % 32; the copies sum exactly
    stats = torch.zeros(32, 2, cout, dtype=torch.int64, device="cuda")
    assert L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(), B,
                              hw, hw, cin, cout, 3, 3, stride, pt, pt, ho, ho, pad_ones, relu, -1,
                              32, st) == 0
    torch.cuda.synchronize()
    tot = stats.sum(0).cpu()
    assert torch.equal(tot[0], flat.sum(0).cpu()) and torch.equal(tot[1], (flat * flat).sum(0).cpu())


@pytest.mark.parametrize("cin,B,hw,pad_ones,relu", [
    (64, 256, 56, 0, 0), (64, 37, 28, 1, 1), (64, 61, 15, 0, 1), (64, 2800, 56, 1, 0),
    (128, 256, 28, 0, 0), (128, 37, 28, 1, 1), (128, 61, 15, 0, 1), (128, 900, 28, 1, 0),
])
def test_bfwd_persistent_matches_conv3(cin, B, hw, pad_ones, relu):
    """The persistent kernel (variant 40, bfwd.hip; Cin 64: 256-pixel tiles,
    Cin 128: 512-pixel tiles and one 64-channel output slice per block) walks
    many tiles per block at these sizes (the float64 test above covers one or
    two): its int16 outputs and striped int64 statistics (flushed mid-run at
    batch 2800 / 900) equal the conv3 tile's (variant 20, itself exact
    against float64) bit for bit, tail tiles included."""
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(11)
    L, st = lib(), stream_ptr()
    cout = cin
    x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, 3, 3, cin, device="cuda")
    sx4 = torch.empty(B, hw, hw, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_sign_pack(x.data_ptr(), None, None, None, sx4.data_ptr(), x.numel() // 32, 1.0,
                          st) == 0
    wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), None, None, None, None, wf4.data_ptr(), cout, 9, cin,
                            st) == 0
    out = {}
    for v, stripes in ((20, 1), (40, 1), (40, 32)):
        y = torch.full((B, hw, hw, cout), -12345, dtype=torch.int16, device="cuda")
        stats = torch.zeros(stripes, 2, cout, dtype=torch.int64, device="cuda")
        assert L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(),
                                  B, hw, hw, cin, cout, 3, 3, 1, 1, 1, hw, hw, pad_ones, relu, v,
                                  stripes, st) == 0
        torch.cuda.synchronize()
        out[(v, stripes)] = (y, stats.sum(0))
    y0, s0 = out[(20, 1)]
    for key in ((40, 1), (40, 32)):
        y1, s1 = out[key]
        assert torch.equal(y1, y0), (key, (y1.long() - y0.long()).abs().max().item())
        assert torch.equal(s1, s0), key


def test_bn_epilogues_write_fp4_sign_images():
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(3)
    L, st = lib(), stream_ptr()
    P, C = 1000, 128
    y = torch.randint(-500, 500, (P, C), dtype=torch.int16, device="cuda")
    scale = torch.rand(C, device="cuda") * 0.01
    shift = torch.randn(C, device="cuda") * 0.5
    res = torch.randn(P, C, device="cuda").to(torch.bfloat16)
    out = torch.empty(P, C, dtype=torch.bfloat16, device="cuda")
    sx = torch.empty_like(out)
    mask = torch.empty(P * C // 32, dtype=torch.int32, device="cuda")
    sx4 = torch.empty(P, C // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_bn_apply_sign(y.data_ptr(), scale.data_ptr(), shift.data_ptr(), res.data_ptr(),
                              out.data_ptr(), sx.data_ptr(), mask.data_ptr(), sx4.data_ptr(),
                              1.0, P, C, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(sx4, fp4_ref(out.float()))
    assert torch.equal(sx.float(), torch.where(out.float() >= 0, 1.0, -1.0))

    coef = torch.cat([scale * 50, shift, torch.zeros(2 * C, device="cuda")])  # [4][C]
    xb = torch.randn(P, C, device="cuda").to(torch.bfloat16)
    out2 = torch.empty_like(out)
    sx2, sx42 = torch.empty_like(sx), torch.empty_like(sx4)
    mask2 = torch.empty_like(mask)
    assert L.zk_bn_apply_bf16_sign(xb.data_ptr(), coef.data_ptr(), out2.data_ptr(),
                                   sx2.data_ptr(), mask2.data_ptr(), sx42.data_ptr(), 1.0, P, C, 0,
                                   st) == 0
    torch.cuda.synchronize()
    assert torch.equal(sx42, fp4_ref(out2.float()))


@pytest.mark.parametrize("cin,cout,stride", [(64, 64, 1), (64, 128, 2), (256, 256, 1)])
def test_binary_block_fp4_matches_bf16_path(monkeypatch, cin, cout, stride):
    """The block's forward is exact on both MFMA forms (integer conv, int64
    BN statistics): outputs and running statistics agree bit for bit, and
    the backward (which does not depend on the forward form) agrees too."""
    from zookeeper_amd.models.binary_resnet import BinaryResBlock
    from zookeeper_amd.ops import binary

    torch.manual_seed(5)
    blk = BinaryResBlock(cin, cout, stride).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        blk.bn.weight.uniform_(0.5, 1.5)
        blk.bn.bias.uniform_(-0.5, 0.5)
    blk.backend = "hip"
    x = (torch.randn(4, cin, 14, 14, device="cuda") * 1.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    ho = (14 + stride - 1) // stride
    g = torch.randn(4, cout, ho, ho, device="cuda").to(torch.bfloat16)
    res = []
    for fp4 in (True, False):
        monkeypatch.setattr(OPTS, "bconv_fp4", fp4)
        b = copy.deepcopy(blk)
        xx = x.clone().requires_grad_(True)
        out = b(xx)
        out.backward(g)
        res.append((out.float(), b.bn.running_mean.clone(), b.bn.running_var.clone(),
                    xx.grad.float(), b.conv.weight.grad.clone()))
    (o1, m1, v1, dx1, dw1), (o2, m2, v2, dx2, dw2) = res
    assert torch.equal(o1, o2)
    assert torch.equal(m1, m2) and torch.equal(v1, v2)
    assert ((dx1 - dx2).norm() / dx2.norm()).item() < 1e-3
    assert ((dw1 - dw2).norm() / dw2.norm()).item() < 1e-3
