"""Row-streaming 3x3 weight gradient (csrc/kernels/wgrad_rows.hip) against an
fp64 oracle.

* the three operand modes: the bf16 +-1 sign image, (sign_act) the bf16
  activation whose sign the kernel takes in registers -- with exact zeros in
  the activation (sign(0) = +1, larq's ste_sign) and +1 padding -- and the
  e2m1 (FP4) sign image the binary forward reads, expanded in LDS, with +1
  and zero padding (bit-identical to the bf16 image: same products, same
  summation order);
* the image mode with zero padding (the float 3x3 convs of ResNet-50);
* every shape of the dispatch (W = 56 / 28, 64 / 128 channels, Cin != Cout),
  and split counts that exercise each depth of the in-launch fixed-order tree
  (no split, 1, 2 and 3 levels);
* accumulation into an existing dW with the kernel STE mask |w| <= clip;
* bit-identical results run to run (the tree sums in a fixed order);
* the dispatch in ops/_native.igemm_wgrad routes these layers to it.
"""

import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _lib():
    from zookeeper_amd.ops._native import lib

    return lib()


def _oracle(s, dy, w, pad, clip):
    """fp64 dW[co][kh][kw][ci] of 'same' 3x3 stride 1, padding value ``pad``."""
    xp = torch.nn.functional.pad(s.double().permute(0, 3, 1, 2), (1, 1, 1, 1), value=pad)
    gw = torch.nn.grad.conv2d_weight(xp, (w.shape[0], w.shape[3], 3, 3),
                                     dy.double().permute(0, 3, 1, 2), padding=0)
    mask = (w.abs() <= clip).double() if clip is not None else 1.0
    return gw.permute(0, 2, 3, 1) * mask


def _fp4(s):
    """e2m1 image of a +-1 tensor [..., C] -> [..., C/2] bytes (channel 2j in
    the low nibble of byte j: +1 = 0x2, -1 = 0xA), zk_sign_pack's layout."""
    code = torch.where(s.float() >= 0, 2, 10).to(torch.uint8)
    return (code[..., 0::2] | (code[..., 1::2] << 4)).contiguous()


def _run(dy, s, w, dw, pad_ones, sign_act, clip, tb):
    L = _lib()
    B, H, W, Cin = s.shape
    Cin *= 2 if sign_act == 2 else 1  # operand 2: e2m1, two channels per byte
    Cout = dy.shape[3]
    sb, cb = ctypes.c_int64(0), ctypes.c_int64(0)
    assert L.zk_wgrad_rows_plan(B, H, W, Cin, Cout, tb, ctypes.byref(sb), ctypes.byref(cb)) == 0
    slab = torch.empty(max(sb.value // 4, 1), dtype=torch.float32, device="cuda")
    cnt = torch.zeros(max(cb.value // 4, 1), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    rc = L.zk_wgrad_rows(dy.data_ptr(), s.data_ptr(), w.data_ptr() if w is not None else None,
                         dw.data_ptr(), slab.data_ptr(), sb.value, cnt.data_ptr(), cb.value,
                         B, H, W, Cin, Cout, int(pad_ones), int(sign_act),
                         float(clip if clip is not None else 0.0), tb, st)
    assert rc == 0
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0  # every launch leaves its counters zero
    return sb.value // 4 // (Cout * 9 * Cin)


def _data(B, H, W, Cin, Cout, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(B, H, W, Cin, device="cuda", generator=g)
    x[x.abs() < 0.05] = 0.0  # exact zeros: sign(0) = +1
    x = x.to(torch.bfloat16)
    s = torch.where(x >= 0, 1.0, -1.0).to(torch.bfloat16)
    dy = torch.randn(B, H, W, Cout, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.rand(Cout, 3, 3, Cin, device="cuda", generator=g) * 2.6 - 1.3).contiguous()
    return x, s, dy, w


SHAPES = [(6, 56, 56, 64, 64), (8, 28, 28, 128, 128), (4, 28, 28, 64, 128),
          (5, 56, 56, 128, 64)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("tb", [1, 3, 20, 256])
@pytest.mark.parametrize("sign_act", [False, True])
def test_matches_fp64_oracle(shape, tb, sign_act):
    B, H, W, Cin, Cout = shape
    x, s, dy, w = _data(B, H, W, Cin, Cout)
    ref = _oracle(s, dy, w, 1.0, 1.0)
    dw = torch.full_like(w, 0.5)
    _run(dy, x if sign_act else s, w, dw, True, sign_act, 1.0, tb)
    err = (dw.double() - 0.5 - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("shape", SHAPES[:2])
def test_float_operand_zero_padding(shape):
    """Image mode on a real-valued operand with zero padding and no mask: the
    float 3x3 weight gradient of ResNet-50's stage-1/2 convs."""
    B, H, W, Cin, Cout = shape
    x, _, dy, w = _data(B, H, W, Cin, Cout, seed=3)
    ref = _oracle(x, dy, w, 0.0, None)
    dw = torch.zeros_like(w)
    _run(dy, x, None, dw, False, False, None, 256)
    err = (dw.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("sign_act", [False, True])
def test_bit_identical_repeats(sign_act):
    x, s, dy, w = _data(16, 56, 56, 64, 64, seed=5)
    outs = []
    for _ in range(3):
        dw = torch.zeros_like(w)
        _run(dy, x if sign_act else s, w, dw, True, sign_act, 1.0, 256)
        outs.append(dw)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


def test_sign_mode_equals_image_mode():
    """sign(x) in registers and the materialised +-1 image give the same bits."""
    x, s, dy, w = _data(12, 28, 28, 128, 128, seed=7)
    a, b = torch.zeros_like(w), torch.zeros_like(w)
    _run(dy, s, w, a, True, False, 1.0, 256)
    _run(dy, x, w, b, True, True, 1.0, 256)
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("pad_ones", [True, False])
@pytest.mark.parametrize("tb", [3, 256])
def test_fp4_operand_equals_image_mode(shape, pad_ones, tb):
    """op 2 (e2m1 image, expanded in LDS) gives the bits of op 0 on the bf16
    image, and matches the fp64 oracle with either padding value."""
    B, H, W, Cin, Cout = shape
    _, s, dy, w = _data(B, H, W, Cin, Cout, seed=11)
    a, b = torch.zeros_like(w), torch.zeros_like(w)
    _run(dy, s, w, a, pad_ones, 0, 1.0, tb)
    _run(dy, _fp4(s), w, b, pad_ones, 2, 1.0, tb)
    assert torch.equal(a, b)
    ref = _oracle(s, dy, w, 1.0 if pad_ones else 0.0, 1.0)
    err = (b.double() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err


def test_unsupported_shapes_rejected():
    L = _lib()
    assert L.zk_wgrad_rows_plan(8, 14, 14, 256, 256, 0, None, None) != 0  # W not 56 / 28
    assert L.zk_wgrad_rows_plan(8, 57, 56, 64, 64, 0, None, None) != 0   # H % R != 0
    assert L.zk_wgrad_rows_plan(8, 56, 56, 96, 64, 0, None, None) != 0   # channels % 64
    # sign_act needs pad_ones
    dy = torch.zeros(2, 56, 56, 64, dtype=torch.bfloat16, device="cuda")
    dw = torch.zeros(64, 3, 3, 64, device="cuda")
    rc = L.zk_wgrad_rows(dy.data_ptr(), dy.data_ptr(), None, dw.data_ptr(), None, 0, None, 0,
                         2, 56, 56, 64, 64, 0, 1, 1.0, 1, torch.cuda.current_stream().cuda_stream)
    assert rc != 0
    rc = L.zk_wgrad_rows(dy.data_ptr(), dy.data_ptr(), None, dw.data_ptr(), None, 0, None, 0,
                         2, 56, 56, 64, 64, 1, 3, 1.0, 1, torch.cuda.current_stream().cuda_stream)
    assert rc != 0  # no operand mode 3


def test_dispatch_routes_3x3_stride1_layers():
    """ops/_native.igemm_wgrad takes the row kernel for these layers (the
    runtime switch off falls back to zk_igemm_wgrad, same result up to the
    summation order)."""
    from zookeeper_amd.ops import _native
    from zookeeper_amd.ops.options import OPTS, set_options

    x, s, dy, w = _data(8, 56, 56, 64, 64, seed=9)
    geom = (8, 56, 56, 64, 56, 56, 64, 3, 3, 1, 1, 1)
    assert _native.wgrad_rows_ok(geom)
    st = torch.cuda.current_stream().cuda_stream
    a, b = torch.zeros_like(w), torch.zeros_like(w)
    _native.igemm_wgrad(dy, x, w, a, geom, 1, 1.0, st, operand="sign")
    c = torch.zeros_like(w)
    _native.igemm_wgrad(dy, _fp4(s), w, c, geom, 1, 1.0, st, operand="fp4")
    old = OPTS.wgrad_rows
    set_options(wgrad_rows=False)
    try:
        assert not _native.wgrad_rows_ok(geom)
        _native.igemm_wgrad(dy, s, w, b, geom, 1, 1.0, st)
        for op in ("sign", "fp4"):
            with pytest.raises(ValueError):
                _native.igemm_wgrad(dy, x, w, b, geom, 1, 1.0, st, operand=op)
    finally:
        set_options(wgrad_rows=old)
    torch.cuda.synchronize()
    ref = _oracle(s, dy, w, 1.0, 1.0)
    for d in (a, b, c):
        err = (d.double() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-6, err
