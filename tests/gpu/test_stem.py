"""Fused ImageNet stem (stem.hip) vs the same modules run one by one
(library conv + bf16 BN/pool kernels), training mode: output, running
statistics and every parameter gradient."""

import copy

import pytest
import torch

from zookeeper_amd.nn.layers import BatchNorm, ImageStem, MaxPool2d, QuantConv2d

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _stem(with_bn2):
    mods = [QuantConv2d(3, 64, 7, 2, "same", kernel_initializer="he_normal"),
            BatchNorm(64, 0.9, 1e-5, activation="relu"), MaxPool2d(3, 2, "same")]
    if with_bn2:
        mods.append(BatchNorm(64, 0.9, 1e-5))
    return ImageStem(*mods)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("hw,with_bn2", [(64, True), (56, False), (224, True)])
def test_fused_stem_matches_unfused(hw, with_bn2):
    """The fused bf16 stem must be as close to the fp32 oracle as the
    unfused bf16 path (library conv + bf16 BN/pool kernels) is: the weight
    gradient goes through a dense bf16 dy1 with large cancelling BN terms in
    both, so only relative-to-baseline accuracy is meaningful there."""
    torch.manual_seed(0)
    fused = _stem(with_bn2).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in fused.modules():
            if isinstance(m, BatchNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    unfused = copy.deepcopy(fused)
    oracle = copy.deepcopy(fused).float()
    B = 4 if hw == 224 else 6
    x = torch.randn(B, 3, hw, hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    assert fused._fusable(x)
    y = fused(x)
    y_bf = torch.nn.Sequential.forward(unfused, x)
    y_ref = torch.nn.Sequential.forward(oracle, x.float())
    assert y.shape == y_ref.shape
    assert _rel(y, y_ref) < max(1.5 * _rel(y_bf, y_ref), 1e-2)
    g = torch.randn_like(y_ref).to(torch.bfloat16)
    y.backward(g)
    y_bf.backward(g)
    y_ref.backward(g.float())
    for (n, p), (_, q), (_, r) in zip(fused.named_parameters(), unfused.named_parameters(),
                                      oracle.named_parameters()):
        assert p.grad is not None, n
        e_fused, e_lib = _rel(p.grad, r.grad), _rel(q.grad, r.grad)
        assert e_fused < max(1.5 * e_lib, 2e-2), (n, e_fused, e_lib)
    for (n, b), (_, c) in zip(fused.named_buffers(), oracle.named_buffers()):
        torch.testing.assert_close(b, c, atol=3e-3, rtol=3e-3)


def test_fused_stem_eval_matches():
    torch.manual_seed(1)
    fused = _stem(True).cuda().to(memory_format=torch.channels_last).eval()
    with torch.no_grad():
        for m in fused.modules():
            if isinstance(m, BatchNorm):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
    x = torch.randn(2, 3, 64, 64, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    ref = copy.deepcopy(fused).float()
    with torch.no_grad():
        assert fused._fusable(x)
        y = fused(x)
        y_ref = torch.nn.Sequential.forward(ref, x.float())
    assert _rel(y, y_ref) < 2e-2


def test_fused_stem_sign_handoff_matches_sign_pack():
    """With ``sign_clip`` the stem's last BN pass also emits the first binary
    block's sign image and STE mask; they must equal zk_sign_pack of the
    stem output bit for bit."""
    from zookeeper_amd.ops._native import lib, stream_ptr

    torch.manual_seed(2)
    stem = _stem(True).cuda().to(memory_format=torch.channels_last)
    stem.sign_clip = 0.75
    x = torch.randn(3, 3, 64, 64, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = stem(x)
    clip, sx, mask, sx4 = y._zk_sign
    assert clip == 0.75
    yn = y.permute(0, 2, 3, 1).contiguous()
    nwords = yn.numel() // 32
    ref_mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    ref_sx = torch.empty_like(yn)
    ref_sx4 = torch.empty(yn.shape[:3] + (yn.shape[3] // 2,), dtype=torch.uint8, device="cuda")
    assert lib().zk_sign_pack(yn.data_ptr(), None, ref_mask.data_ptr(), ref_sx.data_ptr(),
                              ref_sx4.data_ptr(), nwords, 0.75, stream_ptr(y.device)) == 0
    torch.cuda.synchronize()
    assert torch.equal(sx.view(torch.int16), ref_sx.view(torch.int16))
    assert torch.equal(mask, ref_mask)
    if sx4 is not None:
        assert torch.equal(sx4, ref_sx4)


@pytest.mark.parametrize("hw,B", [(64, 5), (56, 6), (224, 3), (50, 2)])
def test_recompute_fused_stem_matches_materialising(hw, B, monkeypatch):
    """stem_fused.hip (conv recomputed in the stats, pool and weight-gradient
    passes; no y1 / dy1 tensors) against stem.hip's materialising kernels and
    the fp32 oracle: the same y1 bf16 values by construction, so the outputs
    agree to the BN-1 statistics' summation order; every gradient is at least
    as close to fp32 as the materialising path's (whose BN-1 backward sums use
    yhat reconstructed from the bf16 pooled value, the fused path the exact
    y1 at the argmax)."""
    import zookeeper_amd.ops.stem as stem_mod

    torch.manual_seed(3)
    base = _stem(True).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in base.modules():
            if isinstance(m, BatchNorm):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    oracle = copy.deepcopy(base).float()
    x = torch.randn(B, 3, hw, hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y_ref = torch.nn.Sequential.forward(oracle, x.float())
    g = torch.randn_like(y_ref).to(torch.bfloat16)
    y_ref.backward(g.float())
    ref = {n: p.grad for n, p in oracle.named_parameters()}
    runs = {}
    for fused in (False, True):
        monkeypatch.setattr(stem_mod.OPTS, "stem_fused", fused)  # runtime.stem_fused
        m = copy.deepcopy(base)
        y = m(x)
        y.backward(g)
        torch.cuda.synchronize()
        runs[fused] = (y.detach().float(), {n: p.grad.clone() for n, p in m.named_parameters()},
                       {n: b.clone() for n, b in m.named_buffers()})
    (y0, g0, b0), (y1, g1, b1) = runs[False], runs[True]
    assert _rel(y1, y0) < 2e-3
    for n in g0:
        e1, e0 = _rel(g1[n], ref[n]), _rel(g0[n], ref[n])
        assert e1 < max(1.5 * e0, 2e-2), (n, e1, e0)
    for n in b0:
        torch.testing.assert_close(b1[n], b0[n], atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("nb", [1500, 50176])
def test_two_pass_finalize_matches_one_pass(nb):
    """zk_bn_finalize_partials_ws (coalesced fp64 first pass over the
    per-tile partial rows, then the finalize over 256 rows) gives the
    coefficients and running statistics of the one-pass kernel."""
    from zookeeper_amd.ops._native import lib, stream_ptr

    L, st = lib(), stream_ptr()
    C = 64
    torch.manual_seed(7)
    part = torch.randn(nb, 2, C, device="cuda")
    part[:, 1] = part[:, 1].abs() * 3 + 1.0  # sums of squares
    P = float(nb * 128)
    outs = []
    for ws in (False, True):
        coef = torch.empty(4, C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        if ws:
            buf = torch.empty(L.zk_bn_finalize_ws_bytes(C) // 8, dtype=torch.float64,
                              device="cuda")
            assert L.zk_bn_finalize_partials_ws(part.data_ptr(), nb, C, P, None, None, 1e-5, 0.9,
                                                rm.data_ptr(), rv.data_ptr(), coef.data_ptr(),
                                                buf.data_ptr(), st) == 0
        else:
            assert L.zk_bn_finalize_partials(part.data_ptr(), nb, C, P, None, None, 1e-5, 0.9,
                                             rm.data_ptr(), rv.data_ptr(), coef.data_ptr(),
                                             st) == 0
        torch.cuda.synchronize()
        outs.append((coef, rm, rv))
    for a, b in zip(outs[0], outs[1]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_bn2_sums_from_the_first_binary_block(monkeypatch):
    """E18's stem hands its BN-2 to the first binary block like the binary
    blocks do among themselves: the block's row-window dgrad epilogue sums
    (dx, dx * yhat) over the stem output's gradient, and the stem backward
    skips its own reduce.  Same BN-2 gradients as the stem's own reduce
    (up to summation order)."""
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.ops import stem as stem_mod

    torch.manual_seed(3)
    x = torch.randn(8, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)

    def run(handoff: bool):
        torch.manual_seed(5)
        model = BinaryResNetE((64, 64, 3), 10, 18, backend="hip").cuda()
        for p in model.parameters():
            if p.dim() == 4:
                p.data = p.data.contiguous(memory_format=torch.channels_last)
        model.train()
        if not handoff:
            orig = stem_mod.fused_stem

            def no_handoff(*a, **k):
                out = orig(*a, **k)
                out.__dict__.pop("_zk_bnsum", None)
                return out
            monkeypatch.setattr(stem_mod, "fused_stem", no_handoff)
        before = stem_mod.FUSED_BN2_SUMS[0]
        out = model(x)
        out.float().square().mean().backward()
        used = stem_mod.FUSED_BN2_SUMS[0] - before
        monkeypatch.undo()
        bn2 = model.stem[3]
        return used, bn2.weight.grad.clone(), bn2.bias.grad.clone()

    used, gw, gb = run(True)
    used0, gw0, gb0 = run(False)
    assert used == 1 and used0 == 0
    torch.testing.assert_close(gw, gw0, rtol=1e-4, atol=1e-4 * gw0.abs().max().item())
    torch.testing.assert_close(gb, gb0, rtol=1e-4, atol=1e-4 * gb0.abs().max().item())


@pytest.mark.parametrize("flip", [False, True])
def test_loader_packed_input_is_bit_identical(flip):
    """runtime.loader_preprocess: the loader's fused normalise + pack kernel
    writes the stem's padded input next to the image (PACK_SPECS, published by
    the first stem forward); the stem then takes it (no pack kernel) and every
    output and gradient must equal the self-packing run bit for bit."""
    from zookeeper_amd import ops
    from zookeeper_amd.ops import stem as stem_ops

    torch.manual_seed(3)
    mean, std = (123.7, 116.3, 103.5), (58.4, 57.1, 57.4)
    img = torch.randint(0, 256, (4, 64, 64, 3), dtype=torch.uint8, device="cuda")
    a = _stem(True).cuda().to(memory_format=torch.channels_last)
    b = copy.deepcopy(a)
    x_ref = ops.normalize_flip(img, mean, std, flip, seed=77).permute(0, 3, 1, 2)
    y_a = a(x_ref)  # publishes the padded-input spec of this shape
    spec = stem_ops.PACK_SPECS[(64, 64, 3)]
    out, xp = ops.normalize_flip_pack(img, mean, std, flip, spec, seed=77)
    assert torch.equal(out, x_ref.permute(0, 2, 3, 1))
    x = out.permute(0, 3, 1, 2)
    x._zk_stem_xp = (xp, spec, x._version)
    n0 = stem_ops.PREPACKED[0]
    y_b = b(x)
    assert stem_ops.PREPACKED[0] == n0 + 1  # the stem took the loader's xp
    assert torch.equal(y_a, y_b)
    g = torch.randn_like(y_a)
    y_a.backward(g)
    y_b.backward(g)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p.grad, q.grad), n
    # a modified input is not paired with a stale padded copy
    x.add_(0)
    n1 = stem_ops.PREPACKED[0]
    b(x)
    assert stem_ops.PREPACKED[0] == n1
