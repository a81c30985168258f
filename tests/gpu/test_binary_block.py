"""Fused binary residual block (XNOR-popcount conv + BN + STE) vs the
pure-PyTorch oracle: forward output, BN running statistics and all
gradients.  The oracle runs in fp32 on the same ±1 semantics."""

import copy

import pytest
import torch

from zookeeper_amd.ops.options import OPTS

from zookeeper_amd.models.binary_resnet import BinaryResBlock
from zookeeper_amd.models.quicknet import QuickNetBlock

pytestmark = pytest.mark.gpu


def _setup():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _run(block, x, backend, g):
    block = block.train()
    block.backend = backend
    xx = x.detach().clone().requires_grad_(True)
    if backend == "torch":
        # fp32 oracle
        blk = copy.deepcopy(block).float()
        out = blk(xx.float())
        out.backward(g.float())
        return out.float(), xx.grad.float(), blk
    out = block(xx)
    out.backward(g)
    return out.float(), xx.grad.float(), block


CASES = [
    # (cin, cout, stride, H)  — E18 shapes (reduced batch)
    (64, 64, 1, 14),
    (64, 64, 1, 28),     # weight gradient on the e2m1 image (wgrad_rows op 2)
    (128, 128, 1, 28),
    (64, 128, 2, 14),
    (128, 128, 1, 7),
    (256, 512, 2, 8),
]


@pytest.mark.parametrize("cin,cout,stride,hw", CASES)
def test_binary_res_block_matches_oracle(cin, cout, stride, hw):
    _setup()
    torch.manual_seed(0)
    blk = BinaryResBlock(cin, cout, stride).cuda()
    with torch.no_grad():
        blk.bn.weight.uniform_(0.5, 1.5)
        blk.bn.bias.uniform_(-0.5, 0.5)
        blk.conv.weight.uniform_(-1, 1)
    x = (torch.randn(4, cin, hw, hw, device="cuda") * 1.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    ho = (hw + stride - 1) // stride
    g = torch.randn(4, cout, ho, ho, device="cuda").to(torch.bfloat16)
    g = g.contiguous(memory_format=torch.channels_last)

    ref_blk = copy.deepcopy(blk)
    out_h, dx_h, b_h = _run(blk, x, "hip", g)
    out_r, dx_r, b_r = _run(ref_blk, x, "torch", g)

    torch.testing.assert_close(out_h, out_r, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(b_h.bn.running_mean, b_r.bn.running_mean, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(b_h.bn.running_var, b_r.bn.running_var, atol=1e-2, rtol=1e-3)
    # gradients: bf16 GEMMs vs fp32 oracle
    scale = dx_r.abs().max().item()
    assert (dx_h - dx_r).abs().max().item() <= 3e-2 * scale + 1e-3
    for name in ("conv.weight", "bn.weight", "bn.bias"):
        gh = dict(b_h.named_parameters())[name].grad.float()
        gr = dict(b_r.named_parameters())[name].grad.float()
        err = (gh - gr).abs().max().item()
        assert err <= 3e-2 * gr.abs().max().item() + 1e-3, f"{name}: {err}"


def test_quicknet_block_matches_oracle():
    _setup()
    torch.manual_seed(1)
    blk = QuickNetBlock(64).cuda()
    with torch.no_grad():
        blk.conv.weight.uniform_(-1.25, 1.25)
    x = (torch.randn(2, 64, 10, 10, device="cuda")).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    g = torch.randn(2, 64, 10, 10, device="cuda").to(torch.bfloat16)
    g = g.contiguous(memory_format=torch.channels_last)
    ref = copy.deepcopy(blk)
    out_h, dx_h, b_h = _run(blk, x, "hip", g)
    out_r, dx_r, b_r = _run(ref, x, "torch", g)
    torch.testing.assert_close(out_h, out_r, atol=5e-2, rtol=2e-2)
    scale = dx_r.abs().max().item()
    assert (dx_h - dx_r).abs().max().item() <= 3e-2 * scale + 1e-3


def test_bconv_forward_exact_integers():
    """The raw XNOR conv output must equal the ±1 convolution exactly."""
    _setup()
    from zookeeper_amd.nn.layers import pad_same_nhwc
    from zookeeper_amd.nn.quantizers import sign_pm1
    from zookeeper_amd.ops._native import lib, stream_ptr
    import torch.nn.functional as F

    torch.manual_seed(3)
    for (cin, cout, stride, hw, pad_ones) in [(32, 64, 1, 9, 0), (64, 128, 2, 12, 0),
                                              (128, 64, 1, 5, 1), (512, 64, 1, 3, 0)]:
        B = 3
        x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, 3, 3, cin, device="cuda")
        L = lib()
        st = stream_ptr()
        nwords = x.numel() // 32
        bits = torch.empty(nwords, dtype=torch.int32, device="cuda")
        L.zk_sign_pack(x.data_ptr(), bits.data_ptr(), None, None, None, nwords, 1.0, st)
        wbits = torch.empty(cout * 9 * cin // 32, dtype=torch.int32, device="cuda")
        wpop = torch.empty(cout * 9, dtype=torch.int32, device="cuda")
        L.zk_weight_pack(w.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), None, None, None, cout, 9,
                         cin, st)
        from zookeeper_amd.nn.layers import same_padding
        pt, pb = same_padding(hw, 3, stride)
        ho = (hw + pt + pb - 3) // stride + 1
        y = torch.empty(B, ho, ho, cout, dtype=torch.int16, device="cuda")
        stats = torch.zeros(2, cout, dtype=torch.int64, device="cuda")
        rc = L.zk_bconv_fwd(bits.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), y.data_ptr(),
                            stats.data_ptr(), B, hw, hw, cin, cout, 3, 3, stride, pt, pt, ho, ho,
                            pad_ones, 0, st)
        assert rc == 0
        xs = sign_pm1(x.float()).permute(0, 3, 1, 2)
        xs = pad_same_nhwc(xs, (3, 3), (stride, stride), 1.0 if pad_ones else 0.0)
        ws = sign_pm1(w).permute(0, 3, 1, 2)
        ref = F.conv2d(xs.double(), ws.double(), stride=stride).permute(0, 2, 3, 1)
        assert torch.equal(y.double(), ref), (cin, cout, stride, hw, pad_ones)
        assert torch.equal(stats[0].double(), ref.sum(dim=(0, 1, 2)))
        assert torch.equal(stats[1].double(), (ref * ref).sum(dim=(0, 1, 2)))


def test_chained_blocks_reuse_fused_quantisation():
    """Block 1's BN epilogue quantises its output for block 2 (sign image +
    STE mask, ``_zk_sign``); the chain must match recomputing them."""
    _setup()
    from zookeeper_amd import ops

    torch.manual_seed(5)
    b1 = BinaryResBlock(64, 64, 1).cuda().to(memory_format=torch.channels_last)
    b2 = BinaryResBlock(64, 128, 2).cuda().to(memory_format=torch.channels_last)
    with torch.no_grad():
        for b in (b1, b2):
            b.bn.weight.uniform_(0.5, 1.5)
            b.bn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(4, 64, 14, 14, device="cuda") * 1.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    g = torch.randn(4, 128, 7, 7, device="cuda").to(torch.bfloat16)
    results = []
    for fused in (True, False):
        c1, c2 = copy.deepcopy(b1), copy.deepcopy(b2)
        xx = x.clone().requires_grad_(True)
        h = ops.binary_block(xx, xx, c1.conv, c1.bn, quantize_output=fused)
        assert hasattr(h, "_zk_sign") == fused
        res = c2.downsample(h) if c2.downsample is not None else h
        out = ops.binary_block(h, res, c2.conv, c2.bn)
        out.backward(g)
        results.append((out.float(), xx.grad.float(), c1.conv.weight.grad.clone(),
                        c2.conv.weight.grad.clone()))
    (o1, *g1), (o2, *g2) = results
    torch.testing.assert_close(o1, o2, atol=0, rtol=0)  # forward is deterministic
    for a, b in zip(g1, g2):  # fp32 atomics in the reductions: order-dependent
        assert ((a - b).norm() / b.norm()).item() < 1e-3


@pytest.mark.parametrize("second_consumer", [False, True])
def test_fused_bn_backward_sums_match_separate_reduce(monkeypatch, second_consumer):
    """A block whose output feeds only the next block (identity shortcut)
    gets its BN-backward sums from that block's dgrad epilogue
    (zk_igemm_dgrad_bnsum): the row-window kernel (conv3rw.hip, 64 -> 64
    stride 1), which always fuses.  Gradients must match the separate reduce
    (dgrad_rw off); with a second consumer of the output (gradient
    accumulated after the dgrad) the block must detect it and fall back."""
    _setup()
    from zookeeper_amd import ops
    from zookeeper_amd.ops import binary

    torch.manual_seed(11)
    blocks = [BinaryResBlock(64, 64, 1).cuda().to(memory_format=torch.channels_last)
              for _ in range(3)]
    with torch.no_grad():
        for b in blocks:
            b.bn.weight.uniform_(0.5, 1.5)
            b.bn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(4, 64, 28, 28, device="cuda") * 1.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    g = torch.randn(4, 64, 28, 28, device="cuda").to(torch.bfloat16)
    res = []
    for fuse in (True, False):
        monkeypatch.setattr(OPTS, "dgrad_rw", fuse)
        bs = [copy.deepcopy(b) for b in blocks]
        xx = x.clone().requires_grad_(True)
        h = xx
        outs = []
        for b in bs:
            h = ops.binary_block(h, h, b.conv, b.bn)
            outs.append(h)
        loss = (h.float() * g.float()).sum()
        if second_consumer:
            loss = loss + (outs[0].float() * 0.5).sum()
        loss.backward()
        res.append([xx.grad.float()] + [p.grad.clone() for b in bs for p in b.parameters()])
    for a, b in zip(*res):
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 2e-3


@pytest.mark.parametrize("hw", [28, 56])
def test_fp4_weight_gradient_skips_bf16_sign_image(monkeypatch, hw):
    """With the consumer links of the model (``sign_consumer``) a block whose
    next conv's weight gradient reads the e2m1 image (wgrad_rows operand 2)
    writes no bf16 sign image, and the gradients equal the bf16-image run
    (runtime.wgrad_fp4 off) -- the weight gradients bit for bit: same products,
    same fixed summation order."""
    _setup()
    from zookeeper_amd import ops

    torch.manual_seed(21)
    blocks = [BinaryResBlock(64, 64, 1).cuda().to(memory_format=torch.channels_last)
              for _ in range(3)]
    with torch.no_grad():
        for b in blocks:
            b.bn.weight.uniform_(0.5, 1.5)
            b.bn.bias.uniform_(-0.5, 0.5)
    x = (torch.randn(2, 64, hw, hw, device="cuda") * 1.5).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    g = torch.randn(2, 64, hw, hw, device="cuda").to(torch.bfloat16)
    res = []
    for fp4 in (True, False):
        monkeypatch.setattr(OPTS, "wgrad_fp4", fp4)
        monkeypatch.setattr(OPTS, "wgrad_side_stream", False)
        bs = [copy.deepcopy(b) for b in blocks]
        xx = x.clone().requires_grad_(True)
        h = xx
        for i, b in enumerate(bs):
            nxt = bs[i + 1].conv if i + 1 < len(bs) else None
            h = ops.binary_block(h, h, b.conv, b.bn, sign_consumer=nxt)
            if nxt is not None:
                # (clip, bf16 sign image, mask, e2m1 image)
                assert (h._zk_sign[1] is None) == fp4
                assert h._zk_sign[3] is not None
        (h.float() * g.float()).sum().backward()
        res.append([xx.grad.float()] + [b.conv.weight.grad.clone() for b in bs])
    (dx1, *w1), (dx2, *w2) = res
    assert ((dx1 - dx2).norm() / dx2.norm()).item() < 1e-3
    for a, b in zip(w1, w2):
        assert torch.equal(a, b)


@pytest.mark.timeout(120)
def test_shortcut_pool_from_the_bn_epilogue_is_bit_identical():
    """ops.binary_block(pool_out=True): a stage's last block writes the next
    block's 2x2/2 average-pooled shortcut input in its BN-apply pass
    (zk_bn_apply_sign_pool) and avg_pool2 takes it; the E18 forward, loss and
    every gradient must equal the separate pooling pass bit for bit."""
    import copy

    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    a = prepare_model(BinaryResNetE((64, 64, 3), 10, 18, backend="hip"), dev).train()
    assert sum(blk.pool_out for blk in a.body) == 3  # one per stage transition
    b = copy.deepcopy(a)
    for blk in b.body:
        blk.pool_out = False
    x = torch.randn(6, 3, 64, 64, device=dev).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    ya, yb = a(x), b(x)
    assert torch.equal(ya, yb)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p.grad, q.grad), n
    for (n, u), (_, v) in zip(a.named_buffers(), b.named_buffers()):
        assert torch.equal(u, v), n
