"""Whole-model checks on the native path against the fp32 torch oracle
(same weights, same bf16-rounded input), at reduced size:

* ResNet-50 (float network, bottleneck tail as ONE fused BN + residual +
  ReLU pass): loss and every parameter gradient agree with the oracle;
* QuickNet-Large / BinaryResNet-E18 (binary networks): the loss agrees and
  every gradient is finite and non-zero.  Binary networks' per-parameter
  gradients are not comparable at model level (a bf16 rounding of the
  input already flips activation signs; see test_conv_family), their
  layers are pinned to fp64 by the kernel tests.
"""

import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


def _prep(m):
    m = m.cuda()
    for mod in m.modules():
        for _, p in mod.named_parameters(recurse=False):
            if p.dim() == 4:
                p.data = p.data.contiguous(memory_format=torch.channels_last)
    return m


@pytest.mark.parametrize("C,relu", [(64, True), (256, True), (128, False)])
def test_bn_residual_relu_matches_fp64(C, relu):
    from zookeeper_amd.nn.layers import BatchNorm
    from zookeeper_amd.ops import norm_pool

    torch.manual_seed(0)
    bn = BatchNorm(C, 0.9, 1e-5).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = _cl(torch.randn(4, C, 9, 9, device="cuda").to(torch.bfloat16)).requires_grad_(True)
    r = _cl(torch.randn(4, C, 9, 9, device="cuda").to(torch.bfloat16)).requires_grad_(True)
    y = norm_pool.batch_norm(x, bn, relu=relu, residual=r)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    xd = x.detach().double().requires_grad_(True)
    rd = r.detach().double().requires_grad_(True)
    w = bn.weight.detach().double().requires_grad_(True)
    b = bn.bias.detach().double().requires_grad_(True)
    ref = F.batch_norm(xd, None, None, w, b, True, 0.0, 1e-5) + rd
    if relu:
        ref = F.relu(ref)
    ref.backward(g.double())
    for got, want, tol in ((y, ref, 2e-2), (x.grad, xd.grad, 3e-2), (r.grad, rd.grad, 1e-2),
                           (bn.weight.grad, w.grad, 2e-2), (bn.bias.grad, b.grad, 2e-2)):
        err = (got.double() - want).abs().max().item()
        assert err <= tol * (want.abs().max().item() + 1e-3), (err, want.abs().max().item())


@pytest.mark.parametrize("C", [64, 256])
def test_bn_relu_backward_recomputes_the_stored_mask(C):
    """BN + ReLU without a residual keeps no output for the backward: the
    ReLU mask is recomputed from x.  Pinned against the fp64 BN backward
    taken through the mask of the STORED forward output (a mask element
    recomputed differently moves dx by ~|g|, far above the tolerance)."""
    from zookeeper_amd.nn.layers import BatchNorm
    from zookeeper_amd.ops import norm_pool

    torch.manual_seed(3)
    bn = BatchNorm(C, 0.9, 1e-5).cuda()
    with torch.no_grad():
        bn.weight.uniform_(-1.5, 1.5)  # negative scales too
        bn.bias.uniform_(-0.5, 0.5)
    x = _cl(torch.randn(8, C, 10, 10, device="cuda").to(torch.bfloat16)).requires_grad_(True)
    y = norm_pool.batch_norm(x, bn, relu=True)
    g = torch.randn_like(y.float()).to(torch.bfloat16)
    y.backward(g)
    xd = x.detach().double()
    n = xd.numel() // C
    mean = xd.mean(dim=(0, 2, 3), keepdim=True)
    var = xd.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    rstd = (var + 1e-5).rsqrt()
    xhat = (xd - mean) * rstd
    gm = g.double() * (y.detach() > 0)
    dbeta = gm.sum(dim=(0, 2, 3), keepdim=True)
    dgamma = (gm * xhat).sum(dim=(0, 2, 3), keepdim=True)
    w = bn.weight.detach().double().view(1, C, 1, 1)
    dx = w * rstd / n * (n * gm - dbeta - xhat * dgamma)
    for got, want in ((x.grad, dx), (bn.bias.grad, dbeta.flatten()),
                      (bn.weight.grad, dgamma.flatten())):
        err = (got.double() - want).abs().max().item()
        assert err <= 2e-2 * (want.abs().max().item() + 1e-3), (err, want.abs().max().item())


def test_bottleneck_residual_handoff_matches_autograd_sum(monkeypatch):
    """Identity bottleneck: x's shortcut gradient added in conv1's dgrad
    epilogue (norm_pool.ResidualHandoff) equals autograd's separate sum."""
    from zookeeper_amd.models.resnet import Bottleneck
    from zookeeper_amd.ops import norm_pool

    torch.manual_seed(4)
    blk = _prep(Bottleneck(256, 64, 1))
    with torch.no_grad():
        blk.bn3.weight.fill_(0.5)
    x = _cl(torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16))
    g = torch.randn(4, 256, 14, 14, device="cuda").to(torch.bfloat16)

    def run():
        xi = x.clone().requires_grad_(True)
        for p in blk.parameters():
            p.grad = None
        blk(xi).backward(g)
        return xi.grad.double(), [p.grad.double().clone() for p in blk.parameters()]

    made = []
    real = norm_pool.ResidualHandoff

    def spy():
        made.append(real())
        return made[-1]

    monkeypatch.setattr(norm_pool, "ResidualHandoff", spy)
    gx, gp = run()
    assert made and made[-1].dres is None  # created, filled and consumed
    monkeypatch.setattr(norm_pool, "ResidualHandoff", lambda: None)
    gx0, gp0 = run()
    # one bf16 rounding of (dgrad + dres) instead of two
    assert (gx - gx0).abs().max().item() <= 1e-2 * gx0.abs().max().item()
    for a, b in zip(gp, gp0):
        assert (a - b).abs().max().item() <= 1e-2 * (b.abs().max().item() + 1e-6)


@pytest.mark.parametrize("cin,width,stride,hw", [(64, 64, 1, 14), (256, 128, 2, 14)])
def test_downsample_bottleneck_handoff_matches_autograd_sum(monkeypatch, cin, width, stride, hw):
    """Downsampling bottleneck: conv1's input gradient handed to the shortcut
    conv's data-gradient epilogue (1x1 pointwise at stride 1, the strided
    conv kernel at stride 2) equals autograd's separate sum."""
    from zookeeper_amd.models.resnet import Bottleneck
    from zookeeper_amd.ops import norm_pool

    torch.manual_seed(6)
    blk = _prep(Bottleneck(cin, width, stride))
    with torch.no_grad():
        blk.bn3.weight.fill_(0.5)
    x = _cl(torch.randn(4, cin, hw, hw, device="cuda").to(torch.bfloat16))
    ho = hw // stride
    g = torch.randn(4, width * 4, ho, ho, device="cuda").to(torch.bfloat16)

    def run():
        xi = x.clone().requires_grad_(True)
        for p in blk.parameters():
            p.grad = None
        blk(xi).backward(g)
        return xi.grad.double(), [p.grad.double().clone() for p in blk.parameters()]

    made = []
    real = norm_pool.ResidualHandoff

    def spy():
        made.append(real())
        return made[-1]

    monkeypatch.setattr(norm_pool, "ResidualHandoff", spy)
    gx, gp = run()
    # created, filled by conv1, consumed (closed) by the shortcut conv
    assert made and made[-1].closed and made[-1].dres is None
    monkeypatch.setattr(norm_pool, "ResidualHandoff", lambda: None)
    gx0, gp0 = run()
    assert (gx - gx0).abs().max().item() <= 1e-2 * gx0.abs().max().item()
    for a, b in zip(gp, gp0):
        assert (a - b).abs().max().item() <= 1e-2 * (b.abs().max().item() + 1e-6)


def test_handoff_order_guard():
    """A producer that runs after its consumer gets False from give() (the
    gradient then goes back to autograd instead of being dropped)."""
    from zookeeper_amd.ops.norm_pool import ResidualHandoff

    h = ResidualHandoff()
    assert h.take() is None and h.closed
    assert h.give(torch.zeros(1)) is False and h.dres is None
    h2 = ResidualHandoff()
    t = torch.ones(2)
    assert h2.give(t) is True and h2.take() is t


def test_binary_transition_handoff_matches_autograd_sum(monkeypatch):
    """E18 stage transition: x's binary-conv gradient handed to the shortcut
    avg-pool's backward (zk_avgpool2_bwd_add) equals autograd's separate sum."""
    from zookeeper_amd.models.binary_resnet import BinaryResBlock
    from zookeeper_amd.ops import norm_pool

    torch.manual_seed(5)
    blk = _prep(BinaryResBlock(64, 128, 2, backend="hip"))
    x = _cl(torch.randn(4, 64, 16, 16, device="cuda").to(torch.bfloat16))
    g = torch.randn(4, 128, 8, 8, device="cuda").to(torch.bfloat16)

    def run():
        xi = x.clone().requires_grad_(True)
        for p in blk.parameters():
            p.grad = None
        blk(xi).backward(g)
        return xi.grad.double(), [p.grad.double().clone() for p in blk.parameters()]

    made = []
    real = norm_pool.ResidualHandoff

    def spy():
        made.append(real())
        return made[-1]

    monkeypatch.setattr(norm_pool, "ResidualHandoff", spy)
    gx, gp = run()
    assert made and made[-1].dres is None  # created, filled and consumed
    monkeypatch.setattr(norm_pool, "ResidualHandoff", lambda: None)
    gx0, gp0 = run()
    assert (gx - gx0).abs().max().item() <= 1e-2 * gx0.abs().max().item()
    for a, b in zip(gp, gp0):
        assert (a - b).abs().max().item() <= 1e-2 * (b.abs().max().item() + 1e-6)


def _step(m, x, y):
    from zookeeper_amd.train.losses import softmax_cross_entropy

    out = m(x)
    loss, _ = softmax_cross_entropy(out, y) if x.dtype == torch.bfloat16 else (
        F.cross_entropy(out.float(), y), None)
    loss.backward()
    return loss.item()


def _cosines(m, ref):
    out = {}
    for (n, p), (_, pr) in zip(m.named_parameters(), ref.named_parameters()):
        a, b = p.grad.flatten().double(), pr.grad.flatten().double()
        assert torch.isfinite(a).all(), n
        if b.norm() > 1e-8:
            out[n] = (a @ b / (a.norm() * b.norm() + 1e-30)).item()
    return out


@pytest.mark.timeout(120)
def test_resnet50_step_matches_fp32_oracle(monkeypatch):
    """Native bf16 ResNet-50 step vs the fp32 oracle, measured against what
    bf16 itself costs: the same model through the library bf16 path (torch
    ops, MIOpen / hipBLASLt) vs the same fp32 oracle.  The native path must
    be at least as close to fp32 as library bf16 is."""
    from zookeeper_amd.models import resnet
    from zookeeper_amd.models.resnet import ResNetModule
    from zookeeper_amd.nn import layers

    torch.manual_seed(1)
    m = _prep(ResNetModule((64, 64, 3), 10, blocks=(1, 1, 2, 1)))
    with torch.no_grad():  # non-zero last-BN gammas so every branch carries gradient
        for mod in m.modules():
            if hasattr(mod, "bn3"):
                mod.bn3.weight.fill_(0.5)
    ref = copy.deepcopy(m)
    lib16 = copy.deepcopy(m)
    x = _cl(torch.randn(8, 3, 64, 64, device="cuda").to(torch.bfloat16))
    y = torch.randint(0, 10, (8,), device="cuda")
    loss = _step(m, x, y)
    loss_r = _step(ref, x.float(), y)
    monkeypatch.setattr(layers, "_use_native", lambda t: False)
    monkeypatch.setattr(resnet, "_use_native", lambda t: False)
    out16 = lib16(x)
    F.cross_entropy(out16.float(), y).backward()
    assert abs(loss - loss_r) < 0.02 * abs(loss_r) + 0.02, (loss, loss_r)
    cn, cl = _cosines(m, ref), _cosines(lib16, ref)
    mean_n, mean_l = sum(cn.values()) / len(cn), sum(cl.values()) / len(cl)
    assert mean_n > 0.9 and mean_n >= mean_l - 0.02, (mean_n, mean_l)
    assert min(cn.values()) >= min(cl.values()) - 0.05, (
        sorted(cn.items(), key=lambda t: t[1])[:4], sorted(cl.items(), key=lambda t: t[1])[:4])


@pytest.mark.timeout(120)
@pytest.mark.parametrize("name", ["QuickNetLarge", "BinaryResNetE18"])
def test_binary_models_step_loss_matches_fp32_oracle(name):
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.models.quicknet import QuickNetModule

    torch.manual_seed(2)
    if name == "QuickNetLarge":
        m = QuickNetModule((64, 64, 3), 10, (2, 2, 2, 2), (64, 128, 256, 512), backend="hip")
        r = QuickNetModule((64, 64, 3), 10, (2, 2, 2, 2), (64, 128, 256, 512), backend="torch")
    else:
        m = BinaryResNetE((64, 64, 3), 10, 18, backend="hip")
        r = BinaryResNetE((64, 64, 3), 10, 18, backend="torch")
    r.load_state_dict(m.state_dict())
    m, r = _prep(m), _prep(r)
    # batch 32: at random init a binary network's loss moves by ~+-15% under
    # a 1e-3 input perturbation even in fp32 (measured on CPU, batch 8), so
    # the bound is loose; the learning test pins convergence instead
    x = _cl(torch.randn(32, 3, 64, 64, device="cuda").to(torch.bfloat16))
    y = torch.randint(0, 10, (32,), device="cuda")
    loss = _step(m, x, y)
    loss_r = _step(r, x.float(), y)
    assert abs(loss - loss_r) < 0.15 * abs(loss_r) + 0.1, (loss, loss_r)
    for n, p in m.named_parameters():
        assert torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0, n


@pytest.mark.timeout(180)
@pytest.mark.parametrize("name", ["QuickNetLarge", "BinaryResNetE18"])
def test_binary_models_grad_direction_vs_fp32_oracle(name):
    """Model-level gradient direction of the binary networks: per-parameter
    cosine similarity of the native bf16 step's gradients with the fp32
    oracle's (torch backend, fp32, same weights and inputs), judged against
    what bf16 itself costs -- the same model on the library bf16 path
    (torch backend, bf16 input) vs the same oracle.  A binary network
    amplifies rounding into sign flips, so the bound is relative: the native
    path must be at least as close to fp32 as library bf16 is (mean cosine
    within 0.03, lower-decile parameter within 0.1), and positively aligned on
    average (> 0.1).  No absolute bound near 1 is possible at random init:
    measured on MI355X, QuickNetLarge's library-bf16 gradients have mean
    cosine 0.21 with the fp32 oracle's (native: 0.23) -- bf16 rounding of the
    activations alone flips enough signs to decorrelate them.  The inputs are
    bf16-exact, so the float stem sees identical data on every path."""
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.models.quicknet import QuickNetModule

    torch.manual_seed(3)

    def make(backend):
        if name == "QuickNetLarge":
            return QuickNetModule((64, 64, 3), 10, (2, 2, 2, 2), (64, 128, 256, 512),
                                  backend=backend)
        return BinaryResNetE((64, 64, 3), 10, 18, backend=backend)

    m = make("hip")
    ref, lib16 = make("torch"), make("torch")
    ref.load_state_dict(m.state_dict())
    lib16.load_state_dict(m.state_dict())
    m, ref, lib16 = _prep(m), _prep(ref), _prep(lib16)
    x = _cl(torch.randn(32, 3, 64, 64, device="cuda").to(torch.bfloat16))
    y = torch.randint(0, 10, (32,), device="cuda")
    _step(m, x, y)
    _step(ref, x.float(), y)
    out16 = lib16(x)
    F.cross_entropy(out16.float(), y).backward()
    cn, cl = _cosines(m, ref), _cosines(lib16, ref)
    mean_n, mean_l = sum(cn.values()) / len(cn), sum(cl.values()) / len(cl)
    worst = sorted(cn.items(), key=lambda t: t[1])[:4]
    print(f"{name}: mean cos native {mean_n:.4f} library-bf16 {mean_l:.4f}; "
          f"worst native {worst}; worst library {min(cl.values()):.4f}")
    assert mean_n > 0.1, (mean_n, worst)
    assert mean_n >= mean_l - 0.03, (mean_n, mean_l)
    # lower decile rather than the single worst parameter: the worst ones are
    # near-cancelling BN biases whose cosine is run-to-run atomic-order noise
    # on both paths (QuickNetLarge stem BN bias: -0.38 .. -0.53 across runs)
    def q10(c):
        v = sorted(c.values())
        return v[len(v) // 10]
    assert q10(cn) >= q10(cl) - 0.1, (worst, q10(cn), q10(cl))


@pytest.mark.timeout(180)
@pytest.mark.parametrize("name", ["BinaryResNetE18", "QuickNetLarge"])
def test_binary_models_teacher_forced_unit_gradients(name):
    """Absolute model-level gradient check of the binary networks (the
    companion of the relative test above).  One native bf16 training step runs
    the whole network; every top-level unit -- the stem, each body block, the
    head -- is then re-run by the fp32 torch oracle on that unit's OWN native
    input and output gradient, captured from the step.  Both sides therefore
    see the same sign decisions (each block binarises its input once, and the
    captured input is bf16-exact), so what is left is bf16 vs fp32 rounding
    inside the unit, and each parameter's gradient must agree at cosine >=
    0.99.  A wrong-but-plausible gradient in any one block fails here even
    when the whole-network cosine stays positive.  Exempt, and printed:
    parameters whose oracle gradient norm is below 1e-3 of the median
    parameter's -- a gradient that vanishes up to rounding has no direction to
    compare.  Such parameters are stem BN parameters that another
    normalisation follows: E18's BN-1 scale (BN-2 normalises the max-pooled
    BN-1 output again, so the loss is invariant to it but for the ReLU / pool
    selection; measured on MI355X: oracle norm 9e-6 against a median of
    ~1e-2, native cosine 0.02) and QuickNet's stem BN scale / bias (norms
    5e-6 / 2e-7 against a median of 0.2).  Reference: the QuantConv2D /
    QuantDense stack of /root/reference/examples/larq_experiment.py:59-103."""
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.models.quicknet import QuickNetModule
    from zookeeper_amd.nn.layers import pooled_dense
    from zookeeper_amd.train.losses import softmax_cross_entropy

    torch.manual_seed(5)

    def make(backend):
        if name == "QuickNetLarge":
            return QuickNetModule((64, 64, 3), 10, (2, 2, 2, 2), (64, 128, 256, 512),
                                  backend=backend)
        return BinaryResNetE((64, 64, 3), 10, 18, backend=backend)

    m = make("hip")
    ref = make("torch")
    ref.load_state_dict(m.state_dict())
    m, ref = _prep(m), _prep(ref).float()
    x = _cl(torch.randn(32, 3, 64, 64, device="cuda").to(torch.bfloat16))
    y = torch.randint(0, 10, (32,), device="cuda")

    units = [("stem", m.stem, ref.stem)] + [
        (f"body.{i}", b, rb) for i, (b, rb) in enumerate(zip(m.body, ref.body))]
    cap = {}

    def hook(nm):
        def fwd(mod, inp, out):
            cap[nm] = [inp[0].detach().clone()]
            out.register_hook(lambda g: cap[nm].append(g.detach().clone()))
        return fwd

    handles = [u.register_forward_hook(hook(nm)) for nm, u, _ in units]
    feats = {}

    def head_in(mod, inp, out):
        feats["x"] = out.detach().clone()
        out.register_hook(lambda g: feats.__setitem__("g_body", g.detach().clone()))

    handles.append(m.body.register_forward_hook(head_in))
    logits = m(x)
    logits.register_hook(lambda g: feats.__setitem__("g_logits", g.detach().clone()))
    loss, _ = softmax_cross_entropy(logits, y)
    loss.backward()
    for hd in handles:
        hd.remove()
    torch.cuda.synchronize()

    rows = []

    def compare(nm, unit, runit):
        for (pn, p), (_, pr) in zip(unit.named_parameters(), runit.named_parameters()):
            a, b = p.grad.flatten().double(), pr.grad.flatten().double()
            assert torch.isfinite(a).all(), (nm, pn)
            cos = (a @ b / (a.norm() * b.norm() + 1e-30)).item()
            rows.append((f"{nm}.{pn}", cos, b.norm().item()))

    for nm, unit, runit in units:
        xin, gout = cap[nm]
        runit.zero_grad(set_to_none=True)
        out = runit(xin.float())
        out.backward(gout.float().reshape(out.shape))
        compare(nm, unit, runit)
    # head: ReLU + global average pool + dense on the last block's native output
    ref.fc.zero_grad(set_to_none=True)
    out = pooled_dense(feats["x"].float(), ref.pool, ref.fc, relu=True)
    out.backward(feats["g_logits"].float())
    compare("head", m.fc, ref.fc)
    med = sorted(r[2] for r in rows)[len(rows) // 2]
    exempt = {r[0] for r in rows if r[2] < 1e-3 * med}
    worst = sorted(rows, key=lambda r: r[1])[:6]
    print(f"{name}: {len(rows)} parameters, median oracle grad norm {med:.3g}, worst cosines "
          + ", ".join(f"{n} {c:.4f} (|g| {gn:.2g}{', exempt' if n in exempt else ''})"
                      for n, c, gn in worst))
    # only stem BN parameters vanish this way (BN after BN / pool, see above)
    assert all(n.startswith("stem.") for n in exempt), exempt
    fails = [(n, round(c, 4)) for n, c, _ in rows if n not in exempt and c < 0.99]
    assert not fails, fails
