"""Determinism of the reductions.

Every mode is bit-reproducible run to run:

* binary-conv forward: exact int16 outputs and exact int64 BN statistics
  (striped integer atomics commute);
* data gradient: no atomics;
* weight gradients: split-K partials summed in a fixed order -- per-split slabs
  + the reduce kernel, or the in-launch fixed-order tree of the row-streaming
  3x3 kernel (wgrad_rows.hip); small-K stem, depthwise and fused-stem weight
  gradients through per-block partials;
* BN-backward sums and the loss: per-block copies summed in a fixed order;
* BN statistics of the float convs (fp64 atomics in the GEMM epilogue): every
  block's partial is rounded to a fixed grid first, so the fp64 additions are
  exact and their order cannot change the result;
* E18, QuickNet and a ResNet (float convs, BN statistics in the epilogues)
  repeat forward + backward bit for bit, and two 5-step default-mode training
  runs end with identical parameters.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _operands(B=4, hw=28, cin=64, cout=64):
    from zookeeper_amd.ops._native import lib, stream_ptr

    L, st = lib(), stream_ptr()
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, hw, hw, cin, device="cuda", generator=g).to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1, 1, generator=g)
    dy = torch.randn(B, hw, hw, cout, device="cuda", generator=g).to(torch.bfloat16)
    nwords = x.numel() // 32
    mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    sx4 = torch.empty(B, hw, hw, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_sign_pack(x.data_ptr(), None, mask.data_ptr(), sx.data_ptr(), sx4.data_ptr(),
                          nwords, 1.0, st) == 0
    wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
    wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
    assert L.zk_weight_pack(w.data_ptr(), None, None, wt.data_ptr(), None, wf4.data_ptr(), cout,
                            9, cin, st) == 0
    return L, st, dict(B=B, hw=hw, cin=cin, cout=cout, x=x, w=w, dy=dy, mask=mask, sx=sx,
                       sx4=sx4, wt=wt, wf4=wf4)


def test_forward_and_dgrad_are_bit_identical():
    L, st, o = _operands()
    B, hw, cin, cout = o["B"], o["hw"], o["cin"], o["cout"]
    outs = []
    for _ in range(3):
        y = torch.empty(B, hw, hw, cout, dtype=torch.int16, device="cuda")
        stats = torch.zeros(32, 2, cout, dtype=torch.int64, device="cuda")
        assert L.zk_igemm_fwd_fp4(o["sx4"].data_ptr(), o["wf4"].data_ptr(), y.data_ptr(),
                                  stats.data_ptr(), B, hw, hw, cin, cout, 3, 3, 1, 1, 1, hw, hw,
                                  0, 0, -1, 32, st) == 0
        dx = torch.empty(B, hw, hw, cin, dtype=torch.bfloat16, device="cuda")
        assert L.zk_igemm_dgrad(o["dy"].data_ptr(), o["wt"].data_ptr(), o["mask"].data_ptr(),
                                None, dx.data_ptr(), B, hw, hw, cin, hw, hw, cout, 3, 3, 1, 1, 1,
                                -1, st) == 0
        torch.cuda.synchronize()
        outs.append((y, stats.sum(0), dx))
    for y, s, dx in outs[1:]:
        assert torch.equal(y, outs[0][0])
        assert torch.equal(s, outs[0][1])
        assert torch.equal(dx, outs[0][2])


@pytest.mark.parametrize("slab", [True, False])
def test_wgrad_reduction_order(slab):
    L, st, o = _operands()
    B, hw, cin, cout = o["B"], o["hw"], o["cin"], o["cout"]
    nb = L.zk_igemm_wgrad_ws_bytes(B, cin, hw, hw, hw, hw, cout, 3, 3, 1, 1, 1, 0, -1)
    ws = torch.empty(max(nb, 4) // 4, device="cuda") if slab else None
    res = []
    for _ in range(3):
        dw = torch.zeros(cout, 3, 3, cin, device="cuda")
        assert L.zk_igemm_wgrad(o["dy"].data_ptr(), o["sx"].data_ptr(), o["w"].data_ptr(),
                                dw.data_ptr(), B, hw, hw, cin, hw, hw, cout, 3, 3, 1, 1, 1, 0,
                                1.0, 0, -1, ws.data_ptr() if ws is not None else None,
                                ws.numel() * 4 if ws is not None else 0, st) == 0
        torch.cuda.synchronize()
        res.append(dw)
    for dw in res[1:]:
        if slab:
            assert torch.equal(dw, res[0])  # fixed-order split-K reduction
        else:
            err = ((dw - res[0]).norm() / res[0].norm()).item()
            assert err < 1e-6, err  # fp32 atomics: ordering noise only


def test_model_forward_and_gradients_bit_identical():
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(1234)
    dev = torch.device("cuda", 0)
    model = prepare_model(BinaryResNetE((64, 64, 3), 10, 18, backend="hip"), dev).train()
    flat = FlatParams(model, dev)
    loss_fn = get_loss("sparse_categorical_crossentropy")
    g = torch.Generator().manual_seed(9)
    x = torch.randn(8, 3, 64, 64, generator=g).to(dev, torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g).to(dev)
    bufs0 = [b.clone() for b in model.buffers()]
    runs = []
    for _ in range(2):
        for b, b0 in zip(model.buffers(), bufs0):
            b.copy_(b0)  # same running statistics before each forward
        flat.zero_grad()
        logits = model(x)
        loss, _ = loss_fn(logits, y)
        loss.backward()
        torch.cuda.synchronize()
        runs.append((logits.detach().clone(), [b.clone() for b in model.buffers()],
                     flat.grad.clone()))
    (l0, b0, g0), (l1, b1, g1) = runs
    assert torch.equal(l0, l1)
    for a, b in zip(b0, b1):
        assert torch.equal(a, b)
    # BN gamma / beta gradients: fixed-order sums -> bit-identical
    for s in flat.slots:
        if s.param.dim() == 1:
            a = g0[s.offset:s.offset + s.numel]
            b = g1[s.offset:s.offset + s.numel]
            assert torch.equal(a, b), s.name
    # conv weight gradients: fixed-order split-K sums -> bit-identical too
    assert torch.equal(g0, g1)


@pytest.fixture
def deterministic():
    from zookeeper_amd.ops import options

    options.set_options(deterministic=True)
    try:
        yield
    finally:
        options.reset()


def _e18_grads(steps_x, model_seed=1234):
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(model_seed)
    dev = torch.device("cuda", 0)
    model = prepare_model(BinaryResNetE((64, 64, 3), 10, 18, backend="hip"), dev).train()
    flat = FlatParams(model, dev)
    loss_fn = get_loss("sparse_categorical_crossentropy")
    x, y = steps_x
    flat.zero_grad()
    from zookeeper_amd.ops import streams

    loss, _ = loss_fn(model(x), y)
    with streams.session(dev):  # side-stream weight gradients on, as in training
        loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), flat.grad.clone(), [b.clone() for b in model.buffers()]


def _batch(seed=9, n=8):
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 3, 64, 64, generator=g).to(dev, torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (n,), generator=g).to(dev)
    return x, y


def _quicknet_grads(steps_x, model_seed=1234):
    from zookeeper_amd.models.quicknet import QuickNetModule
    from zookeeper_amd.ops import streams
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(model_seed)
    dev = torch.device("cuda", 0)
    model = prepare_model(QuickNetModule((64, 64, 3), 10, (1, 1, 1, 1), (64, 128, 256, 512),
                                         backend="hip"), dev).train()
    flat = FlatParams(model, dev)
    loss_fn = get_loss("sparse_categorical_crossentropy")
    x, y = steps_x
    flat.zero_grad()
    loss, _ = loss_fn(model(x), y)
    with streams.session(dev):
        loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), flat.grad.clone(), [b.clone() for b in model.buffers()]


@pytest.mark.parametrize("model", ["e18", "quicknet"])
def test_deterministic_mode_gradients_bit_identical(deterministic, model):
    """Runtime(deterministic=True): no float atomics on the gradient path
    (BN-backward sums per block + fixed-order sum, float BN statistics per
    block, per-row losses summed in order, slab split-K weight gradients; for
    QuickNet also the small-K stem convs' and the depthwise convs' weight
    gradients as per-block partials + a fixed-order reduce): two forward +
    backward passes give bit-identical loss, gradients and BN running
    statistics."""
    batch = _batch()
    fn = _e18_grads if model == "e18" else _quicknet_grads
    l0, g0, b0 = fn(batch)
    l1, g1, b1 = fn(batch)
    assert torch.equal(l0, l1)
    diff = (g0 != g1).nonzero()
    assert diff.numel() == 0, f"{diff.shape[0]} gradient elements differ, first at {diff[:5]}"
    for a, b in zip(b0, b1):
        assert torch.equal(a, b)


def test_deterministic_resume_matches_uninterrupted_run(tmp_path, deterministic):
    """Save at step k, resume in a fresh model/trainer, run to 2k: bit-equal
    to the uninterrupted 2k-step run (deterministic mode)."""
    from zookeeper_amd.core import configure
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.train import Adam, Trainer
    from zookeeper_amd.train import checkpoint as ckpt

    k = 2
    batches = [_batch(seed=100 + i) for i in range(2 * k)]

    def make():
        torch.manual_seed(1234)
        spec = Adam()
        configure(spec, {"learning_rate": 1e-3})
        model = BinaryResNetE((64, 64, 3), 10, 18, backend="hip")
        return Trainer(model, "sparse_categorical_crossentropy", spec)

    full = make()
    for x, y in batches:
        full.train_step(x, y)
    torch.cuda.synchronize()
    ref = full.flat.data.detach().clone()

    first = make()
    for x, y in batches[:k]:
        first.train_step(x, y)
    torch.cuda.synchronize()
    path = ckpt.save(str(tmp_path), k, first.model, first.optimizer)
    resumed = make()
    ckpt.load(path, resumed.model, resumed.optimizer)
    for x, y in batches[k:]:
        resumed.train_step(x, y)
    torch.cuda.synchronize()
    got = resumed.flat.data.detach()
    assert torch.equal(got, ref), (got - ref).abs().max().item()


@pytest.mark.timeout(300)
def test_default_mode_training_runs_bit_identical():
    """Two default-mode E18 training runs (64x64, batch 8, Adam, 5 steps,
    same init and batches) end with bit-identical parameters and losses.
    Before round 4 the BN-backward sums used fp32 atomics and the two runs
    differed at O(1) after two steps (profiles/r3/g_dp_forced_diag.md)."""
    from zookeeper_amd.core import configure
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.train import Adam, Trainer

    batches = [_batch(seed=200 + i) for i in range(5)]

    def run():
        torch.manual_seed(1234)
        spec = Adam()
        configure(spec, {"learning_rate": 1e-3})
        tr = Trainer(BinaryResNetE((64, 64, 3), 10, 18, backend="hip"),
                     "sparse_categorical_crossentropy", spec)
        losses = []
        for x, y in batches:
            loss, _ = tr.train_step(x, y)
            losses.append(float(loss))
        torch.cuda.synchronize()
        return tr.flat.data.detach().clone(), losses

    p0, l0 = run()
    p1, l1 = run()
    assert l0 == l1, (l0, l1)
    assert torch.equal(p0, p1), ((p1 - p0).norm() / p0.norm()).item()


def _resnet_grads(steps_x, model_seed=1234):
    from zookeeper_amd.models.resnet import ResNetModule
    from zookeeper_amd.ops import streams
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    torch.manual_seed(model_seed)
    dev = torch.device("cuda", 0)
    model = prepare_model(ResNetModule((64, 64, 3), 10, blocks=(1, 1)), dev).train()
    flat = FlatParams(model, dev)
    loss_fn = get_loss("sparse_categorical_crossentropy")
    x, y = steps_x
    flat.zero_grad()
    loss, _ = loss_fn(model(x), y)
    with streams.session(dev):
        loss.backward()
    torch.cuda.synchronize()
    return loss.detach().clone(), flat.grad.clone(), [b.clone() for b in model.buffers()]


@pytest.mark.parametrize("model", ["e18", "quicknet", "resnet"])
def test_default_mode_gradients_bit_identical(model):
    """Default mode (runtime.deterministic=False): every split-K weight
    gradient is summed in a fixed order, every BN-backward sum is fixed-order,
    and the float convs' fp64 BN statistics are grid-rounded per block (exact
    fp64 additions), so repeated forward + backward passes give bit-identical
    gradients, loss and BN running statistics -- also for the float ResNet,
    whose 1x1 / 3x3 GEMM epilogues carry those statistics."""
    from zookeeper_amd.ops.options import OPTS

    assert not OPTS.deterministic
    fn = {"e18": _e18_grads, "quicknet": _quicknet_grads, "resnet": _resnet_grads}[model]
    batch = _batch()
    l0, g0, b0 = fn(batch)
    l1, g1, b1 = fn(batch)
    assert torch.equal(l0, l1)
    diff = (g0 != g1).nonzero()
    assert diff.numel() == 0, f"{diff.shape[0]} gradient elements differ, first at {diff[:5]}"
    for a, b in zip(b0, b1):
        assert torch.equal(a, b)


def test_float_wgrad_side_stream_gradients_identical():
    """runtime.float_wgrad_side_stream: the ResNet's 1x1 / 3x3 weight
    gradients run on the side stream (ops.streams.side_wgrad, inputs released
    SIDE_LAG launches later); the gradients must be bit-identical to the
    compute-stream order, and every lagged hold is released at the join."""
    from zookeeper_amd.ops import options, streams

    batch = _batch(seed=17)
    try:
        options.set_options(float_wgrad_side_stream=False)
        base = _resnet_grads(batch)
        options.set_options(float_wgrad_side_stream=True)
        side = _resnet_grads(batch)
    finally:
        options.reset()
    assert not streams._lagged and not streams._keep
    assert torch.equal(base[0], side[0])
    assert torch.equal(base[1], side[1])
