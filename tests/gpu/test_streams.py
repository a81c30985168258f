"""Binary-conv weight gradients on the side stream (ops/streams.py): the
same gradients as the single-stream backward, and every deferred readiness
signalled (each direct-gradient parameter reported ready exactly once)."""

import pytest
import torch

from zookeeper_amd.ops.options import OPTS

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _grads(side: bool, monkeypatch):
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.ops import streams
    from zookeeper_amd.parallel.flat import FlatParams
    from zookeeper_amd.train.losses import get_loss
    from zookeeper_amd.train.trainer import prepare_model

    monkeypatch.setattr(OPTS, "wgrad_side_stream", side)
    torch.manual_seed(1234)
    dev = torch.device("cuda", 0)
    model = prepare_model(BinaryResNetE((64, 64, 3), 10, 18, backend="hip"), dev).train()
    flat = FlatParams(model, dev)
    ready = []
    for s in flat.slots:
        s.param._zk_grad_ready = (lambda n=s.name: ready.append(n))
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 3, 64, 64, generator=g).to(dev, torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g).to(dev)
    loss, _ = get_loss("sparse_categorical_crossentropy")(model(x), y)
    with streams.session(dev):
        loss.backward()
    torch.cuda.synchronize()
    return flat.grad.clone(), ready, flat


def test_side_stream_wgrad_matches_single_stream(monkeypatch):
    g_side, ready_side, flat = _grads(True, monkeypatch)
    g_one, ready_one, _ = _grads(False, monkeypatch)
    # fp32-atomic ordering noise in the split-K / BN-backward sums (~1e-7),
    # amplified through the binary blocks (README "Known issues"): measured
    # 1e-6 .. 3.4e-3 over the whole gradient; a missing or doubled weight
    # gradient is O(1).  The deterministic mode is bit-exact (next test).
    assert ((g_side - g_one).norm() / g_one.norm()).item() < 3e-2
    # every binary conv weight reported ready once, in both modes
    convs = [s.name for s in flat.slots if s.name.endswith("conv.weight")]
    for name in convs:
        assert ready_side.count(name) == 1 and ready_one.count(name) == 1, name


def test_side_stream_wgrad_bit_exact_in_deterministic_mode(monkeypatch):
    """With fixed-order reductions the side stream changes only where the
    weight gradients run, not what they compute: bit-identical gradients."""
    from zookeeper_amd.ops import options

    old = options.OPTS.deterministic
    try:
        options.set_options(deterministic=True)
        g_side, _, _ = _grads(True, monkeypatch)
        g_one, _, _ = _grads(False, monkeypatch)
    finally:
        options.set_options(deterministic=old)
    assert torch.equal(g_side, g_one), ((g_side - g_one).norm() / g_one.norm()).item()
