"""Checkpoint layout, atomic save, pruning and bit-exact resume (CPU)."""

import json
import os

import torch
import torch.nn as nn

from zookeeper_amd.core import configure
from zookeeper_amd.parallel.dist import DistInfo
from zookeeper_amd.train import Adam, Trainer
from zookeeper_amd.train import checkpoint as ckpt


def _trainer(seed=0):
    torch.manual_seed(seed)
    model = nn.Sequential(nn.Linear(6, 8), nn.ReLU(), nn.Linear(8, 3))
    spec = Adam()
    configure(spec, {"learning_rate": 0.05})
    return Trainer(model, "sparse_categorical_crossentropy", spec, DistInfo())


def _batches(n):
    g = torch.Generator().manual_seed(3)
    return [(torch.randn(5, 6, generator=g), torch.randint(0, 3, (5,), generator=g))
            for _ in range(n)]


def test_save_layout_and_prune(tmp_path):
    tr = _trainer()
    for step in (1, 2, 3, 4):
        ckpt.save(str(tmp_path), step, tr.model, tr.optimizer, keep=2)
    d = tmp_path / "checkpoints"
    assert sorted(os.listdir(d)) == ["step_00000003", "step_00000004"]
    files = sorted(os.listdir(d / "step_00000004"))
    assert files == ["meta.json", "model.pt", "optimizer.pt", "rng_rank0.pt"]
    assert json.load(open(d / "step_00000004" / "meta.json"))["step"] == 4
    assert ckpt.latest(str(tmp_path)).endswith("step_00000004")
    # a half-written (tmp) checkpoint is ignored
    os.makedirs(d / "step_00000009.tmp")
    assert ckpt.latest(str(tmp_path)).endswith("step_00000004")


def test_resume_is_bit_exact(tmp_path):
    data = _batches(6)
    ref = _trainer()
    for x, y in data:
        ref.train_step(x, y)

    a = _trainer()
    for x, y in data[:3]:
        a.train_step(x, y)
    ckpt.save(str(tmp_path), 3, a.model, a.optimizer)

    b = _trainer(seed=99)  # different init: everything must come from the checkpoint
    meta = ckpt.load(ckpt.latest(str(tmp_path)), b.model, b.optimizer)
    assert meta["step"] == 3
    for x, y in data[3:]:
        b.train_step(x, y)
    torch.testing.assert_close(b.flat.data, ref.flat.data, atol=0, rtol=0)


def test_graph_mode_is_gpu_single_process_only():
    import pytest

    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(6, 8), nn.ReLU(), nn.Linear(8, 3))
    spec = Adam()
    configure(spec, {"learning_rate": 0.05})
    for mode in (True, "auto"):
        tr = Trainer(model, "sparse_categorical_crossentropy", spec, DistInfo(), graph=mode)
        assert not tr.graph  # CPU device: always eager
        x, y = _batches(1)[0]
        loss, _ = tr.train_step(x, y)
        assert torch.isfinite(loss)
    with pytest.raises(ValueError):
        Trainer(model, "sparse_categorical_crossentropy", spec, DistInfo(), graph="yes")


def test_adam_matches_keras_update_form():
    """Default Adam = tf.keras Adam: p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps)
    (hand-computed over a few steps); "textbook" = m_hat/(sqrt(v_hat)+eps)."""
    import math

    from zookeeper_amd.parallel.flat import FlatParams

    def run(form):
        torch.manual_seed(0)
        lin = nn.Linear(4, 3, bias=False)
        spec = Adam()
        configure(spec, {"learning_rate": 0.1, "epsilon": 1e-3, "epsilon_form": form})
        flat = FlatParams(lin)
        opt = spec.create(flat)
        g = torch.Generator().manual_seed(1)
        grads = [torch.randn(12, generator=g) * 1e-3 for _ in range(4)]
        p0 = flat.data.clone()
        for gr in grads:
            flat.grad[:12].copy_(gr)
            opt.step()
        return p0[:12], flat.data[:12].clone(), grads

    p0, keras_p, grads = run("keras")
    p, m, v = p0.double().clone(), torch.zeros(12, dtype=torch.float64), torch.zeros(12, dtype=torch.float64)
    for t, gr in enumerate(grads, start=1):
        gd = gr.double()
        m = 0.9 * m + 0.1 * gd
        v = 0.999 * v + 0.001 * gd * gd
        lr_t = 0.1 * math.sqrt(1 - 0.999**t) / (1 - 0.9**t)
        p = p - lr_t * m / (v.sqrt() + 1e-3)
    torch.testing.assert_close(keras_p.double(), p, atol=1e-6, rtol=1e-5)
    _, text_p, _ = run("textbook")
    # eps = 1e-3 against |g| ~ 1e-3: the two forms differ measurably early on
    assert (text_p - keras_p).abs().max() > 1e-4
