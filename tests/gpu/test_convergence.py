"""Whole-network training correctness: the native bf16 path (HIP kernels)
against the pure-PyTorch fp32 path on a learnable synthetic task.

Task: 10 classes, each a fixed smooth random image (a class template); a
sample is 0.3x its class template plus Gaussian noise of 2.5x the template's
scale (hard enough that neither path saturates in 150 steps).  Both runs start from the same weights, see the same batches and use
the same Adam settings (the reference trains BinaryNet with Keras Adam,
examples/larq_experiment.py:118-122).  After ~150 steps the native run's
held-out accuracy must be well above chance and within a stated tolerance of
the fp32 run's; the loss curves are written to $ZK_CURVE_DIR when set
(profiles/r3/convergence_{BinaryNet,BinaryResNetE18,QuickNet}.json hold the recorded ones, with the row-window dgrad and fused BN sums on; the GPU suite is run
with ZK_CURVE_DIR=gpurun_out/curves by scripts/gpu.sh).
"""

import copy
import json
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from zookeeper_amd import ops

    assert ops.available(), ops.load_error()


def _templates(n_cls, hw, seed=123):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(n_cls, 3, hw // 8, hw // 8, generator=g)
    t = F.interpolate(t, size=(hw, hw), mode="bilinear", align_corners=False)
    return t / t.std()


def _batch(tpl, n, gen, signal=0.3, noise=2.5):
    y = torch.randint(0, tpl.shape[0], (n,), generator=gen)
    x = signal * tpl[y] + noise * torch.randn((n,) + tpl.shape[1:], generator=gen)
    return x, y


def _progress(msg):
    # a line per 10 steps into $ZK_CURVE_DIR/progress.log: the first fp32
    # steps wait on MIOpen kernel builds, and a GPU box takes a run that
    # writes nothing for minutes to be hung
    out_dir = os.environ.get("ZK_CURVE_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "progress.log"), "a") as f:
            f.write(msg + "\n")


def _run(model, dtype, tpl, steps, batch, lr, seed, tag):
    from zookeeper_amd.train.optimizers import Adam
    from zookeeper_amd.train.trainer import Trainer

    tr = Trainer(model, "softmax_cross_entropy", Adam(learning_rate=lr))
    gen = torch.Generator().manual_seed(seed)
    curve = []
    for i in range(steps):
        x, y = _batch(tpl, batch, gen)
        x = x.to("cuda", dtype).contiguous(memory_format=torch.channels_last)
        loss, _ = tr.train_step(x, y.cuda())
        curve.append(float(loss))
        if i % 10 == 0:
            _progress(f"{tag} step {i} loss {curve[-1]:.4f}")
    # held-out accuracy, eval mode (running BN statistics)
    gen_eval = torch.Generator().manual_seed(seed + 1)
    hits = total = 0
    model.eval()
    with torch.no_grad():
        for _ in range(4):
            x, y = _batch(tpl, 128, gen_eval)
            x = x.to("cuda", dtype).contiguous(memory_format=torch.channels_last)
            out = model(x).float()
            hits += (out.argmax(1).cpu() == y).sum().item()
            total += y.numel()
    return curve, hits / total


def _models(name):
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.models.binarynet import BinaryNetModule

    torch.manual_seed(0)
    if name == "BinaryResNetE18":
        hip = BinaryResNetE((64, 64, 3), 10, 18, backend="hip")
        ref = BinaryResNetE((64, 64, 3), 10, 18, backend="torch")
        ref.load_state_dict(hip.state_dict())
        return hip, ref, 64
    if name == "QuickNet":
        from zookeeper_amd.models.quicknet import QuickNetModule

        hip = QuickNetModule((64, 64, 3), 10, (2, 2, 2, 2), (32, 64, 128, 256), backend="hip")
        ref = QuickNetModule((64, 64, 3), 10, (2, 2, 2, 2), (32, 64, 128, 256), backend="torch")
        ref.load_state_dict(hip.state_dict())
        return hip, ref, 64
    hip = BinaryNetModule((32, 32, 3), 10, filters=64, dense_units=256)
    ref = copy.deepcopy(hip)
    return hip, ref, 32


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["BinaryResNetE18", "BinaryNet", "QuickNet"])
def test_native_training_matches_fp32(name):
    hip, ref, hw = _models(name)
    tpl = _templates(10, hw)
    steps, batch, lr = 150, 64, 2e-3
    c_hip, acc_hip = _run(hip, torch.bfloat16, tpl, steps, batch, lr, seed=7, tag=f"{name} bf16")
    c_ref, acc_ref = _run(ref, torch.float32, tpl, steps, batch, lr, seed=7, tag=f"{name} fp32")
    rec = {"model": name, "steps": steps, "batch": batch, "lr": lr, "input": [hw, hw, 3],
           "task": "0.3 x one of 10 smooth class templates + N(0, 2.5^2) noise",
           "native_bf16": {"loss": c_hip, "heldout_acc": acc_hip},
           "torch_fp32": {"loss": c_ref, "heldout_acc": acc_ref}}
    out_dir = os.environ.get("ZK_CURVE_DIR")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"convergence_{name}.json"), "w") as f:
            json.dump(rec, f)
    print(f"{name}: native acc {acc_hip:.3f} (loss {c_hip[0]:.3f} -> {c_hip[-1]:.3f}), "
          f"fp32 acc {acc_ref:.3f} (loss {c_ref[0]:.3f} -> {c_ref[-1]:.3f})")
    assert all(map(lambda v: v == v, c_hip)), "NaN loss"
    # well above chance (0.1) and within 0.1 (absolute) of the fp32 run
    assert acc_hip >= 0.3, (acc_hip, acc_ref)
    assert acc_hip >= acc_ref - 0.1, (acc_hip, acc_ref)
    # the loss fell on the native path
    assert sum(c_hip[-10:]) < 0.8 * sum(c_hip[:10]), c_hip[::15]
