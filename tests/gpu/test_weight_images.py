"""bf16 weight images kept by the fused optimizer (ops/weight_images.py).

* a ResNet (1x1, stride-1 3x3 and strided convs: ops/pointwise.py,
  ops/conv3x3.py, ops/conv.py) trained for a few steps with the images on
  ends bit-identical to the run that casts / transposes the weights in every
  pass, with Adam and with SGD;
* after training, every image equals the current fp32 weight cast to bf16 in
  its GEMM layout (the optimizer rewrote them: one registry build in the run);
* a parameter change outside the optimizer plus ``invalidate`` (what a
  checkpoint restore does) rebuilds them.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def _run(images: bool, opt: str, steps: int = 3, graph=False, edit_at=None):
    from zookeeper_amd.core import configure
    from zookeeper_amd.models.resnet import ResNetModule
    from zookeeper_amd.ops.options import OPTS, set_options
    from zookeeper_amd.train import SGD, Adam, Trainer

    old = OPTS.weight_images
    set_options(weight_images=images, deterministic=True)
    try:
        torch.manual_seed(7)
        model = ResNetModule((64, 64, 3), 10, blocks=(1, 1))
        spec = SGD() if opt == "sgd" else Adam()
        configure(spec, {"learning_rate": 1e-2})
        tr = Trainer(model, "sparse_categorical_crossentropy", spec, None, graph=graph,
                     graph_warmup=1)
        g = torch.Generator().manual_seed(3)
        for step in range(steps):
            if step == edit_at:
                # a parameter change outside the fused optimizer (after the
                # graph was captured): an in-place edit of one conv weight
                p = next(p for p in tr.model.parameters() if p.dim() == 4 and p.shape[2] == 3)
                with torch.no_grad():
                    p.mul_(0.5)
            x = torch.randn(4, 3, 64, 64, generator=g).cuda().to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            y = torch.randint(0, 10, (4,), generator=g).cuda()
            tr.train_step(x, y)
        torch.cuda.synchronize()
        return tr
    finally:
        set_options(weight_images=old, deterministic=False)


def _expected(p, flip):
    w = p.detach()
    Cout, Cin, KH, KW = w.shape
    wf = w.flip(2, 3) if flip else w
    fwd = wf.permute(2, 3, 0, 1).reshape(KH * KW, Cout, Cin).to(torch.bfloat16)
    bwd = w.permute(2, 3, 1, 0).reshape(KH * KW, Cin, Cout).to(torch.bfloat16)
    return fwd, bwd


@pytest.mark.parametrize("opt", ["adam", "sgd"])
def test_training_with_images_is_bit_identical(opt):
    on = _run(True, opt)
    off = _run(False, opt)
    reg = on.flat.images
    assert len(reg.entries) >= 6  # stride-1 3x3, strided 3x3, several 1x1
    # built at first use (one full build, then one per newly registered
    # weight), then kept by the optimizer: no rebuild in later steps
    assert reg.builds == 1 and reg.row_builds == len(reg.entries) - 1
    assert not off.flat.images.entries
    torch.testing.assert_close(on.flat.data, off.flat.data, atol=0, rtol=0)
    for e in reg.entries.values():
        fwd, bwd = _expected(e.param, e.flip)
        assert torch.equal(e.fwd, fwd), e.param.shape
        assert torch.equal(e.bwd, bwd), e.param.shape


def test_invalidate_rebuilds_images():
    tr = _run(True, "sgd", steps=1)
    reg = tr.flat.images
    e = next(iter(reg.entries.values()))
    with torch.no_grad():
        tr.flat.data.mul_(0.5)
    reg.invalidate()
    reg.get(e.param, e.flip, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fwd, bwd = _expected(e.param, e.flip)
    assert torch.equal(e.fwd, fwd) and torch.equal(e.bwd, bwd)
    assert reg.builds == 2
    # an in-place edit without invalidate() is caught by the version counters
    with torch.no_grad():
        e.param.mul_(2.0)
    reg.get(e.param, e.flip, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fwd, bwd = _expected(e.param, e.flip)
    assert torch.equal(e.fwd, fwd) and torch.equal(e.bwd, bwd)
    assert reg.builds == 3


def test_graph_replay_refreshes_stale_images():
    """a replayed graph never calls images(); the trainer checks
    the registry before each replay, so an in-place weight edit after capture
    gives the same training as the eager run with the same edit."""
    eager = _run(True, "sgd", steps=4, graph=False, edit_at=2)
    graph = _run(True, "sgd", steps=4, graph=True, edit_at=2)
    assert graph._graph is not None  # steps 1.. replayed
    torch.testing.assert_close(graph.flat.data, eager.flat.data, atol=0, rtol=0)
