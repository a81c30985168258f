"""Data parallelism on CPU (gloo, world size 2): broadcast of the initial
parameters, bucketed all-reduce overlapped with backward, equivalence with
a single process on the global batch, and launcher failure propagation."""

import os
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)


def _launch(mode, out, nproc=2):
    from zookeeper_amd.parallel.launch import spawn

    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    return spawn([sys.executable, os.path.join(HERE, "dp_worker.py"), mode, str(out)], nproc,
                 env=env)


@pytest.mark.timeout(300)
def test_ddp_matches_single_process(tmp_path):
    assert _launch("train", tmp_path) == 0
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    # replicas stay identical (initial broadcast + averaged gradients)
    torch.testing.assert_close(r0["params"], r1["params"], atol=0, rtol=0)
    assert r0["buckets"] > 1  # several buckets were exercised

    import dp_worker

    single = dp_worker.train(0, 1, bucket_mb=0.001)
    torch.testing.assert_close(r0["params"], single.flat.data, atol=1e-5, rtol=1e-4)


@pytest.mark.timeout(120)
def test_launcher_propagates_failure(tmp_path):
    assert _launch("fail", tmp_path) == 3


@pytest.mark.timeout(120)
def test_hung_rank_is_detected_by_the_collective_timeout(tmp_path):
    """A rank that never reaches a collective: the others' collective times
    out (ZK_DIST_TIMEOUT_S -> init_process_group(timeout=...)), they exit
    non-zero and the launcher terminates the hung rank — the job ends in
    seconds with a failure code instead of hanging."""
    import time

    from zookeeper_amd.parallel.launch import spawn

    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", ZK_DIST_TIMEOUT_S="5")
    env.pop("RANK", None)
    t0 = time.monotonic()
    rc = spawn([sys.executable, os.path.join(HERE, "dp_worker.py"), "hang", str(tmp_path)], 2,
               env=env)
    assert rc != 0
    assert time.monotonic() - t0 < 90


def test_bucketer_layout():
    import torch.nn as nn

    from zookeeper_amd.parallel.ddp import GradBucketer
    from zookeeper_amd.parallel.flat import ALIGN, FlatParams

    m = nn.Sequential(nn.Linear(100, 200), nn.Linear(200, 300), nn.Linear(300, 10))
    flat = FlatParams(m)
    # reverse registration order: the last layer comes first
    assert flat.slots[0].name.endswith("2.bias")
    assert all(s.offset % ALIGN == 0 for s in flat.slots)
    b = GradBucketer(flat, world=1, bucket_mb=0.1, first_bucket_mb=0.01)
    covered = sorted(i for bucket in b.buckets for i in bucket)
    assert covered == list(range(len(flat.slots)))
    # grads are views into the flat buffer
    for s in flat.slots:
        assert s.param.grad.data_ptr() == flat.grad.data_ptr() + 4 * s.offset


@pytest.mark.timeout(120)
def test_bucketer_waits_for_a_deferred_direct_gradient():
    """A kernel that writes a gradient straight into the flat buffer returns
    None to autograd, whose post-accumulate hook still fires; the bucket must
    launch at the writer's own readiness signal (``_zk_grad_ready``: for a
    side-stream weight gradient that comes a block later, once its event
    exists), not at autograd's call.  Launching at autograd's call all-reduced
    side-stream weight gradients before they were computed
    (``tests/gpu/test_dp_gpu.py`` two-rank mismatch, profiles/r5/dp_hook_race.md)."""
    import socket

    import torch.distributed as dist
    import torch.nn as nn

    from zookeeper_amd.ops._native import direct_grad, grad_ready
    from zookeeper_amd.parallel.ddp import GradBucketer
    from zookeeper_amd.parallel.flat import FlatParams

    deferred = []

    class DirectScale(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(x)
            ctx.w = w
            return x * w

        @staticmethod
        def backward(ctx, g):
            (x,) = ctx.saved_tensors
            gw = direct_grad(ctx.w)
            assert gw is not None
            gw.add_((g * x).sum(0))
            deferred.append(ctx.w)  # readiness signalled later, like ops/streams.py
            return g * ctx.w, None

    class M(nn.Module):
        def __init__(self):
            super().__init__()
            self.w = nn.Parameter(torch.ones(8))

        def forward(self, x):
            return DirectScale.apply(x, self.w)

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1)
    try:
        m = M()
        flat = FlatParams(m)
        b = GradBucketer(flat, world=1, force=True)
        flat.zero_grad()
        m(torch.randn(4, 8, requires_grad=True)).sum().backward()
        assert b._order == []  # autograd's hook call did not launch the bucket
        for p in deferred:
            grad_ready(p)
        assert b._order == [0]
        b.finish()
        assert b.last_order == [0]
        b.remove()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bn_buffers_all_reduced(tmp_path):
    assert _launch("bnsync", tmp_path) == 0
    r = [torch.load(tmp_path / f"bn{i}.pt", weights_only=True) for i in range(2)]
    for key in ("running_mean", "running_var"):
        assert not torch.equal(r[0]["before"][key], r[1]["before"][key])
        mean = (r[0]["before"][key] + r[1]["before"][key]) / 2
        torch.testing.assert_close(r[0]["after"][key], mean)
        torch.testing.assert_close(r[1]["after"][key], mean)
    # integer buffers are left alone
    assert int(r[0]["after"]["num_batches_tracked"]) == 3
