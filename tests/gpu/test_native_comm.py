"""The in-tree RCCL communicator (runtime/comm.cpp via parallel/rccl.py) on
the box's one GPU: a 1-rank communicator, an all-reduce / broadcast on a
chosen stream, and the same all-reduce captured into a HIP graph and
replayed (the property the Trainer's graph mode relies on)."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.timeout(120)
def test_one_rank_all_reduce_broadcast_and_graph_capture():
    from zookeeper_amd.parallel.rccl import NativeComm

    comm = NativeComm(0, 1, tag="zk_test_native")
    s = torch.cuda.Stream()
    x = torch.randn(1 << 20, device="cuda")
    ref = x.clone()
    s.wait_stream(torch.cuda.current_stream())
    comm.all_reduce_(x, stream=s)
    comm.broadcast_(x, root=0, stream=s)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)  # one rank: sum and broadcast are the identity

    y = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        y.add_(1)
        comm.all_reduce_(y)  # captured on the capture stream
        y.mul_(2)
    for k in range(3):
        g.replay()
    torch.cuda.synchronize()
    # ((0+1)*2 + 1)*2 ... : 2, 6, 14
    assert torch.all(y == 14), y[:4]
    comm.close()
