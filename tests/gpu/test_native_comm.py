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


@pytest.mark.timeout(120)
def test_missing_peer_raises_instead_of_hanging():
    """NativeComm(0, 2) with no second rank: the set-up rendezvous raises
    within its deadline (before ncclCommInitRank could hang)."""
    import time
    from datetime import timedelta

    import torch.distributed as dist

    from zookeeper_amd.parallel.rccl import NativeComm

    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    store = dist.TCPStore("127.0.0.1", port, 2, True, timedelta(seconds=30),
                          wait_for_workers=False)
    t0 = time.monotonic()
    with pytest.raises(TimeoutError):
        NativeComm(0, 2, store=store, tag="zk_test_no_peer", timeout_s=3)
    assert time.monotonic() - t0 < 30


@pytest.mark.timeout(120)
def test_watchdog_flags_a_collective_past_its_deadline():
    """The watchdog follows an event that never completes in time (a stream
    blocked behind a long kernel stands in for a hung collective): it aborts
    the communicator and check() raises in the calling thread."""
    import time

    from zookeeper_amd.parallel.rccl import NativeComm

    comm = NativeComm(0, 1, tag="zk_test_watchdog", timeout_s=0.5)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        torch.cuda._sleep(int(3e9))  # ~1.5 s of a spinning kernel
        ev = torch.cuda.Event()
        ev.record(s)
    comm.watch(ev, "test collective")
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="did not complete"):
        while time.monotonic() - t0 < 20:
            comm.check()
            time.sleep(0.05)
    comm._stop.set()
    torch.cuda.synchronize()
