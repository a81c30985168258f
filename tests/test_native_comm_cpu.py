"""Set-up of the native RCCL communicator without RCCL (parallel/rccl.py):
the store rendezvous that hands rank 0's unique id to every rank, with the
RCCL calls replaced by injectable stubs.

* two processes over a TCPStore: both ranks receive the same 128-byte id for
  each tag, and different tags get different ids;
* a rank whose peer never arrives raises TimeoutError within the deadline
  instead of hanging in ncclCommInitRank;
* the gradient bucketer folds buckets below 256 KB into the next one.
"""

import multiprocessing as mp
import os
import socket
import time

import pytest


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out):
    from datetime import timedelta

    import torch.distributed as dist

    from zookeeper_amd.parallel.rccl import NativeComm

    store = dist.TCPStore("127.0.0.1", port, world, rank == 0, timedelta(seconds=60))
    got = {}
    for tag in ("zk_test_a", "zk_test_b"):
        c = NativeComm(rank, world, store=store, tag=tag, timeout_s=60,
                       _make_uid=lambda: os.urandom(128), _init=lambda uid, w, r: 1 + r)
        got[tag] = (c.uid, c.handle)
        c.close()
    out.put((rank, got))
    time.sleep(0.5)  # keep rank 0's store alive until the peer has read


@pytest.mark.timeout(120)
def test_two_ranks_receive_the_same_unique_id_per_tag():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=90) for _ in ps)
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    for tag in ("zk_test_a", "zk_test_b"):
        assert res[0][tag][0] == res[1][tag][0]
        assert len(res[0][tag][0]) == 128
        assert res[0][tag][1] == 1 and res[1][tag][1] == 2  # each rank's own init
    assert res[0]["zk_test_a"][0] != res[0]["zk_test_b"][0]


@pytest.mark.timeout(60)
def test_missing_peer_raises_within_the_deadline():
    from datetime import timedelta

    import torch.distributed as dist

    from zookeeper_amd.parallel.rccl import NativeComm

    store = dist.TCPStore("127.0.0.1", _free_port(), 2, True, timedelta(seconds=30),
                          wait_for_workers=False)
    t0 = time.monotonic()
    with pytest.raises(TimeoutError, match=r"rank\(s\) \[1\] did not join"):
        NativeComm(0, 2, store=store, tag="zk_test_lonely", timeout_s=2,
                   _make_uid=lambda: b"x" * 128, _init=lambda uid, w, r: 1)
    assert time.monotonic() - t0 < 20


def test_small_buckets_are_folded():
    import torch.nn as nn

    from zookeeper_amd.parallel.ddp import MIN_BUCKET_BYTES, GradBucketer
    from zookeeper_amd.parallel.flat import FlatParams

    # head bias (4 KB) first, then a 2 MB head weight: the first-bucket cap
    # (1 MB) used to leave the bias alone in a 4 KB bucket
    m = nn.Sequential(nn.Linear(1024, 1024), nn.Linear(512, 1000))
    flat = FlatParams(m)
    b = GradBucketer(flat, world=1, bucket_mb=10.0, first_bucket_mb=1.0)
    sizes = [(hi - lo) * 4 for lo, hi in b.ranges]
    assert all(s >= MIN_BUCKET_BYTES for s in sizes), sizes  # (cap 10 MB: full threshold)
    covered = sorted(i for bucket in b.buckets for i in bucket)
    assert covered == list(range(len(flat.slots)))


# --- connect(): the agreed set-up of the "auto" transport (VERDICT r5 item 3,
# ADVICE r5).  Two processes over a TCPStore, RCCL replaced by stubs; one rank
# fails in a given phase and BOTH ranks must return None promptly.

def _connect_main(rank, world, port, fail, out):
    from datetime import timedelta

    import torch.distributed as dist

    from zookeeper_amd.parallel import rccl

    store = dist.TCPStore("127.0.0.1", port, world, rank == 0, timedelta(seconds=60))
    bad = rank == 1

    def load():
        if bad and fail == "load":
            raise RuntimeError("stub: no librccl")

    def init(uid, w, r):
        if bad and fail == "init":
            raise RuntimeError("stub: ncclCommInitRank failed")
        if bad and fail == "init_hang":
            time.sleep(600)
        return 100 + r

    def canary(comm):
        if bad and fail == "canary":
            raise RuntimeError("stub: canary sum mismatch")

    t0 = time.monotonic()
    comm = rccl.connect(rank, world, store=store, fallback=True, timeout_s=60,
                        init_timeout_s=3, tag=f"zk_conn_{fail}", log=lambda m: None,
                        _load=load, _make_uid=lambda: os.urandom(128), _init=init,
                        _canary=canary)
    out.put((rank, None if comm is None else comm.handle, time.monotonic() - t0))
    time.sleep(1.0)  # keep rank 0's store alive until the peer has voted/read


@pytest.mark.timeout(120)
@pytest.mark.parametrize("fail", ["none", "load", "init", "init_hang", "canary"])
def test_connect_agrees_on_fallback_when_one_rank_fails(fail):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_connect_main, args=(r, 2, port, fail, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, handle, dt = q.get(timeout=90)
        res[r] = (handle, dt)
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    if fail == "none":
        assert res[0][0] == 100 and res[1][0] == 101
    else:
        # every rank falls back together, none waits out the 60 s rendezvous
        assert res[0][0] is None and res[1][0] is None, res
    for r in (0, 1):
        assert res[r][1] < 30, res


def test_connect_without_fallback_raises():
    from zookeeper_amd.parallel import rccl

    def load():
        raise RuntimeError("stub: no librccl")

    with pytest.raises(RuntimeError, match="RCCL load"):
        rccl.connect(0, 1, fallback=False, tag="zk_conn_strict", log=lambda m: None,
                     _load=load, _make_uid=lambda: b"x" * 128, _init=lambda u, w, r: 1,
                     _canary=lambda c: None)


def test_init_deadline_and_locked_abort():
    """A stub init that never returns raises TimeoutError at the deadline;
    the watchdog's failure path (_fail) takes the handle mutex, so a holder
    (an enqueue in progress) delays it, and check() cancels the hard exit."""
    import threading

    from zookeeper_amd.parallel.rccl import NativeComm

    t0 = time.monotonic()
    with pytest.raises(TimeoutError, match="did not return"):
        NativeComm(0, 1, tag="zk_hang", init_timeout_s=1, _make_uid=lambda: b"u" * 128,
                   _init=lambda u, w, r: time.sleep(60))
    assert time.monotonic() - t0 < 10

    c = NativeComm(0, 1, tag="zk_lock", _make_uid=lambda: b"u" * 128, _init=lambda u, w, r: 7)
    c._mu.acquire()  # this thread is "inside an enqueue"; the watchdog is another
    held = []
    th = threading.Thread(target=lambda: held.append(c._fail("stub expiry", grace_s=0.2)))
    th.start()
    th.join(10)
    assert held == [False]  # mutex held: no abort of a handle in use
    assert c._failed is None and c.handle == 7
    c._mu.release()
    done = []
    th = threading.Thread(target=lambda: done.append(c._fail("stub expiry", grace_s=5)))
    th.start()
    th.join(10)
    assert done == [True] and c.handle == 0
    assert not c._stop.is_set()
    with pytest.raises(RuntimeError, match="stub expiry"):
        c.check()
    assert c._stop.is_set()  # the training thread handles it: no hard exit
