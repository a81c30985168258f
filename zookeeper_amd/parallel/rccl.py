"""Native RCCL communicator: the C ABI of ``csrc/runtime/comm.cpp`` bound for
the data-parallel gradient all-reduce.

ProcessGroupNCCL issues each collective on an internal stream behind work
objects; a HIP graph can neither capture those nor order them with the
kernels that produce the gradients.  :class:`NativeComm` issues
``ncclAllReduce`` straight onto the caller's HIP stream, so

* the bucketer's comm stream orders the collectives with plain events, and
* under ``Trainer(graph=True)`` the collectives are captured into the same
  graph as the backward kernels (``runtime.comm_backend="native"``): graph
  replay keeps the all-reduce overlapped with backward instead of issuing
  every bucket after the replay.

RCCL itself is not linked into ``_zkamd.so``: the library torch bundles (and
ProcessGroupNCCL already loaded) is opened by path, so the process never
holds two RCCLs.  The 128-byte unique id goes from rank 0 to the others
through the torch store of the default process group (or a ``TCPStore`` on
``MASTER_ADDR:MASTER_PORT``).

Failure detection:

* set-up is a store rendezvous with a deadline (``timeout_s``, default
  ``ZK_DIST_TIMEOUT_S`` or 600 s): every rank posts a ready key and waits for
  all of them and for rank 0's unique id, so a missing peer raises
  ``TimeoutError`` instead of hanging inside ``ncclCommInitRank``;
* a watchdog thread follows every step's collectives through an event on the
  comm stream (:meth:`NativeComm.watch`): past the deadline it reads
  ``ncclCommGetAsyncError``, aborts the communicator (``ncclCommAbort``: the
  collective kernels stop waiting for the peer) and records the failure;
  :meth:`NativeComm.check` (called by the bucketer every step) raises it in
  the training thread -- a non-zero exit the launcher's fail-fast turns into
  the end of every rank.  If the training thread is itself stuck in a device
  synchronisation that the abort does not release, the watchdog ends the
  process (exit code 3) after a grace period.
"""

from __future__ import annotations

import ctypes
import glob
import os
import sys
import threading
import time
from datetime import timedelta
from typing import Callable, List, Optional, Tuple

import torch

# rccl.h enums (NCCL 2.x ABI)
DTYPES = {torch.float32: 7, torch.bfloat16: 9, torch.float16: 6, torch.float64: 8,
          torch.int32: 2, torch.int64: 4}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}

_COUNTER = [0]


def rccl_path() -> Optional[str]:
    """torch's bundled librccl (the RCCL ProcessGroupNCCL uses)."""
    cands = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so*"))
    return sorted(cands)[0] if cands else None


def load() -> None:
    """Resolve RCCL's entry points in the native library (idempotent)."""
    from zookeeper_amd.ops._native import lib

    L = lib()
    if L.zk_comm_loaded():
        return
    path = rccl_path()
    if path is None:
        raise RuntimeError("no librccl.so next to torch: the native communicator needs RCCL")
    rc = L.zk_comm_load(path.encode())
    if rc != 0:
        raise RuntimeError(f"zk_comm_load({path}) failed with {rc} "
                           "(1: dlopen failed, 2: RCCL symbol missing)")


def error_string(code: int) -> str:
    from zookeeper_amd.ops._native import lib

    fn = lib().zk_comm_error_string
    fn.restype = ctypes.c_char_p
    fn.argtypes = [ctypes.c_int]
    s = fn(int(code))
    return s.decode() if s else ""


def _check(code: int, what: str) -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed: RCCL {code} ({error_string(code) if code > 0 else ''})")


def unique_id() -> bytes:
    from zookeeper_amd.ops._native import lib

    load()
    buf = ctypes.create_string_buffer(128)
    _check(lib().zk_comm_unique_id(buf), "ncclGetUniqueId")
    return buf.raw


def default_timeout() -> float:
    return float(os.environ.get("ZK_DIST_TIMEOUT_S", "600"))


def exchange_unique_id(store, tag: str, rank: int, world: int, make_uid: Callable[[], bytes],
                       timeout_s: float) -> bytes:
    """Store rendezvous of one communicator: rank 0 publishes a new unique id
    under ``tag``; every rank posts ``tag/ready/<rank>`` and waits (at most
    ``timeout_s``) for all ``world`` ready keys and the id.  Raises
    ``TimeoutError`` naming the ranks that did not arrive."""
    if rank == 0:
        store.set(tag, make_uid())
    store.set(f"{tag}/ready/{rank}", b"1")
    keys = [tag] + [f"{tag}/ready/{r}" for r in range(world)]
    try:
        store.wait(keys, timedelta(seconds=timeout_s))
    except Exception as e:  # torch raises DistStoreError / RuntimeError on timeout
        missing = [r for r in range(world) if not store.check([f"{tag}/ready/{r}"])]
        raise TimeoutError(f"native communicator {tag!r}: rank(s) {missing} did not join "
                           f"within {timeout_s:.0f} s ({e})") from None
    return store.get(tag)


def _store():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        return dist.distributed_c10d._get_default_store()
    from datetime import timedelta

    return dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"),
                         int(os.environ.get("MASTER_PORT", "29500")),
                         int(os.environ.get("WORLD_SIZE", "1")),
                         int(os.environ.get("RANK", "0")) == 0, timedelta(seconds=600))


class NativeComm:
    """An RCCL communicator over ``world`` ranks on the current HIP device.

    Collective construction: every rank creates it with the same ``tag`` (the
    n-th communicator of a process gets tag n by default).  ``timeout_s``
    bounds the set-up rendezvous and every step's collectives (watchdog).
    ``_make_uid`` / ``_init`` replace ``ncclGetUniqueId`` /
    ``ncclCommInitRank`` (tests of the rendezvous without RCCL)."""

    def __init__(self, rank: int, world: int, store=None, tag: Optional[str] = None,
                 timeout_s: Optional[float] = None,
                 _make_uid: Optional[Callable[[], bytes]] = None,
                 _init: Optional[Callable[[bytes, int, int], int]] = None):
        self.rank, self.world = int(rank), int(world)
        self.timeout_s = float(timeout_s if timeout_s is not None else default_timeout())
        if tag is None:
            _COUNTER[0] += 1
            tag = f"zk_native_comm_{_COUNTER[0]}"
        self.tag = tag
        self._comm = ctypes.c_void_p()
        self._failed: Optional[str] = None
        self._watch: List[Tuple[object, float]] = []
        self._watch_mu = threading.Lock()
        self._watchdog: Optional[threading.Thread] = None
        self._stop = threading.Event()
        if _make_uid is None:
            load()
            _make_uid = unique_id
        if self.world == 1:
            self.uid = _make_uid()
        else:
            store = store if store is not None else _store()
            self.uid = exchange_unique_id(store, tag, self.rank, self.world, _make_uid,
                                          self.timeout_s)
        self._owned = _init is None  # a stubbed handle is never destroyed
        if _init is not None:
            self._comm = ctypes.c_void_p(_init(self.uid, self.world, self.rank))
            return
        from zookeeper_amd.ops._native import lib

        comm = ctypes.c_void_p()
        _check(lib().zk_comm_init(self.uid, self.world, self.rank, ctypes.byref(comm)),
               "ncclCommInitRank")
        self._comm = comm
        n = ctypes.c_int(0)
        _check(lib().zk_comm_count(self._comm, ctypes.byref(n)), "ncclCommCount")
        if n.value != self.world:
            raise RuntimeError(f"RCCL communicator has {n.value} ranks, expected {self.world}")

    @property
    def handle(self) -> int:
        return self._comm.value or 0

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        """In place, on ``stream`` (default: the current HIP stream)."""
        from zookeeper_amd.ops._native import lib

        self.check()
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm.all_reduce_ needs a contiguous device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        _check(lib().zk_comm_all_reduce(self._comm, t.data_ptr(), t.data_ptr(), t.numel(),
                                        DTYPES[t.dtype], OPS[op], s.cuda_stream),
               "ncclAllReduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        from zookeeper_amd.ops._native import lib

        self.check()
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm.broadcast_ needs a contiguous device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        _check(lib().zk_comm_broadcast(self._comm, t.data_ptr(), t.data_ptr(), t.numel(),
                                       DTYPES[t.dtype], int(root), s.cuda_stream),
               "ncclBroadcast")
        return t

    # -- failure detection --------------------------------------------------- #

    def async_error(self) -> int:
        """``ncclCommGetAsyncError`` (0: none; -2: not provided by this RCCL)."""
        from zookeeper_amd.ops._native import lib

        if not self._comm or not getattr(self, "_owned", True):
            return 0
        err = ctypes.c_int(0)
        rc = lib().zk_comm_async_error(self._comm, ctypes.byref(err))
        return err.value if rc == 0 else rc

    def watch(self, event, what: str = "collectives") -> None:
        """Follow ``event`` (recorded on the stream after this step's
        collectives): if it has not completed within ``timeout_s``, the
        watchdog aborts the communicator and the next :meth:`check` raises."""
        with self._watch_mu:
            self._watch.append((event, time.monotonic() + self.timeout_s, what))
        if self._watchdog is None:
            self._watchdog = threading.Thread(target=self._run_watchdog, daemon=True,
                                              name=f"zk-comm-watchdog-{self.tag}")
            self._watchdog.start()

    def check(self) -> None:
        """Raise if the watchdog found a collective past its deadline."""
        if self._failed is not None:
            raise RuntimeError(self._failed)

    def _run_watchdog(self, poll_s: float = 0.05, grace_s: float = 30.0) -> None:
        while not self._stop.is_set():
            now = time.monotonic()
            expired = None
            with self._watch_mu:
                keep = []
                for ev, deadline, what in self._watch:
                    if ev.query():
                        continue
                    if now > deadline and expired is None:
                        expired = what
                    keep.append((ev, deadline, what))
                self._watch = keep
            if expired is not None:
                code = self.async_error()
                self._failed = (f"native communicator {self.tag!r} (rank {self.rank}/{self.world}): "
                                f"{expired} did not complete within {self.timeout_s:.0f} s "
                                f"(ncclCommGetAsyncError = {code}); communicator aborted")
                print(f"[zk] {self._failed}", file=sys.stderr, flush=True)
                self.close(abort=True)
                # the training thread raises at its next check(); if it is stuck in a
                # device synchronisation the abort did not release, end the process
                if not self._stop.wait(grace_s):
                    print("[zk] training thread still blocked after the abort: exiting",
                          file=sys.stderr, flush=True)
                    os._exit(3)
                return
            self._stop.wait(poll_s)

    def close(self, abort: bool = False) -> None:
        if self._comm:
            if getattr(self, "_owned", True):
                from zookeeper_amd.ops._native import lib

                lib().zk_comm_destroy(self._comm, int(abort))
            self._comm = ctypes.c_void_p()
        if not abort:
            self._stop.set()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self._stop.set()
            self.close()
        except Exception:
            pass
