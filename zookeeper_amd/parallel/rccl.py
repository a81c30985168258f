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
  process (exit code 3) after a grace period;
* ``ncclCommInitRank`` runs under its own deadline (``init_timeout_s``) in a
  helper thread, so a rank whose peers never finish their init does not hang;
* every use of the handle (enqueue, abort, destroy) holds one mutex, so the
  watchdog's abort never frees a handle the training thread is using;
* :func:`connect` is the set-up the trainer uses: RCCL loaded and rank 0's
  unique id made on every rank, then the rendezvous + init + a canary
  all-reduce of rank-coded values checked against the exact sum -- each
  phase agreed through the store, so with ``fallback`` every rank returns
  ``None`` together (ProcessGroupNCCL takes over) and none is left waiting.
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


def default_init_timeout() -> float:
    """Deadline of ``ncclCommInitRank`` and of the set-up canary
    (``ZK_COMM_INIT_TIMEOUT_S``, default 120 s; an 8-rank init takes seconds)."""
    return float(os.environ.get("ZK_COMM_INIT_TIMEOUT_S", "120"))


def next_tag() -> str:
    """The n-th communicator of a process: the same tag on every rank."""
    _COUNTER[0] += 1
    return f"zk_native_comm_{_COUNTER[0]}"


def call_with_deadline(fn: Callable[[], object], timeout_s: float, what: str):
    """``fn()`` in a daemon helper thread; ``TimeoutError`` if it has not
    returned within ``timeout_s`` (the thread is left behind: a blocking RCCL
    call cannot be interrupted from outside)."""
    box: dict = {}

    def run():
        try:
            box["value"] = fn()
        except BaseException as e:  # noqa: BLE001 -- re-raised in the caller
            box["error"] = e

    t = threading.Thread(target=run, daemon=True, name="zk-comm-init")
    t.start()
    t.join(timeout_s)
    if t.is_alive():
        raise TimeoutError(f"{what} did not return within {timeout_s:.0f} s")
    if "error" in box:
        raise box["error"]
    return box["value"]


def agree(store, key: str, rank: int, world: int, ok: bool, timeout_s: float) -> bool:
    """Every rank votes ``ok`` under ``key``; True iff all voted yes.  A
    store, not a collective: no rank can be left inside a GPU collective the
    others never issue.  Raises ``TimeoutError`` if a rank never votes."""
    if world == 1:
        return bool(ok)
    store.set(f"{key}/{rank}", b"1" if ok else b"0")
    keys = [f"{key}/{r}" for r in range(world)]
    try:
        store.wait(keys, timedelta(seconds=timeout_s))
    except Exception as e:  # noqa: BLE001
        missing = [r for r in range(world) if not store.check([f"{key}/{r}"])]
        raise TimeoutError(f"{key!r}: rank(s) {missing} did not vote within "
                           f"{timeout_s:.0f} s ({e})") from None
    return all(store.get(k) == b"1" for k in keys)


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
                 timeout_s: Optional[float] = None, init_timeout_s: Optional[float] = None,
                 _make_uid: Optional[Callable[[], bytes]] = None,
                 _init: Optional[Callable[[bytes, int, int], int]] = None):
        self.rank, self.world = int(rank), int(world)
        self.timeout_s = float(timeout_s if timeout_s is not None else default_timeout())
        self.init_timeout_s = float(init_timeout_s if init_timeout_s is not None
                                    else default_init_timeout())
        if tag is None:
            tag = next_tag()
        self.tag = tag
        self._comm = ctypes.c_void_p()
        # one mutex over every use of the handle: enqueue (training thread),
        # abort (watchdog), destroy (close)
        self._mu = threading.RLock()
        self._failed: Optional[str] = None
        self._watch: List[Tuple[object, float]] = []
        self._watch_mu = threading.Lock()
        self._watchdog: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._owned = _init is None  # a stubbed handle is never destroyed
        if _make_uid is None:
            load()
            _make_uid = unique_id
        if self.world == 1:
            self.uid = _make_uid()
        else:
            store = store if store is not None else _store()
            self.uid = exchange_unique_id(store, tag, self.rank, self.world, _make_uid,
                                          self.timeout_s)
        if _init is not None:
            handle = call_with_deadline(lambda: _init(self.uid, self.world, self.rank),
                                        self.init_timeout_s,
                                        f"communicator {tag!r} init (rank {self.rank})")
            self._comm = ctypes.c_void_p(handle)
            return
        from zookeeper_amd.ops._native import lib

        dev = torch.cuda.current_device()
        abandoned = threading.Event()

        def init() -> int:
            # the helper thread's current HIP device is the communicator's
            torch.cuda.set_device(dev)
            comm = ctypes.c_void_p()
            rc = lib().zk_comm_init(self.uid, self.world, self.rank, ctypes.byref(comm))
            if rc == 0 and abandoned.is_set():
                # the deadline passed while the peers were still joining: this
                # communicator has no owner, release it
                lib().zk_comm_destroy(comm, 1)
            _check(rc, "ncclCommInitRank")
            return comm.value

        try:
            handle = call_with_deadline(init, self.init_timeout_s,
                                        f"ncclCommInitRank of {tag!r} (rank {self.rank}/"
                                        f"{self.world})")
        except TimeoutError:
            abandoned.set()
            raise
        self._comm = ctypes.c_void_p(handle)
        n = ctypes.c_int(0)
        _check(lib().zk_comm_count(self._comm, ctypes.byref(n)), "ncclCommCount")
        if n.value != self.world:
            raise RuntimeError(f"RCCL communicator has {n.value} ranks, expected {self.world}")

    @property
    def handle(self) -> int:
        return self._comm.value or 0

    def _live_handle(self) -> ctypes.c_void_p:
        """The handle, under ``_mu`` (held by the caller)."""
        self.check()
        if not self._comm:
            raise RuntimeError(f"native communicator {self.tag!r} is closed")
        return self._comm

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        """In place, on ``stream`` (default: the current HIP stream)."""
        from zookeeper_amd.ops._native import lib

        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm.all_reduce_ needs a contiguous device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        with self._mu:
            _check(lib().zk_comm_all_reduce(self._live_handle(), t.data_ptr(), t.data_ptr(),
                                            t.numel(), DTYPES[t.dtype], OPS[op], s.cuda_stream),
                   "ncclAllReduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        from zookeeper_amd.ops._native import lib

        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm.broadcast_ needs a contiguous device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        with self._mu:
            _check(lib().zk_comm_broadcast(self._live_handle(), t.data_ptr(), t.data_ptr(),
                                           t.numel(), DTYPES[t.dtype], int(root), s.cuda_stream),
                   "ncclBroadcast")
        return t

    def canary(self, timeout_s: Optional[float] = None) -> None:
        """Set-up check: all-reduce ``rank + 1`` on a private stream and
        require the exact sum ``world (world + 1) / 2`` within ``timeout_s``
        (default: the init deadline).  A timeout aborts the communicator."""
        timeout_s = self.init_timeout_s if timeout_s is None else float(timeout_s)
        dev = torch.device("cuda", torch.cuda.current_device())
        t = torch.full((256,), float(self.rank + 1), dtype=torch.float32, device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        self.all_reduce_(t, stream=s)
        done = torch.cuda.Event()
        done.record(s)
        deadline = time.monotonic() + timeout_s
        while not done.query():
            if time.monotonic() > deadline:
                self._fail(f"set-up canary all-reduce did not complete within {timeout_s:.0f} s")
                raise TimeoutError(self._failed)
            time.sleep(0.002)
        want = float(self.world * (self.world + 1) // 2)
        got = t.cpu()
        if not bool(torch.all(got == want)):
            raise RuntimeError(f"native communicator {self.tag!r}: canary all-reduce gave "
                               f"{got[:4].tolist()}..., expected {want}")

    # -- failure detection --------------------------------------------------- #

    def async_error(self) -> int:
        """``ncclCommGetAsyncError`` (0: none; -2: not provided by this RCCL)."""
        from zookeeper_amd.ops._native import lib

        with self._mu:
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
        """Raise if the watchdog found a collective past its deadline.  The
        raise hands the failure to the training thread (it is not blocked):
        the watchdog's hard-exit grace period is cancelled."""
        if self._failed is not None:
            self._stop.set()
            raise RuntimeError(self._failed)

    def _fail(self, what: str, grace_s: float = 30.0) -> bool:
        """Record the failure and abort the communicator under ``_mu``.
        False if the mutex could not be taken within ``grace_s`` (the
        training thread is blocked inside an RCCL enqueue on this handle)."""
        if not self._mu.acquire(timeout=grace_s):
            return False
        try:
            if self._failed is None:
                code = 0
                if self._comm and getattr(self, "_owned", True):
                    from zookeeper_amd.ops._native import lib

                    err = ctypes.c_int(0)
                    rc = lib().zk_comm_async_error(self._comm, ctypes.byref(err))
                    code = err.value if rc == 0 else rc
                self._failed = (f"native communicator {self.tag!r} (rank {self.rank}/"
                                f"{self.world}): {what} (ncclCommGetAsyncError = {code}); "
                                "communicator aborted")
            self._destroy(abort=True)
        finally:
            self._mu.release()
        return True

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
                aborted = self._fail(f"{expired} did not complete within {self.timeout_s:.0f} s",
                                     grace_s)
                print(f"[zk] {self._failed or expired}", file=sys.stderr, flush=True)
                # the training thread raises at its next check() (which sets
                # _stop); if it is stuck in a device synchronisation the abort
                # did not release -- or in an enqueue holding the handle's
                # mutex -- end the process
                if not aborted or not self._stop.wait(grace_s):
                    print("[zk] training thread still blocked after the abort: exiting",
                          file=sys.stderr, flush=True)
                    os._exit(3)
                return
            self._stop.wait(poll_s)

    def _destroy(self, abort: bool) -> None:
        with self._mu:
            if self._comm:
                if getattr(self, "_owned", True):
                    from zookeeper_amd.ops._native import lib

                    lib().zk_comm_destroy(self._comm, int(abort))
                self._comm = ctypes.c_void_p()

    def close(self, abort: bool = False) -> None:
        self._destroy(abort)
        self._stop.set()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self._stop.set()
            self.close()
        except Exception:
            pass


def connect(rank: int, world: int, store=None, fallback: bool = True,
            timeout_s: Optional[float] = None, init_timeout_s: Optional[float] = None,
            tag: Optional[str] = None, log: Optional[Callable[[str], None]] = None,
            _load: Optional[Callable[[], None]] = None,
            _make_uid: Optional[Callable[[], bytes]] = None,
            _init: Optional[Callable[[bytes, int, int], int]] = None,
            _canary: Optional[Callable[["NativeComm"], None]] = None) -> Optional["NativeComm"]:
    """Set up the native communicator on every rank together.

    Phase 1: every rank loads RCCL, rank 0 also makes the unique id; the ranks
    vote through the store.  Phase 2: rendezvous, ``ncclCommInitRank`` under
    ``init_timeout_s`` and the canary all-reduce (:meth:`NativeComm.canary`);
    the ranks vote again.  A "no" in either vote returns ``None`` on EVERY
    rank (``fallback``; the caller then uses ProcessGroupNCCL), after
    aborting any communicator this rank built; without ``fallback`` it
    raises.  The votes go through the store, so a failure on one rank costs
    the others one store round trip, not the rendezvous timeout.

    ``_load`` / ``_make_uid`` / ``_init`` / ``_canary`` replace the RCCL calls
    (CPU tests of the agreement, ``tests/test_native_comm_cpu.py``)."""
    timeout_s = float(timeout_s if timeout_s is not None else default_timeout())
    init_timeout_s = float(init_timeout_s if init_timeout_s is not None
                           else default_init_timeout())
    tag = tag or next_tag()
    if world > 1 and store is None:
        store = _store()
    say = log or (lambda msg: print(msg, file=sys.stderr, flush=True))

    def give_up(phase: str, err) -> None:
        msg = (f"[zk] native communicator {tag!r}: {phase} failed on some rank "
               f"({err!r} on rank {rank})")
        if not fallback:
            raise RuntimeError(msg) from (err if isinstance(err, BaseException) else None)
        if rank == 0 or err is not None:
            say(msg + "; gradient all-reduce through ProcessGroupNCCL")

    # phase 1: RCCL on every rank, the unique id on rank 0
    err, uid = None, None
    try:
        (_load or load)()
        if rank == 0:
            uid = (_make_uid or unique_id)()
    except Exception as e:  # noqa: BLE001 -- any failure is a "no" vote
        err = e
    if not agree(store, f"{tag}/vote/load", rank, world, err is None, timeout_s):
        give_up("RCCL load / unique id", err)
        return None

    # phase 2: rendezvous + init + canary
    comm = None
    try:
        comm = NativeComm(rank, world, store=store, tag=tag, timeout_s=timeout_s,
                          init_timeout_s=init_timeout_s,
                          _make_uid=(lambda: uid) if rank == 0 else (lambda: b""),
                          _init=_init)
        (_canary or NativeComm.canary)(comm)
    except Exception as e:  # noqa: BLE001
        err = e
    if not agree(store, f"{tag}/vote/ready", rank, world, err is None, timeout_s):
        if comm is not None:
            comm.close(abort=True)
        give_up("init / canary", err)
        return None
    return comm
