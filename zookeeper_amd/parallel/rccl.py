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
"""

from __future__ import annotations

import ctypes
import glob
import os
from typing import Optional

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
    n-th communicator of a process gets tag n by default)."""

    def __init__(self, rank: int, world: int, store=None, tag: Optional[str] = None):
        from zookeeper_amd.ops._native import lib

        load()
        self.rank, self.world = int(rank), int(world)
        if tag is None:
            _COUNTER[0] += 1
            tag = f"zk_native_comm_{_COUNTER[0]}"
        if self.world == 1:
            uid = unique_id()
        else:
            store = store if store is not None else _store()
            if self.rank == 0:
                uid = unique_id()
                store.set(tag, uid)
            else:
                store.wait([tag])
                uid = store.get(tag)
        comm = ctypes.c_void_p()
        _check(lib().zk_comm_init(uid, self.world, self.rank, ctypes.byref(comm)),
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

        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("NativeComm.all_reduce_ needs a contiguous device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        _check(lib().zk_comm_all_reduce(self._comm, t.data_ptr(), t.data_ptr(), t.numel(),
                                        DTYPES[t.dtype], OPS[op], s.cuda_stream),
               "ncclAllReduce")
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, stream=None) -> torch.Tensor:
        from zookeeper_amd.ops._native import lib

        s = stream if stream is not None else torch.cuda.current_stream(t.device)
        _check(lib().zk_comm_broadcast(self._comm, t.data_ptr(), t.data_ptr(), t.numel(),
                                       DTYPES[t.dtype], int(root), s.cuda_stream),
               "ncclBroadcast")
        return t

    def close(self, abort: bool = False) -> None:
        from zookeeper_amd.ops._native import lib

        if self._comm:
            lib().zk_comm_destroy(self._comm, int(abort))
            self._comm = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass
