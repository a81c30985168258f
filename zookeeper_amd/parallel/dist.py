"""Process-group bootstrap: one process per GPU, ``torch.distributed`` env
contract (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``).

On ROCm the ``"nccl"`` backend *is* RCCL (xGMI transport inside a node);
``"gloo"`` is used on CPU (tests, rehearsals).  The reference has no
distributed layer at all (SURVEY §2.5–2.6).
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


_INFO = DistInfo()


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: str = "auto", timeout_s: float = 600.0, single_group: bool = False) -> DistInfo:
    """Initialise (once) and return the rank / device binding.

    ``single_group``: also create a process group when the job has one rank
    (``force_dp``: a 1-rank RCCL communicator, so the bucketed all-reduce
    path runs on one GPU exactly as it does on eight).

    ``timeout_s`` (overridden by ``ZK_DIST_TIMEOUT_S``) bounds every
    collective: a rank that dies or hangs makes the others' collectives raise
    after it instead of blocking forever, and the launcher then tears the job
    down (failure detection)."""
    timeout_s = float(os.environ.get("ZK_DIST_TIMEOUT_S", timeout_s))
    global _INFO
    if _INFO.backend != "none" or (dist.is_available() and dist.is_initialized()):
        return _INFO
    rank = int(os.environ.get("RANK", "0"))
    world = env_world()
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local % torch.cuda.device_count())
        device = torch.device("cuda", torch.cuda.current_device())
    else:
        device = torch.device("cpu")
    if backend == "auto":
        # ZK_DIST_BACKEND=gloo rehearses a multi-rank GPU run with several
        # ranks sharing one GPU (RCCL wants a distinct GPU per rank)
        backend = os.environ.get("ZK_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if world > 1 or single_group:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            from zookeeper_amd.parallel.launch import free_port

            os.environ["MASTER_PORT"] = str(free_port())
        os.environ.setdefault("MASTER_PORT", "29500")
        kwargs = dict(backend=backend, rank=rank, world_size=world,
                      timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = device
        dist.init_process_group(**kwargs)
    grouped = world > 1 or single_group
    _INFO = DistInfo(rank, world, local, device, backend if grouped else "none")
    return _INFO


def info() -> DistInfo:
    return _INFO


def barrier() -> None:
    if _INFO.world > 1:
        if _INFO.backend == "nccl":
            dist.barrier(device_ids=[_INFO.device.index])
        else:
            dist.barrier()


def all_reduce_max(value: float) -> float:
    if _INFO.world == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64,
                     device=_INFO.device if _INFO.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_max_values(values, device=None):
    """Element-wise MAX of a few floats over the ranks of the default group
    (every rank gets the same list back).  Uses a device tensor for RCCL and
    a host tensor otherwise; a no-op without a process group."""
    values = [float(v) for v in values]
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return values
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor(values, dtype=torch.float64,
                     device=(device if device is not None else _INFO.device) if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    if _INFO.world > 1:
        dist.all_reduce(t)
        t.div_(_INFO.world)
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if _INFO.world > 1:
        dist.broadcast(t, src)
    return t


def shutdown() -> None:
    global _INFO
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _INFO = DistInfo()
