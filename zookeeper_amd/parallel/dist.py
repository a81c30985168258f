"""Process-group bootstrap: one process per GPU, ``torch.distributed`` env
contract (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``).

On ROCm the ``"nccl"`` backend *is* RCCL (xGMI transport inside a node);
``"gloo"`` is used on CPU (tests, rehearsals).  The reference has no
distributed layer at all (SURVEY §2.5–2.6).
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class CommConfig:
    """How the data-parallel communicator is set up (``Runtime`` fields
    ``comm_high_priority``, ``rccl_min_channels``, ``rccl_max_channels``,
    ``cpu_affinity``, ``check_bucket_order``).

    * ``high_priority``: RCCL's internal streams (``ProcessGroupNCCL.Options
      .is_high_priority_stream``) and the bucketer's comm stream are created
      at high HIP priority.  The E18 step keeps the compute stream ~99 % and
      the weight-gradient side stream ~50 % busy; at default priority the
      all-reduce kernels would wait for CU slots behind both, and a bucket
      finishing late is exposed time after backward;
    * ``min_channels`` / ``max_channels`` (0: RCCL's choice): written to
      ``NCCL_MIN_NCHANNELS`` / ``NCCL_MAX_NCHANNELS`` before the communicator
      exists.  Each channel is a workgroup resident on a CU for the whole
      collective; ≤10 MB buckets over xGMI need few channels, and fewer
      channels leave more CUs to the backward kernels;
    * ``cpu_affinity``: pin each rank to its share of the CPUs local to its
      GPU (``parallel/affinity.py``);
    * ``check_bucket_order``: debug -- every step all-reduces a hash of the
      launched bucket sequence (MAX and MIN) and raises if the ranks differ
      (a rank issuing collectives in another order deadlocks or corrupts RCCL);
    * ``backend``: ``"torch"`` -- the gradient all-reduce through
      ProcessGroupNCCL (RCCL behind work objects); ``"native"`` -- through the
      in-tree RCCL communicator (``parallel/rccl.py``), straight onto the comm
      stream, which also lets a HIP graph capture the collectives.
    """

    high_priority: bool = False
    min_channels: int = 0
    max_channels: int = 0
    cpu_affinity: bool = True
    check_bucket_order: bool = False
    backend: str = "torch"


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    comm: CommConfig = field(default_factory=CommConfig)
    cpus: Optional[List[int]] = None  # the CPU affinity set at init (None: untouched)
    rccl_env: dict = field(default_factory=dict)  # NCCL_* knobs in effect at init

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world > 1


_INFO = DistInfo()


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


_RCCL_KEYS = ("NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS")


def apply_rccl_env(comm: CommConfig, env=None) -> dict:
    """Write the channel knobs into the environment (before the communicator
    is created; RCCL reads them at init) and return the ``NCCL_*`` values in
    effect.  0 leaves RCCL's own choice (or a value the user exported)."""
    env = os.environ if env is None else env
    if comm.min_channels > 0:
        env["NCCL_MIN_NCHANNELS"] = str(int(comm.min_channels))
    if comm.max_channels > 0:
        env["NCCL_MAX_NCHANNELS"] = str(int(comm.max_channels))
    if comm.min_channels > 0 and comm.max_channels > 0 and comm.min_channels > comm.max_channels:
        raise ValueError(f"rccl_min_channels {comm.min_channels} > rccl_max_channels "
                         f"{comm.max_channels}")
    return {k: env[k] for k in _RCCL_KEYS if k in env}


def _pg_options(backend: str, comm: CommConfig):
    if backend != "nccl" or not comm.high_priority:
        return None
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def init(backend: str = "auto", timeout_s: float = 600.0, single_group: bool = False,
         comm: Optional[CommConfig] = None) -> DistInfo:
    """Initialise (once) and return the rank / device binding.

    ``comm``: communicator set-up (:class:`CommConfig`; defaults if None):
    CPU affinity is applied first (sysfs + ``sched_setaffinity`` only, before
    any thread of the input pipeline or RCCL exists), then the ``NCCL_*``
    channel knobs, then the process group with high-priority RCCL streams.

    ``single_group``: also create a process group when the job has one rank
    (``force_dp``: a 1-rank RCCL communicator, so the bucketed all-reduce
    path runs on one GPU exactly as it does on eight).

    ``timeout_s`` (overridden by ``ZK_DIST_TIMEOUT_S``) bounds every
    collective: a rank that dies or hangs makes the others' collectives raise
    after it instead of blocking forever, and the launcher then tears the job
    down (failure detection)."""
    timeout_s = float(os.environ.get("ZK_DIST_TIMEOUT_S", timeout_s))
    comm = comm or CommConfig()
    # enough hardware queues for the step's streams (devices.py: effective
    # when this runs before the first GPU use, as in bench.py / Experiment)
    from zookeeper_amd.parallel.devices import configure_hw_queues

    configure_hw_queues()
    global _INFO
    if _INFO.backend != "none" or (dist.is_available() and dist.is_initialized()):
        return _INFO
    rank = int(os.environ.get("RANK", "0"))
    world = env_world()
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    cpus = None
    # a GPU job binds to its GPU's NUMA-local CPUs (gloo CPU rehearsals have
    # no GPU to be local to); device_count goes through amdsmi, not a HIP init
    if comm.cpu_affinity and torch.cuda.device_count() > 0:
        from zookeeper_amd.parallel import affinity

        cpus = affinity.apply(local, int(os.environ.get("LOCAL_WORLD_SIZE", str(world))))
    rccl_env = apply_rccl_env(comm)
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
            opts = _pg_options(backend, comm)
            if opts is not None:
                kwargs["pg_options"] = opts
        dist.init_process_group(**kwargs)
    grouped = world > 1 or single_group
    _INFO = DistInfo(rank, world, local, device, backend if grouped else "none", comm, cpus,
                     rccl_env)
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
