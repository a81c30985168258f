"""``Runtime``: the execution / kernel-selection switches of a run as typed,
configurable Fields.

The reference's premise is that everything a run depends on is injected
through ``Field``s and reproducible from the resolved config
(zookeeper/core/component.py:461-695).  The native training path has a
number of schedule and kernel-variant choices (side-stream weight gradients,
MX-FP4 forward, fused stem, tile rules, HIP-graph replay, deterministic
reductions, ...); they live here instead of in environment variables, so a
run can set them on the CLI (``runtime.bconv_fp4=False``), sweep them
(``--grid runtime.tile_huge=[0,16]``), and they are written into
``config.json`` and the bench JSON.

:meth:`Runtime.apply` pushes the kernel options into
:data:`zookeeper_amd.ops.options.OPTS` (and the native library); the trainer
reads the schedule options (``graph``, ``force_dp``, ``comm_timing``)
directly.
"""

from __future__ import annotations

import dataclasses
from typing import Any, Dict

from zookeeper_amd.core.component import component
from zookeeper_amd.core.field import Field
from zookeeper_amd.ops import options as _options

_KERNEL_FIELDS = tuple(f.name for f in dataclasses.fields(_options.KernelOptions))


@component
class Runtime:
    # --- kernel variants (ops/options.py documents each and its measurement)
    bconv_fp4: bool = Field(True)
    wgrad_side_stream: bool = Field(True)
    float_wgrad_side_stream: bool = Field(True)
    stem_fused: bool = Field(True)
    conv_mfma: bool = Field(True)
    conv3_mfma: bool = Field(True)
    pw_gemm: bool = Field(True)
    tile_huge: int = Field(48)
    dgrad_rw: bool = Field(True)
    bn_stats_epilogue: bool = Field(True)
    wgrad_slab_mb: int = Field(32)
    wgrad_rows: bool = Field(True)
    wgrad_fp4: bool = Field(True)
    dgrad_deep: int = Field(1)
    wgrad_deep: bool = Field(True)
    wgrad_tree: bool = Field(False)
    weight_images: bool = Field(True)
    bn_bwd_fuse: bool = Field(True)
    bn_masked_handoff: bool = Field(True)
    bn_pool_fuse: bool = Field(True)
    epilogue_prefetch: bool = Field(True)
    # Bit-reproducible gradients (fixed-order reductions, no float atomics on
    # the gradient path); slower.
    deterministic: bool = Field(False)

    # --- schedule
    # HIP-graph replay of forward + backward: "off", "on", or "auto" (replay
    # only if the warmup shows the step host-bound; decided on every rank
    # together under data parallelism).
    graph: str = Field("off")
    # Keep the bucketed all-reduce on even with one rank (a 1-rank RCCL
    # group): exercises the data-parallel path on a single GPU.
    force_dp: bool = Field(False)
    # Time every bucket's collective (comm_ms / exposed_ms in metrics.jsonl).
    comm_timing: bool = Field(True)
    # Run the preprocessing's device kernels (normalise + flip) on the
    # loader's copy stream after each H2D copy (Preprocessing.device_transform)
    # instead of at the head of the step on the compute stream.
    loader_preprocess: bool = Field(True)

    # --- data-parallel communicator (parallel/dist.py CommConfig documents each)
    # RCCL streams and the comm stream at high HIP priority.  Off by default:
    # no multi-GPU measurement shows it helps.  (The stale-gradient race once
    # blamed on it, profiles/r4/d_dp_stager_race.md, was the bucketer counting
    # autograd's hook call for directly written gradients:
    # profiles/r5/dp_hook_race.md; the two-rank GPU tests run at high priority.)
    comm_high_priority: bool = Field(False)
    # NCCL_MIN_NCHANNELS / NCCL_MAX_NCHANNELS (0: RCCL's default).
    rccl_min_channels: int = Field(0)
    rccl_max_channels: int = Field(0)
    # Pin each rank to its share of its GPU's NUMA-local CPUs.
    cpu_affinity: bool = Field(True)
    # Debug: compare the launched bucket order across ranks every step (with
    # the native communicator under graph replay: eager steps, plus the
    # captured order once after the capture -- every replay issues that).
    check_bucket_order: bool = Field(False)
    # Gradient all-reduce transport: "torch" (ProcessGroupNCCL), "native"
    # (parallel/rccl.py: the in-tree RCCL communicator; graph-capturable) or
    # "auto": native, falling back to torch on every rank if its set-up fails
    # on any.  Forced 1-rank RCCL, E18 b1536 (scripts/lease/gpu_call23.sh): torch
    # 34.56 ms/step vs native 30.06 vs 29.93 without data parallelism.
    comm_backend: str = Field("auto")

    def __post_configure__(self) -> None:
        if self.graph not in ("off", "on", "auto"):
            raise ValueError(f"runtime.graph must be 'off', 'on' or 'auto', got {self.graph!r}")
        if self.rccl_min_channels < 0 or self.rccl_max_channels < 0:
            raise ValueError("runtime.rccl_min_channels / rccl_max_channels must be >= 0")
        if 0 < self.rccl_max_channels < self.rccl_min_channels:
            raise ValueError("runtime.rccl_min_channels > rccl_max_channels")
        if self.comm_backend not in ("torch", "native", "auto"):
            raise ValueError(f"runtime.comm_backend must be 'torch', 'native' or 'auto', "
                             f"got {self.comm_backend!r}")

    def kernel_options(self) -> Dict[str, Any]:
        return {k: getattr(self, k) for k in _KERNEL_FIELDS}

    def apply(self) -> _options.KernelOptions:
        """Make these kernel options current (``ops.options.OPTS``)."""
        return _options.set_options(**self.kernel_options())

    def trainer_graph(self):
        return {"off": False, "on": True, "auto": "auto"}[self.graph]

    def comm_config(self):
        """The communicator set-up for ``zdist.init(comm=...)``."""
        from zookeeper_amd.parallel.dist import CommConfig

        return CommConfig(high_priority=self.comm_high_priority,
                          min_channels=self.rccl_min_channels,
                          max_channels=self.rccl_max_channels,
                          cpu_affinity=self.cpu_affinity,
                          check_bucket_order=self.check_bucket_order,
                          backend=self.comm_backend)

    def as_dict(self) -> Dict[str, Any]:
        d = self.kernel_options()
        d.update(graph=self.graph, force_dp=self.force_dp, comm_timing=self.comm_timing,
                 loader_preprocess=self.loader_preprocess,
                 comm_high_priority=self.comm_high_priority,
                 rccl_min_channels=self.rccl_min_channels,
                 rccl_max_channels=self.rccl_max_channels, cpu_affinity=self.cpu_affinity,
                 check_bucket_order=self.check_bucket_order, comm_backend=self.comm_backend)
        return d
