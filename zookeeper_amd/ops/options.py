"""Kernel-selection options of the native training path, in one place.

Every switch that picks between kernel variants or execution schedules lives
here as an attribute of :data:`OPTS`, read by the ops **at call time** (not at
import time), so a run can change them before its first step.  They are set
from typed config through the :class:`~zookeeper_amd.train.runtime.Runtime`
component (``runtime.bconv_fp4=False`` on the CLI, sweepable with ``--grid``,
written into ``config.json`` and the bench JSON) — no environment variables.

The native library keeps its own copy of the options it consults on the host
side of a launch (tile rules, K-step order, deterministic reductions); it is
pushed through ``zk_set_option`` whenever :func:`set_options` runs.

Defaults are the measured winners (README "Round-2 measurements that decided
defaults").  Variants that measured slower everywhere were deleted, with
their measurements kept in ``profiles/`` (``profiles/r4/removed_variants.md``).
"""

from __future__ import annotations

import dataclasses
from typing import Any, Dict


@dataclasses.dataclass
class KernelOptions:
    # Binary forward on MX-FP4 MFMA (4x the bf16 rate); False selects the
    # bf16 MFMA form (same exact integer outputs).
    bconv_fp4: bool = True
    # Binary-conv weight gradients on a side HIP stream (44.9k vs 41.7k off).
    wgrad_side_stream: bool = True
    # ... and the float 1x1 / 3x3 convs' (ResNet): MFMA-bound weight
    # gradients next to the memory-bound BN passes (ops.streams.side_wgrad).
    float_wgrad_side_stream: bool = True
    # Recompute-fused ImageNet stem (False: the materialising kernels).
    stem_fused: bool = True
    # Float convolutions on the MFMA implicit-GEMM kernels (False: library).
    conv_mfma: bool = True
    conv3_mfma: bool = True
    # 1x1 float convolutions as MFMA GEMMs.
    pw_gemm: bool = True
    # Batch >= 1024 tile-rule bitmask (igemm.hip, see tile_rule comments).
    tile_huge: int = 48
    # Bit-reproducible gradients: split-K weight gradients reduced from slabs
    # in a fixed order, BN / bias sums without float atomics.
    deterministic: bool = False
    # Row-window data gradient for the 64 -> 64 stride-1 3x3 binary conv
    # (conv3rw.hip: resident weights, LDS ring of dY rows).
    dgrad_rw: bool = True
    # Float conv GEMMs with the LDS epilogue also sum the next BatchNorm's
    # batch statistics (pointwise.forward_with_stats; no statistics pass).
    bn_stats_epilogue: bool = True
    # Cap (MB) on one weight gradient's split-K slabs (fewer splits for the
    # deep 3x3 layers, whose slabs reached ~130 MB of writes + reads; the
    # side stream then also holds fewer CUs); 0 = no cap.  E18, 100 steps:
    # batch 1024 46.6k -> 47.6k, batch 1536 47.7k -> 48.4k img/s (16 MB:
    # 38k, too few splits for the 512-channel layers; 48/64 MB: 48.5k).
    # Same-box sweep at batch 1536: 28 MB 47.52k, 32 MB 47.79k / 47.71k,
    # 36 MB 47.17k, 40 MB 47.46k img/s.
    wgrad_slab_mb: int = 32
    # Row-streaming weight gradient for the 3x3 stride-1 layers it takes
    # (wgrad_rows.hip: every dY / S row loaded once per block, split-K summed
    # inside the launch by a fixed-order tree; 64 / 128-channel stages).
    wgrad_rows: bool = True
    # ... reading the e2m1 (FP4) sign image the binary forward already has
    # (expanded to bf16 in LDS): producers then skip the bf16 sign image of
    # tensors whose consumer takes this path (bconv_fp4 forward only).
    wgrad_fp4: bool = True
    # Phased data-gradient kernel (deep_gemm.hip) for the stride-1 3x3
    # convs with >= 256 input channels: 1 = float convs only, 2 = the binary
    # (STE-mask) ones too, 0 = never.  Same box, 2 rounds: QuickNet-Large
    # b1024 28.19k / 28.15k (1) vs 28.01k / 27.96k (2); E18 b1536 50.67k /
    # 50.77k (1) vs 50.82k / 50.87k (2).
    dgrad_deep: int = 1
    # ... and weight-gradient kernel for the stride-1 3x3 convs with >= 256
    # input and output channels.  Exempt from wgrad_slab_mb: its 256x256 dW
    # tiles leave (Cout/256)(Cin/256)*9 tiles per split, so the cap would cut
    # a 14x14x256 layer from 57 splits (513 blocks) to 13 (117 blocks, under
    # half the CUs).  Peak slab at batch 1536: ~134 MB (14x14x256, 57 x
    # 2.36 MB) and ~141 MB (7x7x512, 15 x 9.4 MB), freed after the layer.
    wgrad_deep: bool = True
    # Split-K of the igemm / deep weight gradients combined inside the launch
    # by a fixed-order tree (splitk_tree.h) instead of per-split slabs and a
    # streaming reduce launch.  Both are bit-reproducible.  Off: same-box E18
    # b1536 pairs 54.05k / 54.30k (reduce launch) vs 53.55k / 53.66k img/s
    # (tree) -- profiles/r6/wgrad_tree.md.
    wgrad_tree: bool = False
    # Float BatchNorm backward sums (sum g, sum g*xhat) added up in the data-
    # gradient epilogue of the 1x1 conv that consumes the BN output (when that
    # epilogue writes the BN output's whole gradient) instead of a separate
    # reduction pass over g and x (outside the deterministic mode).
    bn_bwd_fuse: bool = True
    # The BN tail hands (g, ReLU mask bits) to a 1x1 conv whose epilogue masks
    # and adds them, instead of writing the residual gradient g * mask.
    bn_masked_handoff: bool = True
    # A binary block whose output the next block's shortcut average-pools
    # writes the pooled image in its BN-apply pass (ops.binary_block pool_out)
    # instead of a separate pooling pass over the output.
    bn_pool_fuse: bool = True
    # The LDS-epilogue data gradient prefetches its residual / BN-input loads
    # in groups (igemm.hip dgrad_store_lds) instead of loading at each chunk.
    epilogue_prefetch: bool = True
    # Float conv weights as persistent bf16 GEMM-layout images written by the
    # fused optimizer (ops/weight_images.py) instead of a cast / transpose
    # per conv and pass.
    weight_images: bool = True


OPTS = KernelOptions()

# keys the native library reads (zk_set_option); values are ints
_NATIVE_KEYS = {"tile_huge": 0, "deterministic": 2, "dgrad_rw": 3, "wgrad_slab_mb": 5,
                "dgrad_deep": 6, "wgrad_deep": 7, "epilogue_prefetch": 8, "wgrad_tree": 10}


def _push_native() -> None:
    from zookeeper_amd.ops import _native

    if not _native.available():
        return
    L = _native.lib()
    fn = getattr(L, "zk_set_option", None)
    if fn is None:
        return
    for name, key in _NATIVE_KEYS.items():
        fn(key, int(getattr(OPTS, name)))


def set_options(**kwargs: Any) -> KernelOptions:
    """Update :data:`OPTS` (unknown names raise) and push the native ones."""
    fields = {f.name: f for f in dataclasses.fields(KernelOptions)}
    for k, v in kwargs.items():
        if k not in fields:
            raise TypeError(f"unknown kernel option {k!r}; known: {sorted(fields)}")
        typ = fields[k].type
        if typ in ("bool", bool):
            v = bool(v)
        elif typ in ("int", int):
            v = int(v)
        setattr(OPTS, k, v)
    _push_native()
    return OPTS


def snapshot() -> Dict[str, Any]:
    """The current options as a plain dict (run records, bench JSON)."""
    return dataclasses.asdict(OPTS)


def reset() -> None:
    """Restore the defaults (tests)."""
    set_options(**dataclasses.asdict(KernelOptions()))
