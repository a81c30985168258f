"""Custom operators backed by the hand-written gfx950 HIP kernels.

Every op has a pure-PyTorch reference implementation (the *oracle*) used on
CPU and by the numerics tests; on a GPU the HIP kernels are the only path
(no silent fallback — see ``_native``).
"""

from zookeeper_amd.ops._native import available, load_error, native_disabled
from zookeeper_amd.ops.binary import binary_block
from zookeeper_amd.ops.elementwise import (chunk_table, fused_optimizer_step, normalize_flip,
                                           normalize_flip_pack)
from zookeeper_amd.ops.xent import softmax_xent

__all__ = ["available", "binary_block", "chunk_table", "fused_optimizer_step", "load_error",
           "native_disabled", "normalize_flip", "normalize_flip_pack", "softmax_xent"]
