"""Flat parameter / gradient storage.

All trainable parameters live as strided views into ONE contiguous fp32
buffer, and their ``.grad``s as views into a second one.  This is what lets

* the data-parallel bucketer all-reduce gradient *ranges* in place (no
  flatten/unflatten copies, one RCCL call per bucket), and
* the fused optimizer update every parameter in a single kernel launch over
  the flat buffers (with a per-parameter attribute table for ``weight_clip``
  and weight-decay masks).

Parameters are laid out in **reverse registration order** (the order in which
backward produces their gradients), so the first buckets to fill are the last
layers' — they can start all-reducing while early layers are still in
backward.  Each parameter keeps its own strides (e.g. ``channels_last`` conv
kernels stay physically OHWI).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn as nn

ALIGN = 64  # elements (256 B) — every parameter starts on a 256-B boundary


@dataclass
class ParamSlot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    clip: float  # 0 = no weight_clip constraint
    decay: bool  # weight decay applies (not to BN / bias)


def _clip_value(module: nn.Module, pname: str) -> float:
    if pname != "weight":
        return 0.0
    if getattr(module, "kernel_constraint", None) == "weight_clip":
        return 1.0
    return float(getattr(module, "clip_value", 0.0) or 0.0)


class FlatParams:
    def __init__(self, model: nn.Module, device: Optional[torch.device] = None):
        owners: Dict[int, tuple] = {}
        for mname, mod in model.named_modules():
            for pname, p in mod.named_parameters(recurse=False):
                if p.requires_grad and id(p) not in owners:
                    owners[id(p)] = (f"{mname}.{pname}" if mname else pname, mod, pname)
        params = [p for p in model.parameters() if p.requires_grad]
        params = list(reversed(params))
        slots: List[ParamSlot] = []
        offset = 0
        for p in params:
            name, mod, pname = owners[id(p)]
            decay = p.dim() > 1
            slots.append(ParamSlot(name, p, offset, p.numel(), _clip_value(mod, pname), decay))
            offset += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.total = offset
        dev = device if device is not None else (params[0].device if params else torch.device("cpu"))
        self.data = torch.zeros(self.total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=dev)
        for s in slots:
            p = s.param
            if not _dense(p):
                raise ValueError(f"parameter {s.name} is not densely strided")
            view = torch.as_strided(self.data, p.shape, p.stride(), s.offset)
            view.copy_(p.data)
            p.data = view
            p.grad = torch.as_strided(self.grad, p.shape, p.stride(), s.offset)
            # Fused kernels may accumulate straight into this gradient view
            # (see zookeeper_amd.ops._native.direct_grad).
            p._zk_direct_grad = True
        self.slots = slots

    def zero_grad(self) -> None:
        if self.grad.is_cuda:
            from zookeeper_amd.ops import _native

            if _native.available():  # a runtime memset, not a framework fill kernel
                _native.check(_native.lib().zk_zero(self.grad.data_ptr(),
                                                    self.grad.numel() * 4,
                                                    _native.stream_ptr(self.grad.device)),
                              "zk_zero")
                return
        self.grad.zero_()

    def rebind_grads(self) -> None:
        """Re-point ``.grad`` at the flat buffer (after external code replaced it)."""
        for s in self.slots:
            g = s.param.grad
            if g is None or g.data_ptr() != self.grad.data_ptr() + 4 * s.offset:
                s.param.grad = torch.as_strided(self.grad, s.param.shape, s.param.stride(), s.offset)

    def table(self) -> torch.Tensor:
        """Per-parameter attribute table ``[offset, numel, clip_bits, decay]``
        (int64) consumed by the fused optimizer kernel."""
        import struct

        rows = []
        for s in self.slots:
            clip_bits = struct.unpack("<i", struct.pack("<f", s.clip))[0]
            rows.append([s.offset, s.numel, clip_bits, int(s.decay)])
        return torch.tensor(rows, dtype=torch.int64)


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (a permutation of a contiguous layout)."""
    if t.numel() == 0:
        return True
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz > 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True
