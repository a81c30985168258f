"""Memory-bound fused ops: input normalisation and the fused optimizer."""

from __future__ import annotations

import ctypes
import itertools
from typing import Sequence

import torch

from zookeeper_amd.ops._native import check, lib, stream_ptr

_flip_seed = itertools.count(1)


def normalize_flip(image: torch.Tensor, mean: Sequence[float], std: Sequence[float],
                   flip: bool, seed: int = None, out: torch.Tensor = None) -> torch.Tensor:
    """uint8 ``[B,H,W,3]`` → bf16 ``[B,H,W,3]`` normalised, optionally with a
    per-image random horizontal flip (one kernel).  ``out``: a contiguous bf16
    ``[B,H,W,3]`` tensor to write (the loader's per-slot buffer)."""
    if image.dtype != torch.uint8 or image.dim() != 4 or image.shape[3] != 3:
        raise ValueError("normalize_flip expects uint8 [B,H,W,3]")
    if not image.is_contiguous():
        image = image.contiguous()
    B, H, W, _ = image.shape
    if W % 4:
        raise ValueError("normalize_flip needs W % 4 == 0")
    if out is None:
        out = torch.empty((B, H, W, 3), dtype=torch.bfloat16, device=image.device)
    elif (out.shape != (B, H, W, 3) or out.dtype != torch.bfloat16 or not out.is_contiguous()
          or out.device != image.device):
        raise ValueError("normalize_flip: out must be a contiguous bf16 [B,H,W,3] tensor "
                         "on the image's device")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    seed = next(_flip_seed) if seed is None else seed
    check(lib().zk_normalize_flip_c3(image.data_ptr(), out.data_ptr(), B, H, W, m, s,
                                     int(bool(flip)), seed, stream_ptr(image.device)),
          "zk_normalize_flip_c3")
    return out


def normalize_flip_pack(image: torch.Tensor, mean: Sequence[float], std: Sequence[float],
                        flip: bool, spec, out: torch.Tensor = None, xp: torch.Tensor = None,
                        seed: int = None):
    """:func:`normalize_flip` that also writes the fused stem's padded input
    ``xp`` bf16 ``[B, Hp, Wp, 4]`` in the same pass (``spec = (Hp, Wp, pt,
    pl)``, published by ``ops.stem``).  Returns ``(out, xp)``; both
    bit-identical to ``normalize_flip`` followed by the stem's own pack."""
    if image.dtype != torch.uint8 or image.dim() != 4 or image.shape[3] != 3:
        raise ValueError("normalize_flip_pack expects uint8 [B,H,W,3]")
    if not image.is_contiguous():
        image = image.contiguous()
    B, H, W, _ = image.shape
    Hp, Wp, pt, pl = spec
    dev = image.device
    if out is None:
        out = torch.empty((B, H, W, 3), dtype=torch.bfloat16, device=dev)
    if xp is None:
        xp = torch.empty((B, Hp, Wp, 4), dtype=torch.bfloat16, device=dev)
    for t, shape in ((out, (B, H, W, 3)), (xp, (B, Hp, Wp, 4))):
        if t.shape != shape or t.dtype != torch.bfloat16 or not t.is_contiguous() \
                or t.device != dev:
            raise ValueError(f"normalize_flip_pack: output must be a contiguous bf16 {shape} "
                             "tensor on the image's device")
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    seed = next(_flip_seed) if seed is None else seed
    check(lib().zk_normalize_flip_pack_c3(image.data_ptr(), out.data_ptr(), xp.data_ptr(), B, H,
                                          W, Hp, Wp, pt, pl, m, s, int(bool(flip)), seed,
                                          stream_ptr(dev)), "zk_normalize_flip_pack_c3")
    return out, xp


CHUNK = 16384


def chunk_table(flat, images=None) -> torch.Tensor:
    """Split every parameter of a FlatParams into ≤CHUNK-element chunks:
    rows of ``[offset, numel, clip_bits, flags]`` (int64); flags = decay
    (bit 0) | (1 + the parameter's weight-image row) << 8."""
    import struct

    rows = []
    for s in flat.slots:
        clip_bits = struct.unpack("<i", struct.pack("<f", s.clip))[0]
        img = images.row_of(s.param) if images is not None else -1
        flags = int(s.decay) | ((img + 1) << 8)
        for lo in range(0, s.numel, CHUNK):
            rows.append([s.offset + lo, min(CHUNK, s.numel - lo), clip_bits, flags])
    return torch.tensor(rows, dtype=torch.int64)


def fused_optimizer_step(opt, lr: float) -> None:
    """One launch: Adam/SGD + decay + 1/world grad scaling + weight_clip,
    plus the bf16 weight images of the float convs (ops/weight_images.py)."""
    flat, sp = opt.flat, opt.spec
    reg = getattr(flat, "images", None)
    gen = reg.generation if reg is not None else -1
    if getattr(opt, "_chunks", None) is None or getattr(opt, "_chunks_gen", None) != gen:
        opt._chunks = chunk_table(flat, reg).to(flat.data.device)
        opt._chunks_gen = gen
    ch = opt._chunks
    st = stream_ptr(flat.data.device)
    table = reg.table() if reg is not None else None
    tptr = table.data_ptr() if table is not None else None
    if sp.kind == "adam":
        t = opt.step_count
        check(lib().zk_adam_step(flat.data.data_ptr(), flat.grad.data_ptr(), opt.m.data_ptr(),
                                 opt.v.data_ptr(), ch.data_ptr(), ch.shape[0], lr, sp.beta_1,
                                 sp.beta_2, sp.eps_effective(t), sp.weight_decay, 1 - sp.beta_1**t,
                                 1 - sp.beta_2**t, opt.grad_scale, tptr, st), "zk_adam_step")
    else:
        check(lib().zk_sgd_step(flat.data.data_ptr(), flat.grad.data_ptr(), opt.m.data_ptr(),
                                ch.data_ptr(), ch.shape[0], lr, sp.momentum, sp.weight_decay,
                                opt.grad_scale, int(sp.nesterov), tptr, st), "zk_sgd_step")
    if reg is not None and table is not None:
        reg._mark_current()  # every registered image was rewritten from the new parameters
