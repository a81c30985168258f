"""Binarisation quantizers with straight-through-estimator gradients.

The reference example quantizes with Larq's ``ste_sign`` and constrains
latent weights with ``weight_clip`` (examples/larq_experiment.py:50-56).  Larq
is not a dependency here; the quantizers are re-defined from their published
definitions:

* ``ste_sign``:  forward ``sign(x)`` with ``sign(0) = +1``; backward
  ``g * 1{|x| <= clip}`` (clip = 1).
* ``approx_sign``: forward as ``ste_sign``; backward ``g * (2 - 2|x|)`` on
  ``|x| <= 1`` (Bi-Real Net's piecewise-polynomial estimator).
* ``swish_sign``: forward as ``ste_sign``; backward
  ``β(2 - βx·tanh(βx/2)) / (1 + cosh(βx))`` with β = 5 (SwishSign, BNN+).
* ``magnitude_aware_sign``: ``mean(|w|) per output channel * ste_sign(w)``.

These are the *oracle* (pure PyTorch) implementations.  The fused HIP path
never materialises ±1 tensors: signs are bit-packed inside the producing
kernel (see ``zookeeper_amd.ops``).
"""

from __future__ import annotations

from typing import Callable, Optional, Union

import torch


def sign_pm1(x: torch.Tensor) -> torch.Tensor:
    """``sign`` with ``sign(0) = +1`` (so the result is always ±1)."""
    one = torch.ones((), dtype=x.dtype, device=x.device)
    return torch.where(x >= 0, one, -one)


class _SteSign(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, clip_value: float):
        ctx.save_for_backward(x)
        ctx.clip_value = clip_value
        return sign_pm1(x)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        (x,) = ctx.saved_tensors
        return g * (x.abs() <= ctx.clip_value).to(g.dtype), None


class _ApproxSign(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor):
        ctx.save_for_backward(x)
        return sign_pm1(x)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        (x,) = ctx.saved_tensors
        ax = x.abs()
        return g * torch.where(ax <= 1, 2 - 2 * ax, torch.zeros_like(ax)).to(g.dtype)


class _SwishSign(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, beta: float):
        ctx.save_for_backward(x)
        ctx.beta = beta
        return sign_pm1(x)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        (x,) = ctx.saved_tensors
        b = ctx.beta
        bx = b * x.float()
        grad = b * (2 - bx * torch.tanh(bx / 2)) / (1 + torch.cosh(bx))
        return g * grad.to(g.dtype), None


def ste_sign(x: torch.Tensor, clip_value: float = 1.0) -> torch.Tensor:
    return _SteSign.apply(x, clip_value)


def approx_sign(x: torch.Tensor) -> torch.Tensor:
    return _ApproxSign.apply(x)


def swish_sign(x: torch.Tensor, beta: float = 5.0) -> torch.Tensor:
    return _SwishSign.apply(x, beta)


def magnitude_aware_sign(w: torch.Tensor) -> torch.Tensor:
    """Per-output-channel scaled sign (XNOR-Net style), for kernels."""
    scale = w.detach().abs().mean(dim=tuple(range(1, w.dim())), keepdim=True)
    return scale * ste_sign(w)


QUANTIZERS = {
    "ste_sign": ste_sign,
    "approx_sign": approx_sign,
    "swish_sign": swish_sign,
    "magnitude_aware_sign": magnitude_aware_sign,
}

Quantizer = Optional[Union[str, Callable[[torch.Tensor], torch.Tensor]]]


def get_quantizer(q: Quantizer) -> Optional[Callable[[torch.Tensor], torch.Tensor]]:
    if q is None or callable(q):
        return q
    try:
        return QUANTIZERS[q]
    except KeyError:
        raise ValueError(f"Unknown quantizer '{q}'. Known: {sorted(QUANTIZERS)}") from None


def is_binary_sign(q: Quantizer) -> bool:
    """True if ``q`` produces exactly ±1 (so XNOR-popcount is exact)."""
    return q in ("ste_sign", "approx_sign", "swish_sign") or q in (
        ste_sign,
        approx_sign,
        swish_sign,
    )


def weight_clip(w: torch.Tensor, clip_value: float = 1.0) -> None:
    """In-place ``weight_clip`` constraint: clamp latent weights to [-c, c]."""
    with torch.no_grad():
        w.clamp_(-clip_value, clip_value)


CONSTRAINTS = {"weight_clip": weight_clip}
