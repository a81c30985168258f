"""Depthwise 3×3 convolution on bf16 NHWC activations (HIP kernels in
``csrc/kernels/depthwise.hip``) as an autograd function.

Used by the QuickNet stem (trainable depthwise 3×3/2) and the fixed blur-pool
of QuickNet transitions (no weight gradient).  Weights stay fp32 — the master
parameter (or the fixed blur buffer) is read directly, never cast.
"""

from __future__ import annotations

import torch

from zookeeper_amd.nn.layers import same_padding
from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, lib, slab_reduce,
                                        stream_ptr, zeroed)


def supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    C = x.shape[1]
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and C % 8 == 0
            and weight.device == x.device
            and 256 % (C // 8) == 0 and tuple(weight.shape) == (C, 1, 3, 3)
            and weight.dtype == torch.float32)


def _geometry(H, W, k, s, padding):
    if padding == "same":
        pt, pb = same_padding(H, k, s)
        pl, pr = same_padding(W, k, s)
    else:
        pt = pb = pl = pr = 0
    return pt, pl, (H + pt + pb - k) // s + 1, (W + pl + pr - k) // s + 1


class _DepthwiseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, padding):
        B, C, H, W = x.shape
        pt, pl, Ho, Wo = _geometry(H, W, 3, stride, padding)
        xn = x.permute(0, 2, 3, 1).contiguous()
        w = weight.detach().contiguous()
        y = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=x.device)
        check(lib().zk_dw_fwd(xn.data_ptr(), w.data_ptr(), y.data_ptr(), B, H, W, C, Ho, Wo, 3,
                              stride, pt, pl, stream_ptr(x.device)), "zk_dw_fwd")
        ctx.save_for_backward(xn if weight.requires_grad else None, w)
        ctx.param = weight
        ctx.geom = (B, H, W, C, Ho, Wo, stride, pt, pl)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        xn, w = ctx.saved_tensors
        B, H, W, C, Ho, Wo, s, pt, pl = ctx.geom
        st = stream_ptr(dy.device)
        g = dy.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((B, H, W, C), dtype=torch.bfloat16, device=dy.device)
            check(lib().zk_dw_dgrad(g.data_ptr(), w.data_ptr(), dx.data_ptr(), B, H, W, C, Ho,
                                    Wo, 3, s, pt, pl, st), "zk_dw_dgrad")
            dx = dx.permute(0, 3, 1, 2)
        dw = None
        if ctx.needs_input_grad[1]:
            target = direct_grad(ctx.param, channels_last=False)
            buf = target if target is not None else torch.zeros(C, 9, device=dy.device)
            L = lib()
            # slab policy (default / deterministic): per-block partials +
            # fixed-order reduce instead of fp32 atomics
            slab = (zeroed((L.zk_dw_wgrad_blocks(B, Ho, Wo, C), C * 9), dy.device)
                    if slab_reduce() else None)
            check(L.zk_dw_wgrad(g.data_ptr(), xn.data_ptr(), buf.data_ptr(),
                                slab.data_ptr() if slab is not None else None, B, H, W, C, Ho,
                                Wo, 3, s, pt, pl, st), "zk_dw_wgrad")
            if slab is not None:
                check(L.zk_wgrad_slab_reduce(slab.data_ptr(), slab.shape[0], slab.shape[1], None,
                                             0.0, buf.data_ptr(), st), "zk_wgrad_slab_reduce")
            if target is not None:
                grad_ready(ctx.param)
            else:
                dw = buf.view(C, 1, 3, 3)
        return dx, dw, None, None


def depthwise_conv3x3(x: torch.Tensor, weight: torch.Tensor, stride: int,
                      padding: str = "same") -> torch.Tensor:
    """``x`` NCHW-shaped (channels_last) bf16, ``weight`` fp32 ``(C,1,3,3)``."""
    return _DepthwiseFn.apply(x, weight, stride, padding)
