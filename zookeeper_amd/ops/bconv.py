"""Stand-alone binary convolution and binary dense layer on the packed
kernels — the Larq ``QuantConv2D`` / ``QuantDense`` with ``ste_sign`` input
and kernel quantizers (examples/larq_experiment.py:62-99) when they are not
part of a fused residual block (BinaryNet: conv → max-pool → BN, and its
three dense layers).

forward   ``zk_sign_pack``: x → STE mask bits (``|x| ≤ clip``), the e2m1 ±1
          image (forward operand) and, when a backward will run, the bf16 ±1
          image (weight-gradient operand); ``zk_weight_pack``: latent kernel
          → e2m1 ±1 [T][Cout][Cin/2] and bf16 ±1 [T][Cin][Cout];
          ``zk_igemm_fwd_fp4``: MX-FP4 MFMA implicit GEMM → exact int16;
          ``zk_bn_apply`` with unit scale → bf16 output (exact up to bf16
          rounding of |y| > 256, as any bf16 activation);
backward  ``zk_igemm_dgrad`` (dY ⊛ sign(W)ᵀ with the input STE mask fused in
          its epilogue) and ``zk_igemm_wgrad`` (dYᵀ ⊛ sign(x), kernel STE mask
          ``|w| ≤ clip``, split-K slabs straight into the flat gradient).

A dense layer is the 1×1 conv over a 1×1 "image" per example: M = batch,
K = in_features, N = out_features.  ``out_features`` that do not tile by
64 (BinaryNet's 10-way classifier) run on a zero-padded kernel whose extra
outputs are dropped.
"""

from __future__ import annotations

from typing import Optional

import torch

from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, igemm_wgrad, lib,
                                        stream_ptr, zeroed_scratch)


# The forward kernels store the exact +-1 dot product as int16: a reduction
# length K = kh*kw*Cin of 32768 could reach +32768 (all signs agreeing) and
# wrap, so longer reductions take the library path.
INT16_MAX_K = 32767


def conv_supported(x: torch.Tensor, weight: torch.Tensor, stride, padding: str, groups: int,
                   bias: Optional[torch.Tensor] = None, pad_value: float = 0.0) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and weight.dim() == 4
            and weight.device == x.device
            and groups == 1 and bias is None and pad_value in (0.0, 1.0)
            and padding in ("same", "valid")):
        return False
    Cout, Cin, kh, kw = weight.shape
    s = tuple(stride)
    return (s[0] == s[1] and s[0] <= 2 and kh <= 4 and kw <= 4 and x.shape[1] == Cin
            and Cin % 64 == 0 and Cout % 64 == 0
            and kh * kw * Cin <= INT16_MAX_K
            and x.shape[0] * x.shape[2] * x.shape[3] < (1 << 24))


def dense_supported(x: torch.Tensor, weight: torch.Tensor, bias=None) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 2 and bias is None
            and weight.device == x.device
            and weight.shape[1] == x.shape[1] and x.shape[1] % 64 == 0
            and x.shape[1] <= INT16_MAX_K)


def _ones(owner, C: int, dev) -> tuple:
    """Persistent (scale = 1, shift = 0) vectors for the int16 → bf16 pass."""
    cache = owner.__dict__.setdefault("_zk_unit_affine", {})
    key = (C, str(dev))
    if key not in cache:
        cache[key] = (torch.ones(C, dtype=torch.float32, device=dev),
                      torch.zeros(C, dtype=torch.float32, device=dev))
    return cache[key]


class _BinaryConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, meta):
        stride, padding, clip, kclip, pad_ones, owner, will_backward = meta
        from zookeeper_amd.ops.conv import geometry

        B, Cin, H, W = x.shape
        Cout, _, kh, kw = weight.shape
        T = kh * kw
        pt, pl, Ho, Wo = geometry(H, W, kh, kw, stride, padding)
        dev = x.device
        st = stream_ptr(dev)
        L = lib()
        xn = x.permute(0, 2, 3, 1).contiguous()
        nwords = B * H * W * Cin // 32
        mask = torch.empty(nwords, dtype=torch.int32, device=dev)
        sx = (torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
              if will_backward else None)
        sx4 = torch.empty((B, H, W, Cin // 2), dtype=torch.uint8, device=dev)
        check(L.zk_sign_pack(xn.data_ptr(), None, mask.data_ptr(),
                             sx.data_ptr() if sx is not None else None, sx4.data_ptr(), nwords,
                             float(clip), st), "zk_sign_pack")
        w_ohwi = weight.detach().permute(0, 2, 3, 1).contiguous()
        if w_ohwi.dtype != torch.float32:
            w_ohwi = w_ohwi.float()
        wf4 = torch.empty((T, Cout, Cin // 2), dtype=torch.uint8, device=dev)
        wt = torch.empty((T, Cin, Cout), dtype=torch.bfloat16, device=dev) if will_backward else None
        check(L.zk_weight_pack(w_ohwi.data_ptr(), None, None,
                               wt.data_ptr() if wt is not None else None, None, wf4.data_ptr(),
                               Cout, T, Cin, st), "zk_weight_pack")
        y = torch.empty((B, Ho, Wo, Cout), dtype=torch.int16, device=dev)
        stats = zeroed_scratch(owner, "fwd_stats", (1, 2, Cout), torch.int64, dev)
        check(L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(),
                                 B, H, W, Cin, Cout, kh, kw, stride, pt, pl, Ho, Wo,
                                 int(pad_ones), 0, -1, 1, st), "zk_igemm_fwd_fp4")
        stats.zero_()  # statistics unused here (the BN that follows computes its own)
        # int16 -> bf16 with the unit-affine BN apply, viewed as rows of 64
        # channels (any Cout % 64 == 0; the affine is the same for every row)
        one, zero = _ones(owner, 64, dev)
        out = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=dev)
        check(L.zk_bn_apply(y.data_ptr(), one.data_ptr(), zero.data_ptr(), None, out.data_ptr(),
                            B * Ho * Wo * (Cout // 64), 64, st), "zk_bn_apply(int16->bf16)")
        ctx.save_for_backward(mask, sx, wt, w_ohwi)
        ctx.weight = weight
        ctx.geom = (B, Cin, H, W, Cout, kh, kw, stride, pt, pl, Ho, Wo)
        ctx.clips = (float(kclip), int(pad_ones))
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        weight = ctx.weight
        B, Cin, H, W, Cout, kh, kw = ctx.geom[:7]
        dev = dout.device
        dweight = None
        dw = None
        if ctx.needs_input_grad[1]:
            target = direct_grad(weight, channels_last=True)
            dw = (target.permute(0, 2, 3, 1) if target is not None
                  else torch.zeros((Cout, kh, kw, Cin), dtype=torch.float32, device=dev))
        g = dout.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        dx = _backward(ctx, g, ctx.needs_input_grad[0], dw)
        if dw is not None:
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw.permute(0, 3, 1, 2)
        return (dx.permute(0, 3, 1, 2) if dx is not None else None), dweight, None


def _backward(ctx, g: torch.Tensor, need_dx: bool, dw: Optional[torch.Tensor]):
    """dx (NHWC bf16, input STE mask applied) and dw += (OHWI fp32, kernel
    STE mask) from the saved forward state; g: dY NHWC bf16."""
    mask, sx, wt, w_ohwi = ctx.saved_tensors
    B, Cin, H, W, Cout, kh, kw, s, pt, pl, Ho, Wo = ctx.geom
    kclip, pad_ones = ctx.clips
    dev = g.device
    st = stream_ptr(dev)
    L = lib()
    dxn = None
    if need_dx:
        dxn = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
        check(L.zk_igemm_dgrad(g.data_ptr(), wt.data_ptr(), mask.data_ptr(), None,
                               dxn.data_ptr(), B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl,
                               -1, st), "zk_igemm_dgrad(binary conv)")
    if dw is not None:
        igemm_wgrad(g, sx, w_ohwi, dw, (B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl), pad_ones,
                    kclip, st, "zk_igemm_wgrad(binary conv)")
    return dxn


def binary_conv(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: str,
                clip: float = 1.0, kernel_clip: float = 1.0, pad_value: float = 0.0,
                owner=None) -> torch.Tensor:
    """``conv(ste_sign(x, clip), ste_sign(W, kernel_clip))`` (see
    ``conv_supported``).  ``owner`` (the layer module) holds persistent
    scratch buffers."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    meta = (int(stride), padding, float(clip), float(kernel_clip), pad_value == 1.0,
            owner if owner is not None else weight,
            torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad))
    return _BinaryConvFn.apply(x, weight, meta)


class _BinaryDenseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, meta):
        clip, kclip, owner, will_backward = meta
        Bn, K = x.shape
        N = weight.shape[0]
        Np = (N + 63) // 64 * 64
        w = weight.detach().float()
        if Np != N:
            w = torch.cat([w, w.new_zeros(Np - N, K)])
        # a dense layer is a 1x1 conv over a 1x1 image per example
        y = _BinaryConvFn.forward(ctx, x.reshape(Bn, K, 1, 1), w.view(Np, K, 1, 1),
                                  (1, "valid", clip, kclip, False, owner, will_backward))
        ctx.weight, ctx.N, ctx.Np = weight, N, Np
        return y.reshape(Bn, Np)[:, :N]

    @staticmethod
    def backward(ctx, dout):
        Bn = dout.shape[0]
        N, Np, weight = ctx.N, ctx.Np, ctx.weight
        K = weight.shape[1]
        dev = dout.device
        g = dout.to(torch.bfloat16)
        if Np != N:
            g = torch.cat([g, g.new_zeros(Bn, Np - N)], dim=1)
        g = g.contiguous()
        dweight = dw = target = None
        if ctx.needs_input_grad[1]:
            target = direct_grad(weight) if Np == N else None
            dw = target if target is not None else torch.zeros((Np, K), dtype=torch.float32,
                                                               device=dev)
        dxn = _backward(ctx, g, ctx.needs_input_grad[0], dw)
        if dw is not None:
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw[:N]
        return (dxn.reshape(Bn, K) if dxn is not None else None), dweight, None


def binary_dense(x: torch.Tensor, weight: torch.Tensor, clip: float = 1.0,
                 kernel_clip: float = 1.0, owner=None) -> torch.Tensor:
    """``ste_sign(x) · ste_sign(W)ᵀ`` on the packed binary-conv kernels."""
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    wb = torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad)
    return _BinaryDenseFn.apply(x, weight, (float(clip), float(kernel_clip),
                                            owner if owner is not None else weight, wb))
