"""Small-K convolutions on MFMA (``csrc/kernels/smallconv.hip``): convs whose
reduction ``K = KH·KW·Cin`` is at most 64 — the layers that read the image
or a thin feature map, where the 64-channel-chunked implicit GEMMs of
``igemm.hip`` do not apply:

* BinaryNet's first layer: float input, ``ste_sign`` ±1 kernel, 3×3
  ``valid`` (examples/larq_experiment.py:62-69) — the kernel's sign is taken
  when packing, its STE mask (``|w| ≤ 1``) applied in the weight gradient;
* QuickNet's stem conv (3×3/2 over the image) and its 16→64 1×1 conv at
  small image sizes (``supported`` sends outputs above ``_MAX_PIXELS`` back to
  the library convolution, which is faster there).

3x3 convs over 1 or 3 channels (the image) take the row-band kernels at any
size: a block stages whole input rows in LDS and gathers im2col operands from
there (``zk_band_conv_*``); other shapes the generic 128-pixel-tile kernels.

forward   im2col of a 128-pixel tile built in LDS, ``v_mfma_f32_16x16x32_bf16``
          over the whole K (padded to 32 / 64), bf16 NHWC out;
backward  weight gradient: split-K over pixels, fp32 atomics straight into the
          flat gradient buffer (row-band path: per-block partials summed in a
          fixed order); data gradient (only the 1×1 stride-1 case
          needs one) = the same forward kernel on dY with Wᵀ (K = Cout ≤ 64).
"""

from __future__ import annotations

from typing import Optional

import torch

from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, lib, slab_reduce,
                                        stream_ptr, zeroed)

_INF = float("inf")


def _geometry(H, W, kh, kw, s, padding):
    from zookeeper_amd.ops.conv import geometry

    return geometry(H, W, kh, kw, s, padding)


def supported(x: torch.Tensor, weight: torch.Tensor, stride, padding: str, groups: int,
              bias: Optional[torch.Tensor] = None, pad_value: float = 0.0) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and weight.dim() == 4
            and weight.device == x.device
            and groups == 1 and bias is None and pad_value == 0.0 and padding in ("same", "valid")):
        return False
    Cout, Cin, kh, kw = weight.shape
    s = tuple(stride)
    if not (s[0] == s[1] and x.shape[1] == Cin and Cout % 16 == 0 and Cout <= 128
            and kh * kw * Cin <= 64):
        return False
    # a data gradient is only available for 1x1 stride-1 convs with Cout <= 64
    needs_dx = x.requires_grad and torch.is_grad_enabled()
    if needs_dx and not (kh == kw == 1 and s[0] == 1 and Cout <= 64 and Cin % 16 == 0):
        return False
    # Large images stay on the library convolution: at ImageNet size the
    # split-K weight gradient (im2col built element by element, transposed
    # 2-byte LDS stores) and the forward run far off the HBM roofline --
    # measured on MI355X, QuickNetLarge batch 512: its stem convs took
    # 3.05 ms (wgrad) + 1.21 ms (fwd) per step on these kernels (19.7k img/s)
    # against ~0.7 ms for every library kernel together in round 1 (22.7k).
    # BinaryNet's CIFAR-shape first layer (~0.23 M output pixels) keeps them.
    B, _, H, W = x.shape
    _, _, Ho, Wo = _geometry(H, W, kh, kw, s[0], padding)
    # ... except the image-reading 3x3 convs, which the row-band kernels take
    # at any size (QuickNet's 224x224 stem conv included), and 1x1 stride-1
    # convs, whose im2col rows are contiguous channel vectors (16-B copies)
    if kh == kw == 1 and s[0] == 1 and Cin % 8 == 0:
        return True
    return B * Ho * Wo <= _MAX_PIXELS or _band(B, H, W, Cin, Ho, Wo, Cout, kh, kw, s[0])


def _band(B, H, W, Cin, Ho, Wo, Cout, kh, kw, s) -> bool:
    """The row-band kernels take this geometry (3x3 over 1 or 3 channels)."""
    return bool(lib().zk_band_conv_ok(B, H, W, Cin, Ho, Wo, Cout, kh, kw, s))


_MAX_PIXELS = 1 << 20


def _pack(w2: torch.Tensor, KP: int) -> torch.Tensor:
    """[N][K] float → bf16 [N][KP], zero beyond K."""
    out = torch.zeros((w2.shape[0], KP), dtype=torch.bfloat16, device=w2.device)
    out[:, :w2.shape[1]] = w2.to(torch.bfloat16)
    return out


def _pack_native(weight: torch.Tensor, KP: int, sign: bool, transposed: bool):
    """The same operand from the [Cout][Cin][kh][kw] weight in one native
    launch (``zk_smallk_pack``): rows Cout with K in (kh, kw, Cin) order, or
    (``transposed``, 1x1 only) rows Cin with K = Cout; ``sign``: ±1.  None
    when the weight is not an fp32 CUDA tensor (the caller packs in torch)."""
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_cuda:
        return None
    Cout, Cin, kh, kw = w.shape
    s0, s1, s2, s3 = w.stride()
    if transposed:
        N, dims, strides, sn = Cin, (1, 1, Cout), (0, 0, s0), s1
    else:
        N, dims, strides, sn = Cout, (kh, kw, Cin), (s2, s3, s1), s0
    out = torch.empty((N, KP), dtype=torch.bfloat16, device=w.device)
    check(lib().zk_smallk_pack(w.data_ptr(), out.data_ptr(), N, KP, *dims, sn, *strides,
                               int(sign), stream_ptr(w.device)), "zk_smallk_pack")
    return out


class _SmallConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, padding, kclip):
        B, Cin, H, W = x.shape
        Cout, _, kh, kw = weight.shape
        pt, pl, Ho, Wo = _geometry(H, W, kh, kw, stride, padding)
        K = kh * kw * Cin
        KP = 32 if K <= 32 else 64
        wp = _pack_native(weight, KP, kclip is not None, False)
        if wp is None:
            w2 = weight.detach().permute(0, 2, 3, 1).reshape(Cout, K).float()
            if kclip is not None:  # ste_sign kernel: ±1 (sign(0) = +1)
                w2 = torch.where(w2 >= 0, 1.0, -1.0)
            wp = _pack(w2, KP)
        xn = x.permute(0, 2, 3, 1).contiguous()
        y = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=x.device)
        band = _band(B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride)
        fwd = lib().zk_band_conv_fwd if band else lib().zk_smallk_conv_fwd
        check(fwd(xn.data_ptr(), wp.data_ptr(), y.data_ptr(), B, H, W, Cin, Ho, Wo, Cout, kh, kw,
                  stride, pt, pl, stream_ptr(x.device)),
              "zk_band_conv_fwd" if band else "zk_smallk_conv_fwd")
        ctx.band = band
        ctx.save_for_backward(xn)
        ctx.weight, ctx.kclip = weight, kclip
        ctx.geom = (B, Cin, H, W, Cout, kh, kw, stride, pt, pl, Ho, Wo)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        (xn,) = ctx.saved_tensors
        weight, kclip = ctx.weight, ctx.kclip
        B, Cin, H, W, Cout, kh, kw, s, pt, pl, Ho, Wo = ctx.geom
        g = dout.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        dev = g.device
        L = lib()
        st = stream_ptr(dev)
        dx = dweight = None
        if ctx.needs_input_grad[0]:
            # 1x1 stride 1: dx = dY · W  (a K = Cout conv with Cin outputs)
            KPT = 32 if Cout <= 32 else 64
            wpT = _pack_native(weight, KPT, kclip is not None, True)
            if wpT is None:
                w2 = weight.detach().reshape(Cout, Cin).float()
                if kclip is not None:
                    w2 = torch.where(w2 >= 0, 1.0, -1.0)
                wpT = _pack(w2.t(), KPT)
            dxn = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
            check(L.zk_smallk_conv_fwd(g.data_ptr(), wpT.data_ptr(), dxn.data_ptr(), B, H, W, Cout,
                                       H, W, Cin, 1, 1, 1, 0, 0, st), "zk_smallk_conv_fwd(dgrad)")
            dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            target = direct_grad(weight, channels_last=True)
            dw = (target.permute(0, 2, 3, 1) if target is not None
                  else torch.zeros((Cout, kh, kw, Cin), dtype=torch.float32, device=dev))
            wf = weight.detach().permute(0, 2, 3, 1)
            if wf.dtype != torch.float32 or not wf.is_contiguous():
                wf = wf.float().contiguous()
            clip = _INF if kclip is None else float(kclip)
            if ctx.band:
                # per-block partials + fixed-order reduction (deterministic)
                n = L.zk_band_conv_wgrad_parts(B, Ho, Wo, 0)
                part = torch.empty((n, Cout, 32), dtype=torch.float32, device=dev)
                check(L.zk_band_conv_wgrad(g.data_ptr(), xn.data_ptr(), wf.data_ptr(),
                                           dw.data_ptr(), part.data_ptr(), B, H, W, Cin, Ho, Wo,
                                           Cout, kh, kw, s, pt, pl, clip, 0, st),
                      "zk_band_conv_wgrad")
            else:
                # slab policy (default / deterministic): per-block partials +
                # fixed-order reduce instead of fp32 atomics
                slab = None
                if slab_reduce():
                    nb = L.zk_smallk_conv_wgrad_blocks(B, Ho, Wo, 0)
                    slab = zeroed((nb, Cout * kh * kw * Cin), dev)
                check(L.zk_smallk_conv_wgrad(g.data_ptr(), xn.data_ptr(), wf.data_ptr(),
                                             dw.data_ptr(),
                                             slab.data_ptr() if slab is not None else None,
                                             B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl, clip,
                                             0, st), "zk_smallk_conv_wgrad")
                if slab is not None:
                    check(L.zk_wgrad_slab_reduce(slab.data_ptr(), slab.shape[0], slab.shape[1],
                                                 wf.data_ptr(), clip, dw.data_ptr(), st),
                          "zk_wgrad_slab_reduce")
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw.permute(0, 3, 1, 2)
        return dx, dweight, None, None, None


def small_conv(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: str,
               kernel_clip: Optional[float] = None) -> torch.Tensor:
    """Convolution with ``K = KH·KW·Cin ≤ 64`` (see ``supported``).  With
    ``kernel_clip`` the kernel is ``ste_sign``-quantised: ±1 forward, gradient
    masked by ``|w| ≤ kernel_clip``."""
    return _SmallConvFn.apply(x, weight, int(stride), padding, kernel_clip)
