"""General float convolution (stride 1 or 2, kernel ≤ 4×4, TF ``same`` or
``valid`` padding) as MFMA implicit GEMMs on the ``igemm.hip`` kernels.

This is the MI355X-native path for the float convs that neither the 1×1
stride-1 GEMM (``ops/pointwise.py``) nor the 3×3 stride-1 ``conv3`` path
(``ops/conv3x3.py``) covers — ResNet-50's strided 3×3 convs (first block of
stages 2-4) and strided 1×1 downsampling shortcuts, any strided float conv
in the zoo:

forward   ``y = x ⊛ W``: the binary forward kernel (``igemm_conv_kernel``
          with FWD) on bf16 operands and its bf16 epilogue
          (``zk_igemm_fwd_bf16``), weights as [T][Cout][Cin];
backward  ``dx = dy ⊛ Wᵀ``: the strided dgrad kernel (stride-parity classes,
          weights [T][Cin][Cout], no STE mask);
          ``dW += xᵀ ⊛ dy``: the split-K weight-gradient kernel with the clip
          mask disabled (clip = +inf), straight into the flat gradient buffer.

The reference delegates these convs to Keras; this replaces
the MIOpen ``igemm_*_gtcx35`` kernels that round 1 still ran for them.
"""

from __future__ import annotations

from typing import Optional, Tuple

import torch

from zookeeper_amd.ops import streams, weight_images
from zookeeper_amd.ops._native import check, direct_grad, grad_ready, igemm_wgrad, lib, stream_ptr
from zookeeper_amd.ops.options import OPTS

_INF = float("inf")


def geometry(H: int, W: int, kh: int, kw: int, stride: int, padding: str) -> Tuple[int, int, int, int]:
    """(pt, pl, Ho, Wo) with TensorFlow ``same`` / ``valid`` semantics."""
    from zookeeper_amd.nn.layers import same_padding

    if padding == "same":
        pt, pb = same_padding(H, kh, stride)
        pl, pr = same_padding(W, kw, stride)
    else:
        pt = pb = pl = pr = 0
    return pt, pl, (H + pt + pb - kh) // stride + 1, (W + pl + pr - kw) // stride + 1


def supported(x: torch.Tensor, weight: torch.Tensor, stride, padding: str, groups: int,
              bias: Optional[torch.Tensor] = None, pad_value: float = 0.0) -> bool:
    if not (OPTS.conv_mfma and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and weight.device == x.device
            and weight.dim() == 4 and groups == 1 and bias is None and pad_value == 0.0):
        return False
    Cout, Cin, kh, kw = weight.shape
    s = tuple(stride)
    return (s[0] == s[1] and s[0] in (1, 2) and kh <= 4 and kw <= 4 and x.shape[1] == Cin
            and Cin % 64 == 0 and Cout % 64 == 0 and padding in ("same", "valid")
            and x.shape[0] * x.shape[2] * x.shape[3] < (1 << 24))


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1).contiguous()


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, padding, handoff=None):
        B, Cin, H, W = x.shape
        Cout, _, kh, kw = weight.shape
        pt, pl, Ho, Wo = geometry(H, W, kh, kw, stride, padding)
        T = kh * kw
        xn = _nhwc(x)
        st = stream_ptr(x.device)
        imgs = weight_images.images(weight, False, st)  # kept by the optimizer
        if imgs is not None:
            wf = imgs[0]
        else:
            wf = weight.detach().permute(2, 3, 0, 1).reshape(T, Cout, Cin).to(torch.bfloat16)
            wf = wf.contiguous()
        ctx.wt = imgs[1] if imgs is not None else None
        y = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=x.device)
        check(lib().zk_igemm_fwd_bf16(xn.data_ptr(), wf.data_ptr(), y.data_ptr(), B, H, W, Cin,
                                      Cout, kh, kw, stride, pt, pl, Ho, Wo, 0, -1, st),
              "zk_igemm_fwd_bf16")
        ctx.save_for_backward(xn)
        ctx.weight = weight
        ctx.geom = (B, Cin, H, W, Cout, kh, kw, stride, pt, pl, Ho, Wo)
        ctx.handoff = handoff
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        (xn,) = ctx.saved_tensors
        weight = ctx.weight
        B, Cin, H, W, Cout, kh, kw, s, pt, pl, Ho, Wo = ctx.geom
        T = kh * kw
        g = _nhwc(dout.to(torch.bfloat16))
        dev = g.device
        L = lib()
        st = stream_ptr(dev)
        dx = dweight = None
        side = False
        if ctx.needs_input_grad[1]:
            # weight gradient first, on the side stream when one is active
            target = direct_grad(weight, channels_last=True)
            if target is not None:
                dw_t = target.permute(0, 2, 3, 1)
                wf_t = weight.detach().permute(0, 2, 3, 1)
                if wf_t.dtype == torch.float32 and wf_t.is_contiguous():
                    geo = (B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl)
                    side = streams.side_wgrad(
                        dev, lambda sp: igemm_wgrad(g, xn, wf_t, dw_t, geo, 0, _INF, sp,
                                                    "zk_igemm_wgrad(conv)"),
                        weight, (g, xn))
        # + x's other gradient, left by a consumer that ran first (ResidualHandoff)
        dres = ctx.handoff.take() if ctx.handoff is not None else None
        if ctx.needs_input_grad[0]:
            wt = ctx.wt
            if wt is None:
                wt = weight.detach().permute(2, 3, 1, 0).reshape(T, Cin, Cout).to(torch.bfloat16)
                wt = wt.contiguous()
            dxn = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
            if dres is not None and (tuple(dres.shape) != (B, H, W, Cin)
                                     or not dres.is_contiguous()):
                raise RuntimeError(f"hand-off gradient {tuple(dres.shape)} does not match the "
                                   f"conv input {(B, H, W, Cin)}")
            check(L.zk_igemm_dgrad(g.data_ptr(), wt.data_ptr(), None,
                                   dres.data_ptr() if dres is not None else None, dxn.data_ptr(),
                                   B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl, -1, st),
                  "zk_igemm_dgrad(conv)")
            dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] and not side:
            target = direct_grad(weight, channels_last=True)
            dw = (target.permute(0, 2, 3, 1) if target is not None
                  else torch.zeros((Cout, kh, kw, Cin), dtype=torch.float32, device=dev))
            wf = weight.detach().permute(0, 2, 3, 1)
            if wf.dtype != torch.float32 or not wf.is_contiguous():
                wf = wf.float().contiguous()
            igemm_wgrad(g, xn, wf, dw, (B, H, W, Cin, Ho, Wo, Cout, kh, kw, s, pt, pl), 0, _INF,
                        st, "zk_igemm_wgrad(conv)")
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw.permute(0, 3, 1, 2)
        return dx, dweight, None, None, None


def conv2d(x: torch.Tensor, weight: torch.Tensor, stride: int, padding: str,
           handoff=None) -> torch.Tensor:
    """Float convolution with TF padding semantics (see ``supported``) as MFMA
    implicit GEMMs.  Returns a channels_last bf16 tensor.  ``handoff``: the
    data gradient also adds x's other gradient left there
    (``norm_pool.ResidualHandoff``)."""
    return _ConvFn.apply(x, weight, int(stride), padding, handoff)
