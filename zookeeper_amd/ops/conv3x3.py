"""3×3 stride-1 ``same`` float convolution as MFMA implicit GEMMs.

The float 3×3 convs of ResNet-50's bottlenecks (and any other float 3×3
stride-1 layer with channel counts that tile by 64) run on the binary
conv's bf16 kernels of ``igemm.hip`` — they are plain bf16 MFMA implicit
GEMMs with ``conv3`` horizontal tap reuse underneath:

forward   ``y = x ⊛ W``: a forward convolution IS a data-gradient
          convolution with the taps flipped (``th → 2 − th``) and the
          padding mirrored (``kh − 1 − pt``), so the dgrad kernel runs it
          with roles renamed: act = x, "weights" = flip(W) as [T][Cout][Cin];
backward  ``dx = dy ⊛ Wᵀ``: the dgrad kernel proper (weights [T][Cin][Cout]);
          ``dW += xᵀ ⊛ dy``: the split-K weight-gradient kernel with its clip
          mask disabled (clip = +inf), accumulated in fp32 straight into the
          flat gradient buffer when the trainer manages it.

No padded copy of the activation is ever made (the kernels mask padding
taps per lane); MIOpen's path pads with an extra pass (TF ``same`` padding
through ``F.pad``).  The reference delegates these convs to Keras
(SURVEY §2.4); this is the MI355X-native replacement.
"""

from __future__ import annotations

from typing import Optional

import torch

from zookeeper_amd.ops import pointwise
from zookeeper_amd.ops import streams, weight_images
from zookeeper_amd.ops._native import check, direct_grad, grad_ready, igemm_wgrad, lib, stream_ptr
from zookeeper_amd.ops.options import OPTS

_INF = float("inf")


def supported(x: torch.Tensor, weight: torch.Tensor, stride, padding: str, groups: int,
              bias: Optional[torch.Tensor] = None, pad_value: float = 0.0) -> bool:
    return (OPTS.conv3_mfma and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and weight.device == x.device
            and weight.dim() == 4 and tuple(weight.shape[2:]) == (3, 3) and groups == 1
            and tuple(stride) == (1, 1) and padding == "same" and pad_value == 0.0
            and bias is None and x.shape[1] == weight.shape[1]
            and x.shape[1] % 64 == 0 and weight.shape[0] % 64 == 0
            and x.shape[0] * x.shape[2] * x.shape[3] < (1 << 24))


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor → contiguous NHWC storage (no copy if channels_last)."""
    return t.permute(0, 2, 3, 1).contiguous()


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stats_for=None):
        B, Cin, H, W = x.shape
        Cout = weight.shape[0]
        xn = _nhwc(x)
        st = stream_ptr(x.device)
        # forward as a dgrad: flipped taps, [T][N = Cout][K = Cin]
        imgs = weight_images.images(weight, True, st)
        if imgs is not None:  # kept by the optimizer
            wf = imgs[0]
        else:
            wd = weight.detach()
            wf = wd.flip(2, 3).permute(2, 3, 0, 1).reshape(9, Cout, Cin).to(torch.bfloat16)
            wf = wf.contiguous()
        ctx.wt = imgs[1] if imgs is not None else None
        y = torch.empty((B, H, W, Cout), dtype=torch.bfloat16, device=x.device)
        # dgrad geometry with roles renamed: "Cin" = Cout (N), "Cout" = Cin (K),
        # mirrored pads kh - 1 - 1 = 1
        if not pointwise.forward_with_stats(stats_for, xn, wf, y, Cout,
                                            (B, H, W, Cout, H, W, Cin, 3, 3, 1, 1, 1), st):
            check(lib().zk_igemm_dgrad(xn.data_ptr(), wf.data_ptr(), None, None, y.data_ptr(), B,
                                       H, W, Cout, H, W, Cin, 3, 3, 1, 1, 1, -1, st),
                  "zk_igemm_dgrad(3x3 fwd)")
        ctx.save_for_backward(xn)
        # (the producing BatchNorm's backward sums are not taken here: the 3x3
        # data gradients with an LDS epilogue are the 256-channel ones, whose
        # default is the phased deep kernel -- faster than v45 carrying the
        # fused sums, profiles/r5/c_resnet50_bn_fusion.md)
        ctx.weight = weight
        ctx.shape = (B, Cin, H, W, Cout)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        (xn,) = ctx.saved_tensors
        weight = ctx.weight
        B, Cin, H, W, Cout = ctx.shape
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
                    side = streams.side_wgrad(
                        dev, lambda sp: igemm_wgrad(g, xn, wf_t, dw_t,
                                                    (B, H, W, Cin, H, W, Cout, 3, 3, 1, 1, 1),
                                                    0, _INF, sp, "zk_igemm_wgrad(3x3)"),
                        weight, (g, xn))
        if ctx.needs_input_grad[0]:
            wt = ctx.wt
            if wt is None:
                wt = weight.detach().permute(2, 3, 1, 0).reshape(9, Cin, Cout).to(torch.bfloat16)
                wt = wt.contiguous()
            dxn = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
            check(L.zk_igemm_dgrad(g.data_ptr(), wt.data_ptr(), None, None, dxn.data_ptr(), B, H,
                                   W, Cin, H, W, Cout, 3, 3, 1, 1, 1, -1, st),
                  "zk_igemm_dgrad(3x3)")
            dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] and not side:
            target = direct_grad(weight, channels_last=True)
            dw = (target.permute(0, 2, 3, 1) if target is not None
                  else torch.zeros((Cout, 3, 3, Cin), dtype=torch.float32, device=dev))
            wf = weight.detach().permute(0, 2, 3, 1)
            if wf.dtype != torch.float32 or not wf.is_contiguous():
                wf = wf.float().contiguous()
            # clip = +inf: the kernel's |w| <= clip gradient mask is all-pass
            igemm_wgrad(g, xn, wf, dw, (B, H, W, Cin, H, W, Cout, 3, 3, 1, 1, 1), 0, _INF, st,
                        "zk_igemm_wgrad(3x3)")
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw.permute(0, 3, 1, 2)
        return dx, dweight, None


def conv3x3(x: torch.Tensor, weight: torch.Tensor, stats_for=None) -> torch.Tensor:
    """``same``-padded 3×3 stride-1 float convolution (see ``supported``) as
    MFMA implicit GEMMs.  Returns a channels_last bf16 tensor.  ``stats_for``:
    see ``pointwise.forward_with_stats`` (tiles with the LDS epilogue only)."""
    return _Conv3x3Fn.apply(x, weight, stats_for)
