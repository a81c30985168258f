"""1×1 (pointwise) float convolution as implicit GEMMs on the MFMA kernels.

A 1×1 stride-1 convolution over an NHWC (channels_last) activation is the
GEMM ``[P, Cin] × [Cin, Cout]`` with ``P = B·H·W`` — no im2col, no layout
change.  The binary-conv kernels of ``igemm.hip`` are plain bf16 MFMA
GEMMs underneath, so they run these float GEMMs directly:

forward   ``y = x · Wᵀ``: the dgrad kernel with its roles renamed (act = x,
          "weights" = W as [N = Cout][K = Cin]), bf16 out;
backward  ``dx = dy · W``: the dgrad kernel proper (weights Wᵀ [Cin][Cout]);
          ``dW += dyᵀ · x``: the split-K weight-gradient kernel with the clip
          mask disabled (clip = +inf), accumulated in fp32 straight into the
          flat gradient buffer.

Shapes whose channel counts do not tile by 64, or with a bias, stay on the
library convolution (``supported`` is False): as plain hipBLASLt GEMMs
their weight gradient (K = B·H·W, tiny M·N) measured up to 10× slower.

Used by BinaryResNet-E's downsampling shortcuts (AvgPool → 1×1 conv → BN),
QuickNet's transition 1×1 convs and ResNet-50's bottleneck 1×1 convs
(stride 1).  The reference has no kernels of its own; the
float convs it delegates to Keras are covered by this + MIOpen.
"""

from __future__ import annotations

from typing import Optional

import torch

from zookeeper_amd.ops import streams, weight_images
from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, igemm_wgrad, lib,
                                        stream_ptr, zeroed_scratch)
from zookeeper_amd.ops.options import OPTS

_INF = float("inf")
# Striped fp64 copies of the forward BN statistics the GEMM epilogue adds
# into (block b into copy b % FSTAT_STRIPES; zk_bn_finalize_f64_stripes sums
# and re-zeroes them).
FSTAT_STRIPES = 32
_HIP_INVALID_VALUE = 1  # hipErrorInvalidValue: no LDS-epilogue tile for this shape


def supported(x: torch.Tensor, weight: torch.Tensor, stride, groups: int,
              bias: Optional[torch.Tensor] = None) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and weight.device == x.device
            and weight.dim() == 4 and weight.shape[2:] == (1, 1) and groups == 1
            and tuple(stride) == (1, 1) and x.shape[1] == weight.shape[1]
            and bias is None and x.shape[1] % 64 == 0 and weight.shape[0] % 64 == 0
            and x.shape[0] * x.shape[2] * x.shape[3] < (1 << 24))


def forward_with_stats(stats_for, x, wt, y, n: int, geom, st) -> bool:
    """The float forward GEMM ``y = x * wt`` (``zk_igemm_dgrad`` geometry
    ``geom`` = B, H, W, N, Ho, Wo, K, kh, kw, stride, pt, pl) with the batch
    statistics of the BatchNorm ``stats_for`` summed in its LDS epilogue
    (``zk_igemm_dgrad_fstats``); ``_BatchNormFn`` picks them up by y's
    address instead of running a statistics pass.  Only in training outside
    the deterministic mode (fp64 atomics).  False: nothing was launched
    (no BN, or no LDS-epilogue tile for this shape) -- run the plain GEMM."""
    if (stats_for is None or not stats_for.training or OPTS.deterministic
            or not OPTS.bn_stats_epilogue):
        return False
    parts = zeroed_scratch(stats_for, "fstats", (FSTAT_STRIPES, 2, n), torch.float64, y.device)
    if stats_for.__dict__.pop("_zk_pending_fstats", None) is not None:
        # the previous GEMM's statistics were never consumed (its output
        # reached the BatchNorm some other way, or not at all): the
        # accumulator was not finalised and re-zeroed -- do it here, or this
        # epilogue would add onto stale sums
        parts.zero_()
    rc = lib().zk_igemm_dgrad_fstats(x.data_ptr(), wt.data_ptr(), y.data_ptr(), parts.data_ptr(),
                                     FSTAT_STRIPES, *geom, -1, st)
    if rc == _HIP_INVALID_VALUE:
        return False
    check(rc, "zk_igemm_dgrad_fstats")
    stats_for.__dict__["_zk_pending_fstats"] = (parts, y.data_ptr(), FSTAT_STRIPES)
    return True


def _rows(x: torch.Tensor) -> torch.Tensor:
    """[B, C, H, W] (any layout) → contiguous [B·H·W, C] (a view when the
    input is channels_last)."""
    xn = x.permute(0, 2, 3, 1)
    if not xn.is_contiguous():
        xn = xn.contiguous()
    return xn.reshape(-1, x.shape[1])


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, handoff=None, give=None, stats_for=None):
        B, Cin, H, W = x.shape
        Cout = weight.shape[0]
        x2 = _rows(x)
        L = lib()
        st = stream_ptr(x.device)
        imgs = weight_images.images(weight, False, st)
        if imgs is not None:  # kept by the optimizer: [1][Cout][Cin], [1][Cin][Cout]
            w2, wt = imgs[0].view(Cout, Cin), imgs[1].view(Cin, Cout)
        else:
            w2, wt = weight.detach().reshape(Cout, Cin).to(torch.bfloat16), None
        y2 = torch.empty((x2.shape[0], Cout), dtype=torch.bfloat16, device=x.device)
        # dgrad kernel, roles renamed: N = Cout ("Cin"), K = Cin ("Cout")
        if not forward_with_stats(stats_for, x2, w2, y2, Cout, (B, H, W, Cout, H, W, Cin,
                                                                 1, 1, 1, 0, 0), st):
            check(L.zk_igemm_dgrad(x2.data_ptr(), w2.data_ptr(), None, None, y2.data_ptr(),
                                   B, H, W, Cout, H, W, Cin, 1, 1, 1, 0, 0, -1, st),
                  "zk_igemm_dgrad(1x1 fwd)")
        ctx.save_for_backward(x2, w2)
        # the producing BatchNorm's backward sums, reduced in our dgrad
        # epilogue when it writes x's whole gradient (norm_pool.FloatBnSum)
        fsum = getattr(x, "_zk_fbnsum", None)
        ctx.fsum = (fsum if fsum is not None and give is None
                    and tuple(fsum.xn.shape) == (B, H, W, Cin) else None)
        ctx.wt = wt
        ctx.weight = weight
        ctx.handoff, ctx.give = handoff, give
        if handoff is not None:
            handoff.masked_ok = True  # our epilogue masks a (g, mask) hand-off itself
        ctx.shape = (B, Cin, H, W, Cout)
        return y2.view(B, H, W, Cout).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        x2, w2 = ctx.saved_tensors
        weight = ctx.weight
        B, Cin, H, W, Cout = ctx.shape
        g2 = _rows(dout.to(torch.bfloat16))
        dev = g2.device
        L = lib()
        st = stream_ptr(dev)
        dx = dweight = None
        side = False
        if ctx.needs_input_grad[1]:
            # weight gradient first, on the side stream when one is active: it
            # then overlaps this data gradient and the BN passes that follow
            target = direct_grad(weight)
            if target is not None:
                dw_t = target.view(Cout, Cin)
                wf_t = weight.detach().reshape(Cout, Cin)
                if wf_t.dtype == torch.float32 and wf_t.is_contiguous():
                    side = streams.side_wgrad(
                        dev, lambda sp: igemm_wgrad(g2, x2, wf_t, dw_t,
                                                    (B, H, W, Cin, H, W, Cout, 1, 1, 1, 0, 0),
                                                    0, _INF, sp, "zk_igemm_wgrad(1x1)"),
                        weight, (g2, x2))
        # + the identity shortcut's gradient of x (norm_pool.ResidualHandoff):
        # a tensor, or (g, ReLU mask bits) that the epilogue masks itself
        dres = ctx.handoff.take() if ctx.handoff is not None else None
        dmask = None
        if isinstance(dres, tuple):
            dres, dmask = dres
        if ctx.needs_input_grad[0]:
            dx2 = torch.empty((g2.shape[0], Cin), dtype=torch.bfloat16, device=dev)
            wt = ctx.wt if ctx.wt is not None else w2.t().contiguous()  # [Cin][Cout]
            if dres is not None and dres.numel() != B * H * W * Cin:
                raise RuntimeError(f"residual gradient {tuple(dres.shape)} does not match the "
                                   f"1x1 conv input {(B, H, W, Cin)}")
            fs = ctx.fsum
            rc = _HIP_INVALID_VALUE
            if fs is not None or dmask is not None:
                rc = L.zk_igemm_dgrad_ex(
                    g2.data_ptr(), wt.data_ptr(), dres.data_ptr() if dres is not None else None,
                    dmask.data_ptr() if dmask is not None else None, dx2.data_ptr(),
                    fs.xn.data_ptr() if fs is not None else None,
                    fs.coef.data_ptr() if fs is not None else None,
                    fs.mask.data_ptr() if fs is not None and fs.mask is not None else None,
                    fs.relu if fs is not None else 0,
                    fs.sums.data_ptr() if fs is not None else None,
                    fs.sums.shape[0] if fs is not None else 1, B, H, W, Cin, H, W, Cout, 1, 1, 1,
                    0, 0, -1, st)
                if rc != _HIP_INVALID_VALUE:
                    check(rc, "zk_igemm_dgrad_ex(1x1)")
                    if fs is not None:
                        fs.take(dx2)
            if rc == _HIP_INVALID_VALUE:  # no LDS-epilogue tile: the plain GEMM
                if dmask is not None:  # materialise g * mask
                    bits = (dmask.unsqueeze(-1) >> torch.arange(8, device=dev, dtype=torch.uint8)) & 1
                    dres = dres.reshape(-1) * bits.reshape(-1).to(dres.dtype)
                check(L.zk_igemm_dgrad(g2.data_ptr(), wt.data_ptr(), None,
                                       dres.data_ptr() if dres is not None else None,
                                       dx2.data_ptr(), B, H, W, Cin, H, W, Cout, 1, 1, 1, 0, 0,
                                       -1, st), "zk_igemm_dgrad(1x1)")
            if ctx.give is not None and ctx.give.give(dx2.view(B, H, W, Cin)):
                dx = None  # x's other consumer adds it (a downsampling shortcut conv)
            else:
                dx = dx2.view(B, H, W, Cin).permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1] and not side:
            target = direct_grad(weight)
            dw = target.view(Cout, Cin) if target is not None else torch.zeros(
                (Cout, Cin), dtype=torch.float32, device=dev)
            wf = weight.detach().reshape(Cout, Cin)
            if wf.dtype != torch.float32 or not wf.is_contiguous():
                wf = wf.float().contiguous()
            # clip = +inf: the kernel's |w| <= clip gradient mask is all-pass
            igemm_wgrad(g2, x2, wf, dw, (B, H, W, Cin, H, W, Cout, 1, 1, 1, 0, 0), 0, _INF, st,
                        "zk_igemm_wgrad(1x1)")
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw.view(Cout, Cin, 1, 1)
        return dx, dweight, None, None, None


def conv1x1(x: torch.Tensor, weight: torch.Tensor, handoff=None, give=None,
            stats_for=None) -> torch.Tensor:
    """``F.conv2d(x, weight)`` for a 1×1 stride-1 kernel (see ``supported``),
    as MFMA implicit GEMMs.  Returns a channels_last bf16 tensor.  With a
    ``norm_pool.ResidualHandoff`` as ``handoff`` the data gradient also adds
    the gradient another consumer of the same input left there; as ``give``
    the data gradient is left there for that consumer instead of returned.
    ``stats_for``: the BatchNorm module that normalises the output next; in
    training (outside the deterministic mode) its batch statistics come from
    this GEMM's epilogue (``zk_igemm_dgrad_fstats``) instead of a separate
    pass over y."""
    return _Conv1x1Fn.apply(x, weight, handoff, give, stats_for)
