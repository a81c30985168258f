"""Fused binary residual block: ``out = BN(act(bconv(sign(x)))) + residual``.

One autograd op per block (used by BinaryResNet-E and QuickNet on the
``hip`` backend).  Forward kernels:

1. ``zk_sign_pack``   x bf16 → STE mask bits (|x| ≤ clip), the sign image
   sx (bf16 ±1, weight-gradient operand) and sx4 (e2m1 ±1 nibbles, forward
   operand); packed sign bits only for the XNOR fallback;
2. ``zk_weight_pack`` latent fp32 kernel → ±1 as e2m1 [T][Cout][Cin/2]
   (forward) and bf16 [T][Cin][Cout] (dgrad);
3. ``zk_igemm_fwd_fp4`` MX-FP4 MFMA implicit GEMM (v_mfma_f32_32x32x64_f8f6f4,
   ±1 exact in e2m1, 4× the bf16 MFMA rate) on an LDS-DMA ring
   (igemm.hip) → exact int16 output (+ optional ReLU) and exact int64 BN
   statistics (``runtime.bconv_fp4=False``: the bf16 MFMA form ``zk_igemm_fwd``;
   ``zk_bconv_fwd``, XNOR-popcount on bit tiles, for channel counts that do
   not tile by 64);
4. ``zk_bn_finalize`` per-channel scale/shift, running statistics (Keras
   momentum, Bessel-corrected variance);
5. ``zk_bn_apply``    out = scale·y + shift + residual, bf16.

Backward: ``zk_bn_bwd_reduce`` (Σg, Σg·ŷ) → ``zk_bn_bwd_coef`` →
``zk_bn_bwd_dx`` (dy, ReLU mask) → ``zk_igemm_dgrad`` (dy ⊛ sign(W)ᵀ with
the input STE mask and the identity-residual gradient fused into its
epilogue) and ``zk_igemm_wgrad`` (dyᵀ ⊛ sx, kernel STE mask in the
epilogue, split-K fp32 atomics straight into the flat gradient buffer).

Saved for backward: the STE mask bits, the sign image (the e2m1 one when
the weight gradient reads it: ``wgrad_reads_fp4``, then no bf16 sign image is
written at all), the int16 conv output and per-channel vectors — no bf16
copy of the real-valued input.
"""

from __future__ import annotations

from typing import Optional

import torch

from zookeeper_amd.nn.layers import same_padding
from zookeeper_amd.ops import streams
from zookeeper_amd.ops.options import OPTS
from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, igemm_wgrad, lib,
                                        stream_ptr, wgrad_rows_ok, zeroed_scratch)


# Copies of the forward BN statistics the conv blocks add into (block b into
# copy b % STAT_STRIPES; zk_bn_finalize sums them): one [2][Cout] array took
# thousands of serialised int64 atomics per cache line on the 56x56 layers.
STAT_STRIPES = 32
# Variant switch (ops/options.py, set through the Runtime component):
#   bconv_fp4  -- binary forward on MX-FP4 MFMA (4x the bf16 rate); off: the
#                 bf16 MFMA form (same exact integer outputs).
# The BN-backward reduction of a block whose output only feeds the next
# block's identity shortcut + 64-channel conv is done in that block's
# row-window dgrad epilogue (runtime.dgrad_rw, zk_igemm_dgrad_bnsum), which
# writes exactly this gradient.


def bwd_stripes() -> int:
    """Copies of the BN-backward sums: one per reduce block (plain stores,
    summed in a fixed order by zk_bn_bwd_coef), in every mode.  The sums feed
    the BN coefficients of the whole data-gradient chain below the layer;
    with fp32 atomics their run-to-run rounding noise was amplified by the
    binary blocks into O(1) gradient differences (profiles/r3/g_dp_forced_diag.md).
    The copies cost 512 x 2 x C floats of plain stores + one read."""
    return int(lib().zk_bn_bwd_reduce_blocks())


def _fp4() -> bool:
    return OPTS.bconv_fp4


def _geom(B, H, W, Cin, Cout, kh, kw, stride):
    """(B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl) of a 'same' conv."""
    pt, pb = same_padding(H, kh, stride)
    pl, pr = same_padding(W, kw, stride)
    Ho, Wo = (H + pt + pb - kh) // stride + 1, (W + pl + pr - kw) // stride + 1
    return (B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl)


def wgrad_reads_fp4(geom) -> bool:
    """Whether a binary conv's weight gradient reads the e2m1 sign image the
    MX-FP4 forward already has (``zk_wgrad_rows`` operand 2, expanded to bf16
    in LDS) instead of a bf16 +-1 image: FP4 forward, ``runtime.wgrad_fp4``
    and a layer the row kernel takes (3x3 stride 1, 64 / 128-channel stages)."""
    B, H, W, Cin, Ho, Wo, Cout = geom[:7]
    return (OPTS.bconv_fp4 and OPTS.wgrad_fp4 and Cin % 64 == 0 and Cout % 64 == 0
            and wgrad_rows_ok(geom))


def bf16_sign_needed(consumer=None, shape=None) -> bool:
    """Whether the producer of a binary block's input (a BN epilogue, the
    stem) must also write the bf16 +-1 sign image, the weight gradient's
    operand.  ``consumer``: the binary ``QuantConv2d`` that reads the tensor
    (unknown: needed); ``shape``: the tensor's NHWC shape.  Not needed when
    that conv's weight gradient reads the e2m1 image (:func:`wgrad_reads_fp4`);
    a consumer that needs it after all re-quantises its input (correct, one
    extra pass)."""
    if consumer is None or shape is None:
        return True
    B, H, W, C = shape
    kh, kw = consumer.kernel_size
    geom = _geom(B, H, W, C, consumer.weight.shape[0], kh, kw, consumer.stride[0])
    return not (consumer.padding == "same" and consumer.stride[0] == consumer.stride[1]
                and wgrad_reads_fp4(geom))


class _BnSum:
    """What the successor's dgrad needs to reduce this block's BN gradient:
    the BN input (the int16 conv output of a binary block, or the bf16 pooled
    tensor of the stem: ``bf16``), BN mean / rstd, the striped sums buffer,
    and (set by the successor's backward) the dx it reduced and its version."""

    __slots__ = ("y", "mean", "rstd", "sums", "bf16", "dx", "dx_version")

    def __init__(self, y, mean, rstd, sums, bf16: bool = False):
        self.y, self.mean, self.rstd, self.sums = y, mean, rstd, sums
        self.bf16 = bool(bf16)
        self.dx = self.dx_version = None

    def reduced(self, dout: torch.Tensor) -> bool:
        """True if the successor's epilogue reduced exactly ``dout``: the
        same storage (``self.dx`` holds it, so no other tensor can reuse the
        address), not modified since (autograd accumulates a second
        consumer's gradient in place, bumping the version counter, or into
        a new tensor)."""
        ok = (self.dx is not None and dout.data_ptr() == self.dx.data_ptr()
              and dout._version == self.dx_version)
        self.dx = None
        return ok


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    """NCHW-shaped tensor → contiguous NHWC storage (no copy if channels_last)."""
    return t.permute(0, 2, 3, 1).contiguous()


class _BinaryBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, gamma, beta, bn, meta):
        (stride, act_relu, clip, pad_ones, identity, will_backward, next_sign, side) = meta
        B, Cin, H, W = x.shape
        Cout, _, kh, kw = weight.shape
        T = kh * kw
        pt, pb = same_padding(H, kh, stride)
        pl, pr = same_padding(W, kw, stride)
        Ho, Wo = (H + pt + pb - kh) // stride + 1, (W + pl + pr - kw) // stride + 1
        dev = x.device
        st = stream_ptr(dev)
        L = lib()

        xn = _nhwc(x)
        nwords = B * H * W * Cin // 32
        # MFMA path (igemm.hip) for channel counts that tile by 64: the
        # forward and both gradients run as bf16 ±1 implicit GEMMs on the
        # sign image sx; otherwise the XNOR-popcount forward on packed bits.
        # (K = kh*kw*Cin <= 32767: the exact dot product is stored as int16)
        mfma = (Cout % 64 == 0 and Cin % 64 == 0 and stride <= 2 and kh <= 4 and kw <= 4
                and kh * kw * Cin <= 32767)
        FP4 = _fp4()
        fp4 = mfma and FP4
        # weight gradient on the e2m1 image (no bf16 sign image at all)
        wfp4 = fp4 and will_backward and wgrad_reads_fp4(
            (B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl))
        # The previous block may already have quantised this input in its BN
        # epilogue (zk_bn_apply_sign): reuse its sign images and STE mask.
        cached = getattr(x, "_zk_sign", None)
        sx4 = None
        need_sx = mfma and not wfp4  # bf16 sign image (wgrad / bf16 fwd)
        if (mfma and cached is not None and cached[0] == clip
                and tuple(cached[2].shape) == (B * H * W * Cin // 32,)
                and (not need_sx or cached[1] is not None)
                and (not fp4 or (len(cached) > 3 and cached[3] is not None))):
            bits, sx, mask = None, cached[1], cached[2]
            sx4 = cached[3] if fp4 else None
        else:
            bits = None if mfma else torch.empty(nwords, dtype=torch.int32, device=dev)
            mask = torch.empty(nwords, dtype=torch.int32, device=dev)
            # bf16 image: the weight-gradient operand (and the bf16 forward's)
            sx = (torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
                  if need_sx and (will_backward or not fp4) else None)
            sx4 = (torch.empty((B, H, W, Cin // 2), dtype=torch.uint8, device=dev)
                   if fp4 else None)
            check(L.zk_sign_pack(xn.data_ptr(), bits.data_ptr() if bits is not None else None,
                                 mask.data_ptr(), sx.data_ptr() if sx is not None else None,
                                 sx4.data_ptr() if sx4 is not None else None, nwords, clip, st),
                  "zk_sign_pack")

        w_ohwi = weight.permute(0, 2, 3, 1).contiguous()  # no copy for channels_last
        wbits = None if mfma else torch.empty(Cout * T * Cin // 32, dtype=torch.int32, device=dev)
        wpop = None if mfma else torch.empty(Cout * T, dtype=torch.int32, device=dev)
        # ±1 kernel as [T][Cout][Cin] (forward GEMM: e2m1 nibbles, or bf16)
        # and transposed to [T][Cin][Cout] bf16 for the dgrad GEMM (only when
        # a backward will run).
        wf = (torch.empty((T, Cout, Cin), dtype=torch.bfloat16, device=dev)
              if mfma and not fp4 else None)
        wf4 = torch.empty((T, Cout, Cin // 2), dtype=torch.uint8, device=dev) if fp4 else None
        wt = (torch.empty((T, Cin, Cout), dtype=torch.bfloat16, device=dev)
              if will_backward else None)
        _p = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        check(L.zk_weight_pack(w_ohwi.data_ptr(), _p(wbits), _p(wpop), _p(wt), _p(wf), _p(wf4),
                               Cout, T, Cin, st), "zk_weight_pack")

        P = B * Ho * Wo
        y = torch.empty((B, Ho, Wo, Cout), dtype=torch.int16, device=dev)
        # persistent accumulator, re-zeroed by zk_bn_finalize (eval: no finalize)
        stats = (zeroed_scratch(bn, "stats_i64", (STAT_STRIPES, 2, Cout), torch.int64, dev)
                 if bn.training
                 else torch.zeros((STAT_STRIPES, 2, Cout), dtype=torch.int64, device=dev))
        if fp4:
            check(L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(),
                                     stats.data_ptr(), B, H, W, Cin, Cout, kh, kw, stride, pt, pl,
                                     Ho, Wo, int(pad_ones), int(act_relu), -1, STAT_STRIPES,
                                     st), "zk_igemm_fwd_fp4")
        elif mfma:
            check(L.zk_igemm_fwd(sx.data_ptr(), wf.data_ptr(), y.data_ptr(), stats.data_ptr(), B,
                                 H, W, Cin, Cout, kh, kw, stride, pt, pl, Ho, Wo, int(pad_ones),
                                 int(act_relu), -1, STAT_STRIPES, st), "zk_igemm_fwd")
        else:
            check(L.zk_bconv_fwd(bits.data_ptr(), wbits.data_ptr(), wpop.data_ptr(),
                                 y.data_ptr(), stats.data_ptr(), B, H, W, Cin, Cout, kh, kw,
                                 stride, pt, pl, Ho, Wo, int(pad_ones), int(act_relu), st),
                  "zk_bconv_fwd")
        if not will_backward:
            sx = sx4 = None

        scale = torch.empty(Cout, dtype=torch.float32, device=dev)
        shift = torch.empty_like(scale)
        mean = torch.empty_like(scale)
        rstd = torch.empty_like(scale)
        gp = gamma.data_ptr() if gamma is not None else None
        bp = beta.data_ptr() if beta is not None else None
        if bn.training:
            # (the XNOR kernel adds into copy 0 only; the others stay zero)
            check(L.zk_bn_finalize(stats.data_ptr(), Cout, STAT_STRIPES, float(P), gp, bp, bn.eps, bn.momentum,
                                   bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                   scale.data_ptr(), shift.data_ptr(), mean.data_ptr(),
                                   rstd.data_ptr(), st), "zk_bn_finalize")
        else:
            rstd.copy_(torch.rsqrt(bn.running_var + bn.eps))
            mean.copy_(bn.running_mean)
            g_ = gamma if gamma is not None else torch.ones_like(rstd)
            b_ = beta if beta is not None else torch.zeros_like(rstd)
            scale.copy_(g_ * rstd)
            shift.copy_(b_ - mean * scale)

        res = xn if identity else (_nhwc(residual) if residual is not None else None)
        out = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=dev)
        if next_sign is not None and Cout % 64 == 0:
            # also quantise the output for the next binary block (same clip)
            sx_next = (torch.empty_like(out)
                       if bf16_sign_needed(side.get("sign_consumer"), (B, Ho, Wo, Cout)) else None)
            mask_next = torch.empty(P * Cout // 32, dtype=torch.int32, device=dev)
            sx4_next = (torch.empty((B, Ho, Wo, Cout // 2), dtype=torch.uint8, device=dev)
                        if FP4 else None)
            pool_box = side.get("pool_out")
            if pool_box is not None and Ho % 2 == 0 and Wo % 2 == 0:
                # the next block's shortcut pools this output 2x2/2: in this pass
                pooled = torch.empty((B, Ho // 2, Wo // 2, Cout), dtype=torch.bfloat16,
                                     device=dev)
                check(L.zk_bn_apply_sign_pool(
                    y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                    res.data_ptr() if res is not None else None, out.data_ptr(),
                    sx_next.data_ptr() if sx_next is not None else None, mask_next.data_ptr(),
                    sx4_next.data_ptr() if sx4_next is not None else None, clip,
                    pooled.data_ptr(), B, Ho, Wo, Cout, st), "zk_bn_apply_sign_pool")
                pool_box.append(pooled)
            else:
                check(L.zk_bn_apply_sign(y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                         res.data_ptr() if res is not None else None,
                                         out.data_ptr(),
                                         sx_next.data_ptr() if sx_next is not None else None,
                                         mask_next.data_ptr(),
                                         sx4_next.data_ptr() if sx4_next is not None else None,
                                         clip, P, Cout, st), "zk_bn_apply_sign")
            next_sign[:] = [clip, sx_next, mask_next, sx4_next]
        else:
            check(L.zk_bn_apply(y.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                res.data_ptr() if res is not None else None, out.data_ptr(), P,
                                Cout, st), "zk_bn_apply")

        # BN-backward fusion hand-off: this block's reduction may be done by
        # its successor's row-window dgrad (64 channels, W <= 64: its
        # persistent blocks add the sums once per block); the predecessor's
        # by this block.
        ctx.bnsum = None
        rw_out = OPTS.dgrad_rw and Cout == 64 and Wo <= 64
        if rw_out and not OPTS.deterministic and will_backward and bn.training:
            # one copy per row-window block (fixed-order combination, below
            # the reduce's 512 copies): the same buffer as the separate reduce
            sums_buf = zeroed_scratch(bn, "bwd_sums", (2, Cout, bwd_stripes()), torch.float32,
                                      dev)
            ctx.bnsum = _BnSum(y, mean, rstd, sums_buf)
            side["bnsum"] = ctx.bnsum
        pred = side.get("pred")
        rw_in = (OPTS.dgrad_rw and Cin == 64 and Cout == 64 and stride == 1 and kh == kw == 3
                 and W <= 64 and pt == pl == 1)
        ctx.pred = (pred if (pred is not None and identity and mfma
                             and rw_in
                             and tuple(pred.y.shape) == (B, H, W, Cin)) else None)
        ctx.save_for_backward(bits, mask, wt, y, mean, rstd, gamma, w_ohwi, sx, sx4)
        ctx.params = (weight, gamma, beta)
        ctx.geom = (B, Cin, H, W, Cout, kh, kw, stride, pt, pb, pl, pr, Ho, Wo)
        ctx.wfp4 = wfp4
        ctx.meta = meta
        ctx.bn = bn
        ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
        ctx.has_residual = residual is not None and not identity
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        bits, mask, wt, y, mean, rstd, gamma, w_ohwi, sx, sx4 = ctx.saved_tensors
        (B, Cin, H, W, Cout, kh, kw, stride, pt, pb, pl, pr, Ho, Wo) = ctx.geom
        (_, act_relu, clip, pad_ones, identity, _, _, _) = ctx.meta
        dev = dout.device
        st = stream_ptr(dev)
        L = lib()
        P = B * Ho * Wo

        g = _nhwc(dout.to(torch.bfloat16))
        weight_p, gamma_p, beta_p = ctx.params
        # deterministic mode: one copy of the sums per reduce block (plain
        # stores, fixed-order sum in zk_bn_bwd_coef) instead of striped atomics
        stripes = bwd_stripes()
        # channel-major copies [2][C][stripes]: zk_bn_bwd_coef reads each
        # channel's copies as one contiguous row
        sums = zeroed_scratch(ctx.bn, "bwd_sums", (2, Cout, stripes), torch.float32, dev)
        bs = ctx.bnsum
        fused = bs is not None and bs.dx is not None
        # BN coefficients + gamma/beta gradients; gradients go straight into
        # the flat gradient buffer when the trainer manages it.
        dg_direct = direct_grad(gamma_p) if ctx.has_gamma else None
        db_direct = direct_grad(beta_p) if ctx.has_beta else None
        dgamma = dg_direct if dg_direct is not None else (
            torch.zeros(Cout, device=dev) if ctx.has_gamma else None)
        dbeta = db_direct if db_direct is not None else (
            torch.zeros(Cout, device=dev) if ctx.has_beta else None)
        coef = torch.empty((3, Cout), dtype=torch.float32, device=dev)
        if not (fused and bs.reduced(dout)):
            if fused:
                sums.zero_()  # the successor reduced a gradient that was accumulated later
            check(L.zk_bn_bwd_reduce(g.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                     rstd.data_ptr(), sums.data_ptr(), P, Cout, stripes, st),
                  "zk_bn_bwd_reduce")
        # else: the successor's dgrad epilogue reduced exactly this gradient
        check(L.zk_bn_bwd_coef(sums.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                               gamma.data_ptr() if gamma is not None else None, float(P),
                               Cout, stripes, stripes, coef.data_ptr(),
                               dgamma.data_ptr() if dgamma is not None else None,
                               dbeta.data_ptr() if dbeta is not None else None, st),
              "zk_bn_bwd_coef")
        if dg_direct is not None:
            grad_ready(gamma_p)
            dgamma = None
        if db_direct is not None:
            grad_ready(beta_p)
            dbeta = None
        dy = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=dev)
        check(L.zk_bn_bwd_dx(g.data_ptr(), y.data_ptr(), coef.data_ptr(), dy.data_ptr(), P,
                             Cout, int(act_relu), st), "zk_bn_bwd_dx")

        need_dx = ctx.needs_input_grad[0]
        native = Cout % 64 == 0 and Cin % 64 == 0 and stride <= 2 and kh <= 4 and kw <= 4
        dx = None
        if native:
            # weight gradient first: on the side stream (ops/streams.py) it
            # then overlaps this block's dgrad and the next block's backward
            w_direct = direct_grad(weight_p, channels_last=True)
            dweight = None
            # weight-gradient sign operand: the bf16 image, or the e2m1 one
            sxw, operand = (sx4, "fp4") if ctx.wfp4 else (sx, "image")
            side = streams.active() and w_direct is not None and sxw is not None
            if side:
                sstream = streams.side_stream(dev)
                ready = torch.cuda.Event()
                ready.record()  # dy written (compute stream)
                sstream.wait_event(ready)
                with torch.cuda.stream(sstream):
                    _wgrad(L, dy, sxw, w_ohwi, w_direct.permute(0, 2, 3, 1), ctx,
                           sstream.cuda_stream, operand)
                    done = torch.cuda.Event()
                    done.record(sstream)
                streams.keep(dy, sxw, w_ohwi)  # released once the compute stream joins
            else:
                dw = (w_direct.permute(0, 2, 3, 1) if w_direct is not None  # OHWI view
                      else torch.zeros((Cout, kh, kw, Cin), dtype=torch.float32, device=dev))
                if sxw is not None:
                    _wgrad(L, dy, sxw, w_ohwi, dw, ctx, st, operand)
                else:
                    check(L.zk_bconv_wgrad(dy.data_ptr(), bits.data_ptr(), w_ohwi.data_ptr(),
                                           dw.data_ptr(), B, H, W, Cin, Ho, Wo, Cout, kh, kw,
                                           stride, pt, pl, int(pad_ones), clip, 0, -1, st),
                          "zk_bconv_wgrad")
                if w_direct is None:
                    dweight = dw.permute(0, 3, 1, 2)
            # MFMA implicit GEMMs; STE mask + residual gradient fused in dgrad.
            if need_dx:
                dx = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
                dres = g if identity else None
                pred = ctx.pred
                if pred is not None:
                    # + the predecessor's BN-backward sums over this dx
                    check(L.zk_igemm_dgrad_bnsum(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(),
                                                 dres.data_ptr() if dres is not None else None,
                                                 dx.data_ptr(), pred.y.data_ptr(),
                                                 pred.mean.data_ptr(), pred.rstd.data_ptr(),
                                                 pred.sums.data_ptr(), pred.sums.shape[2],
                                                 int(pred.bf16), B, H, W,
                                                 Cin,
                                                 Ho, Wo, Cout, kh, kw, stride, pt, pl, -1, st),
                          "zk_igemm_dgrad_bnsum")
                    pred.dx, pred.dx_version = dx, dx._version
                else:
                    check(L.zk_igemm_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(),
                                           dres.data_ptr() if dres is not None else None,
                                           dx.data_ptr(), B, H, W, Cin, Ho, Wo, Cout, kh, kw,
                                           stride, pt, pl, -1, st), "zk_igemm_dgrad")
                handoff = ctx.meta[7].get("dx_handoff")
                if handoff is not None and handoff.give(dx):
                    # x's other consumer (the shortcut's avg-pool) adds it in
                    # its backward, which runs after this one
                    dx = None
                else:
                    dx = dx.permute(0, 3, 1, 2)
            if side:
                # earlier blocks' side-stream wgrads: signal their readiness
                # (the bucketer's comm stream waits for their events; the
                # compute stream only at the end of the backward)
                streams.flush(wait=False)
                streams.defer_ready(done, weight_p)
            elif w_direct is not None:
                grad_ready(weight_p)
        else:
            dx, dweight = _library_conv_backward(ctx, dy, g, bits, mask, wt, w_ohwi, need_dx)
        dres_out = dout if ctx.has_residual else None
        return dx, dres_out, dweight, dgamma, dbeta, None, None


def _wgrad(L, dy, sx, w_ohwi, dw, ctx, st, operand: str = "image") -> None:
    """Binary-conv weight gradient (dyᵀ ⊛ sign(x), kernel STE mask) added
    into ``dw`` (OHWI fp32) on stream ``st`` (split-K reduction:
    ``_native.igemm_wgrad``); ``sx`` the bf16 sign image, or the e2m1 one
    with ``operand="fp4"``."""
    (B, Cin, H, W, Cout, kh, kw, stride, pt, pb, pl, pr, Ho, Wo) = ctx.geom
    (_, _, clip, pad_ones) = ctx.meta[:4]
    igemm_wgrad(dy, sx, w_ohwi, dw, (B, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pt, pl),
                int(pad_ones), clip, st, operand=operand)


def _library_conv_backward(ctx, dy, g, bits, mask, wt, w_ohwi, need_dx):
    """Fallback for channel counts the MFMA kernels do not tile (Cin or Cout
    not a multiple of 64): bf16 library convolution backward on unpacked ±1
    operands, then the fused STE/residual kernel."""
    (B, Cin, H, W, Cout, kh, kw, stride, pt, pb, pl, pr, Ho, Wo) = ctx.geom
    (_, _, clip, pad_ones, identity) = ctx.meta[:5]
    dev = dy.device
    st = stream_ptr(dev)
    L = lib()
    xs = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
    check(L.zk_unpack_sign(bits.data_ptr(), xs.data_ptr(), bits.numel(), st), "zk_unpack_sign")
    xs_nchw = xs.permute(0, 3, 1, 2)
    w_nchw = wt.permute(2, 1, 0).reshape(Cout, Cin, kh, kw).contiguous(
        memory_format=torch.channels_last)
    symmetric = (pt == pb and pl == pr) and not pad_ones
    if symmetric:
        inp, pad = xs_nchw, (pt, pl)
    else:
        inp = torch.nn.functional.pad(xs_nchw, (pl, pr, pt, pb), value=1.0 if pad_ones else 0.0)
        inp = inp.contiguous(memory_format=torch.channels_last)
        pad = (0, 0)
    dgrad, dw, _ = torch.ops.aten.convolution_backward(
        dy.permute(0, 3, 1, 2), inp, w_nchw, None, (stride, stride), pad, (1, 1), False,
        (0, 0), 1, (need_dx, True, False))
    dx = None
    if need_dx:
        if not symmetric:
            dgrad = dgrad[:, :, pt:pt + H, pl:pl + W]
        dgn = _nhwc(dgrad)
        dx = torch.empty((B, H, W, Cin), dtype=torch.bfloat16, device=dev)
        dres = g if identity else None
        check(L.zk_ste_combine(dgn.data_ptr(), mask.data_ptr(),
                               dres.data_ptr() if dres is not None else None, dx.data_ptr(),
                               dx.numel(), st), "zk_ste_combine")
        dx = dx.permute(0, 3, 1, 2)
    w = w_ohwi.permute(0, 3, 1, 2)
    dweight = dw.float() * (w.abs() <= clip).to(torch.float32)
    return dx, dweight


def binary_block(x: torch.Tensor, residual: Optional[torch.Tensor], conv, bn,
                 act: Optional[str] = None, clip_value: float = 1.0,
                 pad_value: float = 0.0, quantize_output: bool = True,
                 dx_handoff=None, sign_consumer=None, pool_out: bool = False) -> torch.Tensor:
    """Run ``bn(act(conv(x))) + residual`` with the fused HIP kernels.

    ``conv`` must be a binary ``QuantConv2d`` (ste_sign input and kernel,
    ``same`` padding), ``bn`` a :class:`~zookeeper_amd.nn.BatchNorm`.
    ``residual`` may be ``x`` itself (identity shortcut, fused into the
    backward) or a separately computed tensor, or ``None``.

    With ``quantize_output`` the BN epilogue also writes the sign images
    (bf16 and e2m1) and STE mask of the output for the next binary block
    (attached to the returned tensor as ``_zk_sign`` = (clip, sx, mask, sx4);
    a block with the same clip value reuses them instead of re-reading its
    input).

    ``sign_consumer``: the binary conv that reads the output's sign images
    (the next block's); the bf16 sign image is skipped when its weight
    gradient reads the e2m1 one (:func:`bf16_sign_needed`).

    ``pool_out``: the output's consumer also 2x2/2-average-pools it (the next
    block's downsampling shortcut): the BN epilogue writes that pooled image
    in the same pass, attached as ``_zk_pooled`` for ``ops.norm_pool.avg_pool2``.

    ``dx_handoff`` (an ``ops.norm_pool.ResidualHandoff``): x's gradient is left
    there instead of returned, for x's other consumer whose backward runs
    after this one and adds it (a stage transition's shortcut
    ``avg_pool2(x, handoff=...)``), saving autograd's separate add pass.
    """
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if x.shape[1] % 32 or conv.weight.shape[0] % 8:
        raise ValueError("binary_block needs Cin % 32 == 0 and Cout % 8 == 0")
    if conv.stride[0] != conv.stride[1]:
        raise ValueError("binary_block needs a square stride")
    if conv.weight.shape[1] * conv.weight.shape[2] * conv.weight.shape[3] > 32767:
        raise ValueError("binary_block needs kh*kw*Cin <= 32767 (exact int16 conv output)")
    for name, t in (("conv.weight", conv.weight), ("bn.weight", bn.weight),
                    ("residual", residual)):
        if t is not None and t.device != x.device:
            # a host pointer handed to a kernel faults the GPU instead of raising
            raise ValueError(f"binary_block: {name} is on {t.device}, the input on {x.device}")
    identity = residual is x
    if residual is not None and not identity and residual.dtype != torch.bfloat16:
        residual = residual.to(torch.bfloat16)
    will_backward = torch.is_grad_enabled() and (
        x.requires_grad or conv.weight.requires_grad or bn.training)
    holder: list = [] if quantize_output else None
    side = {"pred": getattr(x, "_zk_bnsum", None), "dx_handoff": dx_handoff,
            "sign_consumer": sign_consumer,
            "pool_out": [] if (pool_out and OPTS.bn_pool_fuse) else None}
    meta = (conv.stride[0], act == "relu", float(clip_value), pad_value == 1.0, identity,
            will_backward, holder, side)
    out = _BinaryBlockFn.apply(x, None if identity else residual, conv.weight, bn.weight,
                               bn.bias, bn, meta)
    if holder:
        # consumed by the next binary block (same clip) instead of re-reading out
        out._zk_sign = tuple(holder)
    if side.get("bnsum") is not None:
        out._zk_bnsum = side["bnsum"]
    if side["pool_out"]:
        out._zk_pooled = (side["pool_out"][0], out._version)
    return out
