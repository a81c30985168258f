"""BatchNorm(+ReLU) and pooling on bf16 NHWC tensors (HIP kernels in
``csrc/kernels/norm_pool.hip``), as autograd functions.

Tensors are NCHW-*shaped* with ``channels_last`` strides (physically NHWC),
the layout every model in the zoo uses.
"""

from __future__ import annotations

import ctypes

import torch

from zookeeper_amd.nn.layers import same_padding
from zookeeper_amd.ops.options import OPTS
from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, lib, stream_ptr,
                                        zeroed_scratch)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1).contiguous() if t.dim() == 4 else t.contiguous()


def _back(t: torch.Tensor, like_dim: int) -> torch.Tensor:
    return t.permute(0, 3, 1, 2) if like_dim == 4 else t


def supported(x: torch.Tensor) -> bool:
    # the kernels are instantiated for C/8 a power of two (ZK_CG_CASES in
    # norm_pool.hip): e.g. a 1000-way classifier's BN stays on the formula path
    cg = x.shape[1] // 8 if x.dim() >= 2 else 0
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() in (2, 4)
            and x.shape[1] % 8 == 0 and 1 <= cg <= 256 and cg & (cg - 1) == 0)


class FloatBnSum:
    """Hand-off of a float BatchNorm's backward reduction to the data gradient
    of the layer that consumes its output (``pointwise.conv1x1``,
    ``conv3x3``): that kernel's LDS epilogue writes (sum g', sum g' * xhat)
    over each of its M tiles of the gradient it stores into ``sums``
    [tiles][2][C] (plain stores, one row per tile; ``zk_bn_bwd_tiles_reduce``
    folds the rows in a fixed order -- bit-reproducible -- into the copies
    ``zk_bn_bwd_coef`` reads, and re-zeroes them), with
    g' masked by the BN's ReLU (``relu``: 0 none, 1 recomputed from the input
    ``xn`` and ``coef``, 2 the stored ``mask`` bits).
    The BN backward uses them only if they were taken over exactly the
    gradient it receives (:meth:`reduced`: same storage, not modified since);
    otherwise it re-zeroes ``sums`` and runs its own reduction."""

    __slots__ = ("xn", "coef", "mask", "relu", "sums", "dx", "dx_version")

    def __init__(self, xn, coef, mask, relu: int, sums):
        self.xn, self.coef, self.mask, self.relu, self.sums = xn, coef, mask, relu, sums
        self.dx = self.dx_version = None

    def take(self, dx) -> None:
        """Consumer side: the sums were added over ``dx`` (its final value)."""
        self.dx, self.dx_version = dx, dx._version

    def reduced(self, dout: torch.Tensor) -> bool:
        ok = (self.dx is not None and dout.data_ptr() == self.dx.data_ptr()
              and dout._version == self.dx_version)
        used = self.dx is not None
        self.dx = None
        if used and not ok:
            self.sums.zero_()  # added over another gradient: not this BN's
        return ok


class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, residual, bn, relu, handoff=None, holder=None):
        dim = x.dim()
        C = x.shape[1]
        xn = _nhwc(x)
        P = xn.numel() // C
        dev = x.device
        st = stream_ptr(dev)
        L = lib()
        coef = torch.empty((4, C), dtype=torch.float32, device=dev)
        pend = bn.__dict__.pop("_zk_pending_fstats", None)
        if pend is not None and not (bn.training and pend[1] == xn.data_ptr()):
            pend[0].zero_()  # produced for another tensor: unused, keep the buffer zero
            pend = None
        if pend is not None:
            # statistics the producing GEMM's epilogue added up
            # (pointwise.conv1x1(stats_for=bn)); the finalize re-zeroes them
            parts, _, nparts = pend
            check(L.zk_bn_finalize_f64_stripes(parts.data_ptr(), nparts, C, float(P),
                                               gamma.data_ptr() if gamma is not None else None,
                                               beta.data_ptr() if beta is not None else None,
                                               bn.eps, bn.momentum, bn.running_mean.data_ptr(),
                                               bn.running_var.data_ptr(), coef.data_ptr(), st),
                  "zk_bn_finalize_f64_stripes")
        elif bn.training and OPTS.deterministic:
            # per-block partials, summed in block order (no fp64 atomics)
            parts = torch.empty((L.zk_bn_bwd_parts_max(), 2, C), dtype=torch.float64, device=dev)
            n = ctypes.c_int(0)
            check(L.zk_bn_stats_bf16_parts(xn.data_ptr(), parts.data_ptr(), P, C, ctypes.byref(n),
                                           st), "zk_bn_stats_bf16_parts")
            check(L.zk_bn_finalize_f64_parts(parts.data_ptr(), n.value, C, float(P),
                                             gamma.data_ptr() if gamma is not None else None,
                                             beta.data_ptr() if beta is not None else None,
                                             bn.eps, bn.momentum, bn.running_mean.data_ptr(),
                                             bn.running_var.data_ptr(), coef.data_ptr(), st),
                  "zk_bn_finalize_f64_parts")
        elif bn.training:
            sums = zeroed_scratch(bn, "stats_f64", (2, C), torch.float64, dev)
            check(L.zk_bn_stats_bf16(xn.data_ptr(), sums.data_ptr(), P, C, st), "zk_bn_stats_bf16")
            check(L.zk_bn_finalize_f64(sums.data_ptr(), C, float(P),
                                       gamma.data_ptr() if gamma is not None else None,
                                       beta.data_ptr() if beta is not None else None,
                                       bn.eps, bn.momentum, bn.running_mean.data_ptr(),
                                       bn.running_var.data_ptr(), coef.data_ptr(), st),
                  "zk_bn_finalize_f64")
        else:
            rstd = torch.rsqrt(bn.running_var + bn.eps)
            g = gamma if gamma is not None else torch.ones_like(rstd)
            b = beta if beta is not None else torch.zeros_like(rstd)
            coef[0] = g * rstd
            coef[1] = b - bn.running_mean * coef[0]
            coef[2] = bn.running_mean
            coef[3] = rstd
        y = torch.empty_like(xn)
        omask = None
        if residual is not None:
            rn = _nhwc(residual.to(torch.bfloat16))
            # BN + residual + ReLU: the backward needs the output's ReLU mask,
            # which x alone does not give: 1 bit per element, not the output
            omask = (torch.empty((P, C // 8), dtype=torch.uint8, device=dev)
                     if relu and any(ctx.needs_input_grad) else None)
            check(L.zk_bn_apply_res_bf16(xn.data_ptr(), coef.data_ptr(), rn.data_ptr(),
                                         y.data_ptr(),
                                         omask.data_ptr() if omask is not None else None, P, C,
                                         int(relu), st), "zk_bn_apply_res_bf16")
        else:
            check(L.zk_bn_apply_bf16(xn.data_ptr(), coef.data_ptr(), y.data_ptr(), P, C, int(relu),
                                     st), "zk_bn_apply_bf16")
        ctx.has_res = residual is not None
        ctx.handoff = handoff if residual is not None else None
        # BN + ReLU without a residual keeps no output: the backward kernels
        # recompute the ReLU mask from x (one read less in each of them)
        ctx.relu_rc = relu and residual is None
        ctx.save_for_backward(xn, omask, coef, gamma)
        # backward reduction handed to the consumer's data-gradient epilogue
        ctx.fsum = None
        if (holder is not None and bn.training and not OPTS.deterministic and OPTS.bn_bwd_fuse
                and any(ctx.needs_input_grad)):
            mode = 2 if omask is not None else (1 if relu else 0)
            if not (relu and residual is not None and omask is None):
                # one row per M tile of the consumer's LDS-epilogue GEMM (>= 128 pixels)
                tiles = (P + 127) // 128
                sums = zeroed_scratch(bn, "bwd_sums_fused", (tiles, 2, C), torch.float32, dev)
                ctx.fsum = FloatBnSum(xn, coef, omask, mode, sums)
                holder.append(ctx.fsum)
        ctx.params = (gamma, beta)
        ctx.dim, ctx.P, ctx.C = dim, P, C
        ctx.bn = bn
        ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
        return _back(y, dim)

    @staticmethod
    def backward(ctx, dy):
        xn, m, coef, gamma = ctx.saved_tensors
        P, C = ctx.P, ctx.C
        dev = dy.device
        st = stream_ptr(dev)
        L = lib()
        g = _nhwc(dy.to(torch.bfloat16))
        # per-block partials (plain stores), summed in block order by
        # zk_bn_bwd_coef (stripes = parts): bit-reproducible in every mode --
        # these sums set the BN coefficients of the whole gradient chain below
        # (and fp32 atomics of 512 blocks into one [2][C] row also contend)
        # channel-major copies [2][C][parts_max]
        sums = torch.empty((2, C, L.zk_bn_bwd_parts_max()), dtype=torch.float32, device=dev)
        n = ctypes.c_int(0)
        fused = ctx.fsum is not None and ctx.fsum.reduced(g)
        if fused:
            # the consumer's data-gradient epilogue reduced exactly this g
            rows = ctx.fsum.sums
            check(L.zk_bn_bwd_tiles_reduce(rows.data_ptr(), rows.shape[0], C, sums.data_ptr(), st),
                  "zk_bn_bwd_tiles_reduce")
            n.value = sums.shape[2]
        elif ctx.relu_rc:
            check(L.zk_bn_bwd_reduce_relu_bf16_parts(g.data_ptr(), xn.data_ptr(),
                                                     coef.data_ptr(), sums.data_ptr(), P, C,
                                                     ctypes.byref(n), st),
                  "zk_bn_bwd_reduce_relu_bf16_parts")
        else:
            check(L.zk_bn_bwd_reduce_bf16_parts(g.data_ptr(), xn.data_ptr(),
                                                m.data_ptr() if m is not None else None,
                                                coef.data_ptr(), sums.data_ptr(), P, C,
                                                ctypes.byref(n), st),
                  "zk_bn_bwd_reduce_bf16_parts")
        stripes = n.value
        gamma_p, beta_p = ctx.params
        dg_direct = direct_grad(gamma_p) if ctx.has_gamma else None
        db_direct = direct_grad(beta_p) if ctx.has_beta else None
        dgamma = dg_direct if dg_direct is not None else (
            torch.zeros(C, device=dev) if ctx.has_gamma else None)
        dbeta = db_direct if db_direct is not None else (
            torch.zeros(C, device=dev) if ctx.has_beta else None)
        bcoef = torch.empty((3, C), dtype=torch.float32, device=dev)
        check(L.zk_bn_bwd_coef(sums.data_ptr(), coef[2].data_ptr(), coef[3].data_ptr(),
                               gamma.data_ptr() if gamma is not None else None, float(P), C,
                               stripes, sums.shape[2],
                               bcoef.data_ptr(), dgamma.data_ptr() if dgamma is not None else None,
                               dbeta.data_ptr() if dbeta is not None else None, st),
              "zk_bn_bwd_coef")
        if dg_direct is not None:
            grad_ready(gamma_p)
            dgamma = None
        if db_direct is not None:
            grad_ready(beta_p)
            dbeta = None
        dx = torch.empty_like(g)
        dres = None
        h = ctx.handoff
        if (ctx.has_res and ctx.needs_input_grad[3] and h is not None and h.masked_ok
                and OPTS.bn_masked_handoff and m is not None and not h.closed):
            # the residual's consumer masks g itself (its epilogue reads g and
            # the mask bits): no residual-gradient tensor is written
            check(L.zk_bn_bwd_dx_bf16(g.data_ptr(), xn.data_ptr(), m.data_ptr(),
                                      bcoef.data_ptr(), dx.data_ptr(), P, C, st),
                  "zk_bn_bwd_dx_bf16")
            h.give((g, m))
        elif ctx.has_res and ctx.needs_input_grad[3]:
            dres = torch.empty_like(g)
            check(L.zk_bn_bwd_dx_res_bf16(g.data_ptr(), xn.data_ptr(),
                                          m.data_ptr() if m is not None else None,
                                          bcoef.data_ptr(), dx.data_ptr(), dres.data_ptr(), P, C,
                                          st), "zk_bn_bwd_dx_res_bf16")
            if ctx.handoff is not None and ctx.handoff.give(dres):
                # the residual's consumer adds it in its data-gradient epilogue
                # (see ResidualHandoff): no separate gradient-accumulation pass
                dres = None
            else:
                dres = _back(dres, ctx.dim)
        elif ctx.relu_rc:
            check(L.zk_bn_bwd_dx_relu_bf16(g.data_ptr(), xn.data_ptr(), coef.data_ptr(),
                                           bcoef.data_ptr(), dx.data_ptr(), P, C, st),
                  "zk_bn_bwd_dx_relu_bf16")
        else:
            check(L.zk_bn_bwd_dx_bf16(g.data_ptr(), xn.data_ptr(),
                                      m.data_ptr() if m is not None else None, bcoef.data_ptr(),
                                      dx.data_ptr(), P, C, st), "zk_bn_bwd_dx_bf16")
        return _back(dx, ctx.dim), dgamma, dbeta, dres, None, None, None, None


class ResidualHandoff:
    """Gradient hand-off between a residual block's tail and the first layer
    of its main path when both read the same tensor ``x`` (an identity
    shortcut).  Autograd would sum the two gradients of ``x`` in a separate
    elementwise pass (read both, write the sum); instead the tail's backward
    (which runs first: the main path feeds it) leaves the shortcut's gradient
    here and returns none for it, and the first layer's data-gradient kernel
    adds it in its epilogue (``zk_igemm_dgrad``'s ``dres``).  Only valid when
    that first layer computes the full gradient of ``x`` — the caller pairs a
    handoff with a native layer it knows consumes it.

    The same object serves any producer / consumer pair whose backward order
    follows from the graph (a stage transition's binary conv → its shortcut
    avg-pool, a downsampling bottleneck's conv1 → its shortcut conv).
    ``take`` closes it: a producer that would run after its consumer
    (``give`` returns False) returns its gradient to autograd instead, so an
    unexpected order costs the fused add, never a gradient."""

    __slots__ = ("dres", "closed", "masked_ok")

    def __init__(self):
        self.dres = None
        self.closed = False
        # set by a consumer whose epilogue can take the gradient as (g, ReLU
        # mask bits) and mask it itself (pointwise.conv1x1): the BN tail then
        # hands over its incoming gradient and mask instead of writing g*mask
        self.masked_ok = False

    def give(self, d) -> bool:
        """Producer side: leave ``d`` for the consumer; False if it already ran."""
        if self.closed:
            return False
        self.dres = d
        return True

    def take(self):
        """Consumer side: the producer's gradient (or None); closes the hand-off."""
        d, self.dres = self.dres, None
        self.closed = True
        return d


def batch_norm(x: torch.Tensor, bn, relu: bool = False,
               residual: torch.Tensor = None, handoff: ResidualHandoff = None) -> torch.Tensor:
    """``act(bn(x) [+ residual])`` in one pass (forward) / one pass (the
    data gradient, plus the residual's gradient when given — or left in
    ``handoff`` for the residual's other consumer).  In training the output
    carries ``_zk_fbnsum`` (:class:`FloatBnSum`): a consumer that computes
    its whole gradient may reduce the backward sums in its epilogue."""
    holder: list = []
    y = _BatchNormFn.apply(x, bn.weight, bn.bias, residual, bn, relu, handoff, holder)
    if holder:
        y._zk_fbnsum = holder[0]
    return y


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, padding, relu):
        B, C, H, W = x.shape
        if padding == "same":
            pt, pb = same_padding(H, k, s)
            pl, pr = same_padding(W, k, s)
        else:
            pt = pb = pl = pr = 0
        Ho, Wo = (H + pt + pb - k) // s + 1, (W + pl + pr - k) // s + 1
        xn = _nhwc(x)
        y = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=x.device)
        arg = torch.empty((B, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        check(lib().zk_maxpool_fwd(xn.data_ptr(), y.data_ptr(), arg.data_ptr(), B, H, W, C, Ho,
                                   Wo, k, s, pt, pl, int(relu), stream_ptr(x.device)),
              "zk_maxpool_fwd")
        ctx.save_for_backward(arg)
        ctx.geom = (B, H, W, C, Ho, Wo, k, s, pt, pl)
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        B, H, W, C, Ho, Wo, k, s, pt, pl = ctx.geom
        g = _nhwc(dy.to(torch.bfloat16))
        dx = torch.empty((B, H, W, C), dtype=torch.bfloat16, device=dy.device)
        check(lib().zk_maxpool_bwd(g.data_ptr(), arg.data_ptr(), dx.data_ptr(), B, H, W, C, Ho,
                                   Wo, k, s, pt, pl, stream_ptr(dy.device)), "zk_maxpool_bwd")
        return dx.permute(0, 3, 1, 2), None, None, None, None


def max_pool(x: torch.Tensor, k: int, s: int, padding: str = "valid",
             relu: bool = False) -> torch.Tensor:
    """Max pooling; ``relu=True`` returns ``relu(max_pool(x))`` from the same
    pass (no separate ReLU forward / backward launch)."""
    return _MaxPoolFn.apply(x, k, s, padding, relu)


class _AvgPool2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, handoff=None):
        B, C, H, W = x.shape
        Ho, Wo = H // 2, W // 2
        pre = getattr(x, "_zk_pooled", None)
        if (pre is not None and pre[1] == x._version and tuple(pre[0].shape) == (B, Ho, Wo, C)
                and pre[0].dtype == x.dtype and H % 2 == 0 and W % 2 == 0):
            # written by the producer's BN epilogue (ops.binary_block pool_out),
            # bit-identical to this kernel's output
            y = pre[0]
        else:
            xn = _nhwc(x)
            y = torch.empty((B, Ho, Wo, C), dtype=x.dtype, device=x.device)
            check(lib().zk_avgpool2_fwd(xn.data_ptr(), y.data_ptr(), B, H, W, C, Ho, Wo,
                                        stream_ptr(x.device)), "zk_avgpool2_fwd")
        ctx.geom = (B, H, W, C, Ho, Wo)
        ctx.handoff = handoff
        return y.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C, Ho, Wo = ctx.geom
        g = _nhwc(dy.to(torch.bfloat16))
        dx = torch.empty((B, H, W, C), dtype=torch.bfloat16, device=dy.device)
        add = ctx.handoff.take() if ctx.handoff is not None else None
        if add is not None:
            # x's main-path gradient, left by the block that ran first
            if tuple(add.shape) != (B, H, W, C) or not add.is_contiguous():
                raise RuntimeError("avg_pool2: hand-off gradient has the wrong layout")
            check(lib().zk_avgpool2_bwd_add(g.data_ptr(), add.data_ptr(), dx.data_ptr(), B, H, W,
                                            C, Ho, Wo, stream_ptr(dy.device)),
                  "zk_avgpool2_bwd_add")
        else:
            check(lib().zk_avgpool2_bwd(g.data_ptr(), dx.data_ptr(), B, H, W, C, Ho, Wo,
                                        stream_ptr(dy.device)), "zk_avgpool2_bwd")
        return dx.permute(0, 3, 1, 2), None


def avg_pool2(x: torch.Tensor, handoff: "ResidualHandoff" = None) -> torch.Tensor:
    """2x2/2 average pool.  ``handoff``: x's other gradient (left there by a
    consumer whose backward runs first, e.g. ``ops.binary_block`` of a stage
    transition) is added in the backward pass instead of autograd's separate
    add."""
    return _AvgPool2Fn.apply(x, handoff)
