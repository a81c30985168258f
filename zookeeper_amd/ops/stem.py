"""Fused ImageNet stem (``csrc/kernels/stem.hip``):
conv KxK/2 (3 input channels) → BN → ReLU → max-pool 3×3/2 [→ BN].

BinaryResNet-E18 (and ResNet-50 without the trailing BN) spend a fifth of
a training step here when the stem runs as library conv + separate
BN / ReLU / pool passes over the 112×112×64 activation.  The fused version:

forward   pack (zero-padded 4-channel image, bf16 [KH][Cout][32] kernel) →
          (stem_fused.hip, the default) ONE conv pass that takes the BN-1
          partial sums and max-pools y1 · sign(γ1) (argmax tap + y1 there:
          BN-1 + ReLU is monotone in y1 in the direction of γ1) → BN-1
          finalize → p = relu(BN-1(ya)) with BN-2 partial sums → BN-2
          finalize → BN-2 apply (+ the first binary block's sign images);
backward  BN-2 backward dx together with the BN-1 sums from the pooled side
          (the pooled value is BN-1's output at the argmax tap: no gather) →
          conv recomputed, dense dy1 routed in LDS, MFMA weight gradient
          straight into the flat gradient buffer.  y1 and dy1 never exist.

The image itself never needs a gradient; the op is only used when it does
not (``x.requires_grad`` is False).
"""

from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional, Tuple

import torch

from zookeeper_amd.nn.layers import same_padding
from zookeeper_amd.ops.options import OPTS
from zookeeper_amd.ops._native import (check, direct_grad, grad_ready, lib, slab_reduce,
                                        stream_ptr, zeroed, zeroed_scratch)

# The recompute-fused kernels of stem_fused.hip are the default
# (``runtime.stem_fused=False`` selects the materialising kernels of stem.hip):
# they never write the 112x112x64 conv output or its gradient.  Round-2
# measurements (tools/grad_determinism.py): the fp32-atomic ordering noise of
# the BN-backward sums (~1e-7) is amplified through the binary blocks, and the
# stem BN-1 scale gradient, a near-total cancellation (BN-2 re-normalises the
# pooled BN-1 output), changes by O(1) relative on some repeats with either
# stem -- a property of the reductions, not of these kernels (the stem alone
# is bit-reproducible, tools/one_stem.py --check).


def supported(x: torch.Tensor, conv, bn1, pool_k: int, pool_s: int) -> bool:
    Cout, Cin, KH, KW = conv.weight.shape
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and not x.requires_grad
            and conv.weight.device == x.device
            and Cin <= 4 and Cout == 64 and KH <= 8 and KW <= 8 and conv.stride == (2, 2)
            and conv.padding == "same" and conv.bias is None and conv.groups == 1
            and conv.input_quantizer is None and conv.kernel_quantizer is None
            and pool_k * pool_k <= 255)


def _fused_ok(KH, Cout, Cin, KW, s, pk, ps, Ho, Wo, pt2, pl2, H2, W2) -> bool:
    """Geometry the recompute-fused kernels (stem_fused.hip) cover: 7-row
    kernels, 64 output channels, stride 2, 3x3/2 'same' max pool."""
    return (OPTS.stem_fused and KH == 7 and Cout == 64 and Cin <= 4 and KW <= 8 and s == 2 and pk == 3
            and ps == 2 and pt2 in (0, 1) and pl2 in (0, 1) and H2 == (Ho + pt2 + 1) // 2
            and W2 == (Wo + pl2 + 1) // 2)


def _bn_eval_coef(bn, C, dev):
    rstd = torch.rsqrt(bn.running_var + bn.eps)
    g = bn.weight if bn.weight is not None else torch.ones_like(rstd)
    b = bn.bias if bn.bias is not None else torch.zeros_like(rstd)
    coef = torch.empty((4, C), dtype=torch.float32, device=dev)
    coef[0] = g * rstd
    coef[1] = b - bn.running_mean * coef[0]
    coef[2] = bn.running_mean
    coef[3] = rstd
    return coef


def _bn_bwd_coef(L, st, sums, coef, gamma_p, beta_p, P, C, dev, stripes: int = 1,
                 stride: int = 1):
    """BN backward coefficients [k1, k0, k3] from channel-major copies
    ``sums`` [2][C][stride] (the first ``stripes`` of each row are summed);
    γ/β gradients go into the flat buffer when the trainer manages it, else
    are returned."""
    dg = direct_grad(gamma_p) if gamma_p is not None else None
    db = direct_grad(beta_p) if beta_p is not None else None
    dgamma = dg if dg is not None else (torch.zeros(C, device=dev) if gamma_p is not None else None)
    dbeta = db if db is not None else (torch.zeros(C, device=dev) if beta_p is not None else None)
    bcoef = torch.empty((3, C), dtype=torch.float32, device=dev)
    check(L.zk_bn_bwd_coef(sums.data_ptr(), coef[2].data_ptr(), coef[3].data_ptr(),
                           gamma_p.data_ptr() if gamma_p is not None else None, float(P), C,
                           stripes, stride,
                           bcoef.data_ptr(), dgamma.data_ptr() if dgamma is not None else None,
                           dbeta.data_ptr() if dbeta is not None else None, st), "zk_bn_bwd_coef")
    if dg is not None:
        grad_ready(gamma_p)
        dgamma = None
    if db is not None:
        grad_ready(beta_p)
        dbeta = None
    return bcoef, dgamma, dbeta


# BN-2 backward sums taken from the first binary block's dgrad epilogue
# (backward passes; tests / diagnostics)
FUSED_BN2_SUMS = [0]

# Padded-input layouts of the stems that ran: (H, W, Cin) -> (Hp, Wp, pt, pl).
# The loader's preprocessing (data/preprocessing.py device_transform) writes
# that layout itself on its copy stream, next to the normalised image, and
# hands it over as ``x._zk_stem_xp = (xp, spec, x._version)``; the stem then
# skips its pack kernel (PREPACKED counts those forwards).
PACK_SPECS: Dict[Tuple[int, int, int], Tuple[int, int, int, int]] = {}
PREPACKED = [0]


def prepacked_input(x: torch.Tensor, spec) -> Optional[torch.Tensor]:
    """The loader-written padded input of ``x`` if it matches ``spec`` and x
    was not modified since."""
    h = getattr(x, "_zk_stem_xp", None)
    if h is None:
        return None
    xp, hspec, version = h
    if tuple(hspec) != tuple(spec) or version != x._version or xp.device != x.device:
        return None
    return xp


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, g1, b1, g2, b2, bn1, bn2, pool):
        pk, ps, sign_clip, holder, bnsum_holder, sign_consumer = pool
        B, Cin, H, W = x.shape
        Cout, _, KH, KW = weight.shape
        s = 2
        pt, pb = same_padding(H, KH, s)
        pl, pr = same_padding(W, KW, s)
        Ho, Wo = (H + pt + pb - KH) // s + 1, (W + pl + pr - KW) // s + 1
        Hp = (Ho - 1) * s + KH
        Wp = (Wo - 1) * s + 8
        Wp += Wp % 2
        dev = x.device
        st = stream_ptr(dev)
        L = lib()

        xn = x.permute(0, 2, 3, 1).contiguous()
        spec = (Hp, Wp, pt, pl)
        PACK_SPECS[(H, W, Cin)] = spec
        xp = prepacked_input(x, spec) if Cin == 3 else None
        if xp is not None:
            PREPACKED[0] += 1
        else:
            xp = torch.empty((B, Hp, Wp, 4), dtype=torch.bfloat16, device=dev)
            check(L.zk_stem_pack_input(xn.data_ptr(), xp.data_ptr(), B, H, W, Cin, Hp, Wp, pt,
                                       pl, st), "zk_stem_pack_input")
        w_ohwi = weight.detach().permute(0, 2, 3, 1).contiguous()
        ws = torch.empty((KH, Cout, 32), dtype=torch.bfloat16, device=dev)
        if os.environ.get("ZK_DEBUG_STEM"):
            for nm, t in (("x", x), ("xn", xn), ("xp", xp), ("weight", weight),
                          ("w_ohwi", w_ohwi), ("ws", ws)):
                st_ = t.untyped_storage()
                print(f"[stem] {nm}: shape {tuple(t.shape)} stride {t.stride()} {t.dtype} "
                      f"{t.device} ptr {t.data_ptr():#x} storage {st_.data_ptr():#x}+"
                      f"{st_.nbytes()} offset {t.storage_offset()}", flush=True)
            print(f"[stem] geom B={B} Cin={Cin} H={H} W={W} Cout={Cout} KH={KH} KW={KW} "
                  f"Ho={Ho} Wo={Wo} Hp={Hp} Wp={Wp} pt={pt} pl={pl} stream={st:#x}", flush=True)
            if os.environ.get("ZK_DEBUG_STEM") == "dry":
                raise RuntimeError("ZK_DEBUG_STEM=dry: stopping before the stem kernels")
        check(L.zk_stem_pack_weight(w_ohwi.data_ptr(), ws.data_ptr(), Cout, KH, KW, Cin, st),
              "zk_stem_pack_weight")
        pt2, pb2 = same_padding(Ho, pk, ps)
        pl2, pr2 = same_padding(Wo, pk, ps)
        H2, W2 = (Ho + pt2 + pb2 - pk) // ps + 1, (Wo + pl2 + pr2 - pk) // ps + 1
        fused = _fused_ok(KH, Cout, Cin, KW, s, pk, ps, Ho, Wo, pt2, pl2, H2, W2)
        P1 = B * Ho * Wo
        geo = (B, Cin, KW, Ho, Wo, Hp, Wp, H2, W2, pt2, pl2)

        def finalize1(part, nb):
            coef1 = torch.empty((4, Cout), dtype=torch.float32, device=dev)
            # one partial row per conv tile (~25-50k): coalesced two-pass reduction
            fws = torch.empty(L.zk_bn_finalize_ws_bytes(Cout) // 8, dtype=torch.float64,
                              device=dev)
            check(L.zk_bn_finalize_partials_ws(part.data_ptr(), nb, Cout, float(P1),
                                               g1.data_ptr() if g1 is not None else None,
                                               b1.data_ptr() if b1 is not None else None,
                                               bn1.eps, bn1.momentum,
                                               bn1.running_mean.data_ptr(),
                                               bn1.running_var.data_ptr(), coef1.data_ptr(),
                                               fws.data_ptr(), st),
                  "zk_bn_finalize_partials_ws")
            return coef1

        p = torch.empty((B, H2, W2, Cout), dtype=torch.bfloat16, device=dev)
        arg = torch.empty((B, H2, W2, Cout), dtype=torch.uint8, device=dev)
        want_part2 = bn2 is not None and bn2.training
        nb2 = ctypes.c_int(0)
        y1 = ya = None
        if fused:
            # one conv pass: BN-1 statistics and the pool of y1 * sign(gamma1)
            # (the direction of relu(BN-1(y)) in y); p once BN-1 is finalised
            # (stem_fused.hip F / P).  y1 never exists.
            ya = torch.empty_like(p)
            part = (torch.empty((L.zk_stem_fused_blocks(1, B, Ho, Wo, H2, W2), 2, Cout),
                                dtype=torch.float32, device=dev) if bn1.training else None)
            nb = ctypes.c_int(0)
            check(L.zk_stem_fwd_fused(xp.data_ptr(), ws.data_ptr(),
                                      g1.data_ptr() if g1 is not None else None, ya.data_ptr(),
                                      arg.data_ptr(), part.data_ptr() if part is not None else None,
                                      *geo, ctypes.byref(nb), st), "zk_stem_fwd_fused")
            coef1 = finalize1(part, nb.value) if bn1.training else _bn_eval_coef(bn1, Cout, dev)
            part2 = torch.empty((L.zk_stem_max_pool_parts(), 2, Cout), dtype=torch.float32,
                                device=dev) if want_part2 else None
            check(L.zk_stem_pool_relu(ya.data_ptr(), coef1.data_ptr(), p.data_ptr(),
                                      part2.data_ptr() if part2 is not None else None,
                                      B * H2 * W2, ctypes.byref(nb2), st), "zk_stem_pool_relu")
        else:
            y1 = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=dev)
            part = torch.empty((L.zk_stem_max_parts(B, Ho, Wo), 2, Cout), dtype=torch.float32,
                               device=dev)
            nb = ctypes.c_int(0)  # number of partial-sum rows, written by the launcher
            check(L.zk_stem_conv_fwd(xp.data_ptr(), ws.data_ptr(), y1.data_ptr(),
                                     part.data_ptr(), B, Cin, Cout, KH, KW, s, Ho, Wo, Hp, Wp, -1,
                                     ctypes.byref(nb), st), "zk_stem_conv_fwd")
            coef1 = finalize1(part, nb.value) if bn1.training else _bn_eval_coef(bn1, Cout, dev)
            part2 = torch.empty((L.zk_stem_max_pool_parts(), 2, Cout), dtype=torch.float32,
                                device=dev) if want_part2 else None
            check(L.zk_stem_pool_fwd(y1.data_ptr(), coef1.data_ptr(), p.data_ptr(),
                                     arg.data_ptr(),
                                     part2.data_ptr() if part2 is not None else None, B, Ho, Wo,
                                     Cout, H2, W2, pk, ps, pt2, pl2, ctypes.byref(nb2), st),
                  "zk_stem_pool_fwd")
        P2 = B * H2 * W2
        coef2 = None
        out = p
        if bn2 is not None:
            if bn2.training:
                coef2 = torch.empty((4, Cout), dtype=torch.float32, device=dev)
                fws2 = torch.empty(L.zk_bn_finalize_ws_bytes(Cout) // 8, dtype=torch.float64,
                                   device=dev)
                check(L.zk_bn_finalize_partials_ws(part2.data_ptr(), nb2.value, Cout, float(P2),
                                                   g2.data_ptr() if g2 is not None else None,
                                                   b2.data_ptr() if b2 is not None else None,
                                                   bn2.eps, bn2.momentum,
                                                   bn2.running_mean.data_ptr(),
                                                   bn2.running_var.data_ptr(), coef2.data_ptr(),
                                                   fws2.data_ptr(), st),
                      "zk_bn_finalize_partials_ws")
            else:
                coef2 = _bn_eval_coef(bn2, Cout, dev)
            out = torch.empty_like(p)
            if holder is not None and Cout % 32 == 0:
                # also quantise the output for the first binary block
                from zookeeper_amd.ops.binary import _fp4, bf16_sign_needed

                sx = (torch.empty_like(p)
                      if bf16_sign_needed(sign_consumer, (B, H2, W2, Cout)) else None)
                mask = torch.empty(P2 * Cout // 32, dtype=torch.int32, device=dev)
                sx4 = (torch.empty((B, H2, W2, Cout // 2), dtype=torch.uint8, device=dev)
                       if _fp4() else None)
                check(L.zk_bn_apply_bf16_sign(p.data_ptr(), coef2.data_ptr(), out.data_ptr(),
                                              sx.data_ptr() if sx is not None else None,
                                              mask.data_ptr(),
                                              sx4.data_ptr() if sx4 is not None else None,
                                              sign_clip, P2, Cout, 0, st),
                      "zk_bn_apply_bf16_sign")
                holder[:] = [sign_clip, sx, mask, sx4]
            else:
                check(L.zk_bn_apply_bf16(p.data_ptr(), coef2.data_ptr(), out.data_ptr(), P2,
                                         Cout, 0, st), "zk_bn_apply_bf16")
        # BN-2's backward sums reduced by the first binary block's row-window
        # dgrad epilogue (its dx is exactly this output's gradient: identity
        # shortcut, single consumer), as between binary blocks
        ctx.bnsum = None
        if (bnsum_holder is not None and bn2 is not None and bn2.training
                and OPTS.dgrad_rw and not OPTS.deterministic
                and Cout == 64 and W2 <= 64):
            from zookeeper_amd.ops.binary import _BnSum, bwd_stripes

            sums_buf = zeroed_scratch(bn2, "bwd_sums", (2, Cout, bwd_stripes()), torch.float32,
                                      dev)
            ctx.bnsum = _BnSum(p, coef2[2], coef2[3], sums_buf, bf16=True)
            bnsum_holder.append(ctx.bnsum)
        ctx.save_for_backward(xp, ws, y1 if y1 is not None else ya, arg, p, coef1, coef2, g1,
                              g2)
        ctx.fused = fused
        ctx.params = (weight, g1, b1, g2, b2)
        ctx.geom = (B, Cin, Cout, KH, KW, s, Ho, Wo, Hp, Wp, H2, W2, pk, ps, pt2, pl2)
        ctx.has_bn2 = bn2 is not None
        ctx.bn2 = bn2
        return out.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, dout):
        xp, ws, y1, arg, p, coef1, coef2, g1, g2 = ctx.saved_tensors  # fused: y1 = ya
        weight, g1p, b1p, g2p, b2p = ctx.params
        (B, Cin, Cout, KH, KW, s, Ho, Wo, Hp, Wp, H2, W2, pk, ps, pt2, pl2) = ctx.geom
        dev = dout.device
        st = stream_ptr(dev)
        L = lib()
        P2 = B * H2 * W2
        g = dout.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
        dg2 = db2 = None
        if ctx.has_bn2:
            bs = ctx.bnsum
            touched = bs is not None and bs.dx is not None  # the successor wrote the sums
            if touched and bs.reduced(dout):
                # the first binary block's row-window dgrad epilogue reduced
                # exactly this gradient (one copy per block, fixed order)
                n = bs.sums.shape[2]
                FUSED_BN2_SUMS[0] += 1
                bcoef2, dg2, db2 = _bn_bwd_coef(L, st, bs.sums, coef2, g2p, b2p, P2, Cout, dev,
                                                stripes=n, stride=n)
            else:
                if touched:
                    bs.dx = None
                    bs.sums.zero_()  # a gradient that was accumulated after the reduction
                # per-block partials summed in a fixed order: the stem's BN-1 /
                # conv gradients amplify run-to-run noise of these sums (BN-2
                # makes dL/dgamma1 a near-total cancellation)
                sums2 = torch.empty((2, Cout, L.zk_bn_bwd_parts_max()), dtype=torch.float32,
                                    device=dev)  # channel-major copies
                nb2 = ctypes.c_int(0)
                check(L.zk_bn_bwd_reduce_bf16_parts(g.data_ptr(), p.data_ptr(), None,
                                                    coef2.data_ptr(), sums2.data_ptr(), P2, Cout,
                                                    ctypes.byref(nb2), st),
                      "zk_bn_bwd_reduce_bf16_parts")
                bcoef2, dg2, db2 = _bn_bwd_coef(L, st, sums2, coef2, g2p, b2p, P2, Cout, dev,
                                                stripes=nb2.value, stride=sums2.shape[2])
        part = torch.empty((L.zk_stem_max_pool_parts(), 2, Cout), dtype=torch.float32,
                           device=dev)
        nb = ctypes.c_int(0)
        b1_done = False
        if ctx.has_bn2:
            dp = torch.empty_like(g)
            if ctx.fused:
                # BN-2 dx and the BN-1 sums (B1) in one pass over g, p, ya
                check(L.zk_stem_bn2_bwd_sums(g.data_ptr(), p.data_ptr(), y1.data_ptr(),
                                             bcoef2.data_ptr(), coef1.data_ptr(), dp.data_ptr(),
                                             part.data_ptr(), P2, ctypes.byref(nb), st),
                      "zk_stem_bn2_bwd_sums")
                b1_done = True
            else:
                check(L.zk_bn_bwd_dx_bf16(g.data_ptr(), p.data_ptr(), None, bcoef2.data_ptr(),
                                          dp.data_ptr(), P2, Cout, st), "zk_bn_bwd_dx_bf16")
        else:
            dp = g
        if b1_done:
            pass  # the BN-1 sums came with dp
        elif ctx.fused:
            check(L.zk_stem_pool_bwd_sums_ya(dp.data_ptr(), y1.data_ptr(), coef1.data_ptr(),
                                             part.data_ptr(), P2, ctypes.byref(nb), st),
                  "zk_stem_pool_bwd_sums_ya")
        else:
            check(L.zk_stem_pool_bwd_sums(dp.data_ptr(), arg.data_ptr(), y1.data_ptr(),
                                          p.data_ptr(), coef1.data_ptr(), part.data_ptr(), B, Ho,
                                          Wo, Cout, H2, W2, pk, ps, pt2, pl2, ctypes.byref(nb),
                                          st), "zk_stem_pool_bwd_sums")
        sums1 = torch.empty((2, Cout), dtype=torch.float32, device=dev)
        check(L.zk_reduce_partials(part.data_ptr(), nb.value, 2 * Cout, sums1.data_ptr(), st),
              "zk_reduce_partials")
        if os.environ.get("ZK_DEBUG_STEM"):
            torch.cuda.synchronize()

            def cs(t):
                return f"{t.double().sum().item():.9e}/{t.double().abs().sum().item():.9e}"
            print(f"[stem bwd] g {cs(g)} dp {cs(dp)} y1 {cs(y1)} arg {cs(arg)} p {cs(p)} "
                  f"coef1 {cs(coef1)} nb {nb.value} part {cs(part[:nb.value])} "
                  f"sums1 {sums1.tolist()[0][:3]}", flush=True)
        P1 = B * Ho * Wo
        bcoef1, dg1, db1 = _bn_bwd_coef(L, st, sums1, coef1, g1p, b1p, P1, Cout, dev)
        dweight = None
        if ctx.needs_input_grad[1]:
            target = direct_grad(weight, channels_last=True)
            if target is not None:
                dw = target.permute(0, 2, 3, 1)  # OHWI view of the flat gradient
            else:
                dw = torch.zeros((Cout, KH, KW, Cin), dtype=torch.float32, device=dev)
            if ctx.fused:
                nblk = L.zk_stem_fused_blocks(0, B, Ho, Wo, H2, W2)
                slab = torch.empty((nblk + L.zk_stem_fused_slab_extra(),
                                    L.zk_stem_fused_slab_floats()), dtype=torch.float32,
                                   device=dev)
                check(L.zk_stem_bwd_fused(xp.data_ptr(), ws.data_ptr(), dp.data_ptr(),
                                          arg.data_ptr(), coef1.data_ptr(), bcoef1.data_ptr(),
                                          slab.data_ptr(), dw.data_ptr(), B, Cin, KW, Ho, Wo, Hp,
                                          Wp, H2, W2, pt2, pl2, st), "zk_stem_bwd_fused")
            else:
                dy1 = torch.empty_like(y1)
                check(L.zk_stem_dy1(dp.data_ptr(), arg.data_ptr(), y1.data_ptr(),
                                    coef1.data_ptr(), bcoef1.data_ptr(), dy1.data_ptr(), B, Ho,
                                    Wo, Cout, H2, W2, pk, ps, pt2, pl2, st), "zk_stem_dy1")
                # slab policy (default / deterministic): per-split partials +
                # fixed-order reduce
                slab = (zeroed((L.zk_stem_wgrad_splits(B, Ho, Wo, 0), Cout * KH * KW * Cin), dev)
                        if slab_reduce() else None)
                check(L.zk_stem_wgrad(dy1.data_ptr(), xp.data_ptr(), dw.data_ptr(),
                                      slab.data_ptr() if slab is not None else None, B, Cin,
                                      Cout, KH, KW, s, Ho, Wo, Hp, Wp, 0, st), "zk_stem_wgrad")
                if slab is not None:
                    check(L.zk_wgrad_slab_reduce(slab.data_ptr(), slab.shape[0], slab.shape[1],
                                                 None, 0.0, dw.data_ptr(), st),
                          "zk_wgrad_slab_reduce")
            if target is not None:
                grad_ready(weight)
            else:
                dweight = dw.permute(0, 3, 1, 2)
        return None, dweight, dg1, db1, dg2, db2, None, None, None


def fused_stem(x: torch.Tensor, conv, bn1, pool_k: int = 3, pool_s: int = 2, bn2=None,
               sign_clip: Optional[float] = None, sign_consumer=None):
    """``bn2(maxpool(relu(bn1(conv(x)))))`` with the fused stem kernels.

    With ``sign_clip`` (and ``bn2``) the final BN pass also writes the sign
    image and STE mask (|y| <= sign_clip) of the output, attached as
    ``_zk_sign`` for the first binary block (see ``ops.binary_block``;
    ``sign_consumer``: that block's conv, which decides whether the bf16 sign
    image is needed: ``ops.binary.bf16_sign_needed``)."""
    holder = [] if (sign_clip is not None and bn2 is not None) else None
    # consumer: a binary block; only when a backward will run (grad mode is
    # off inside the autograd function's forward)
    bnsum = [] if holder is not None and torch.is_grad_enabled() else None
    out = _StemFn.apply(x, conv.weight, bn1.weight, bn1.bias,
                        bn2.weight if bn2 is not None else None,
                        bn2.bias if bn2 is not None else None, bn1, bn2,
                        (pool_k, pool_s, float(sign_clip or 0.0), holder, bnsum, sign_consumer))
    if holder:
        out._zk_sign = tuple(holder)
    if bnsum:
        out._zk_bnsum = bnsum[0]
    return out
