"""Fused softmax cross-entropy + top-1 correctness (``csrc/kernels/xent.hip``)."""

from __future__ import annotations

import torch

from zookeeper_amd.ops._native import check, lib, stream_ptr


# Accumulator [loss_sum, correct (int32 bits)] per (device, stream), zero
# between calls: zk_xent_finalize reads and re-zeroes it right after the
# zk_xent_fwd that fills it, on the same stream, so work on two streams (a
# training step and an eval pass) never shares one.  If the launch pair fails
# half-way the accumulator is re-zeroed (zk_zero) before the error propagates.
_ACC = {}


def _acc(dev: torch.device, stream: int) -> torch.Tensor:
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), stream)
    a = _ACC.get(key)
    if a is None:
        a = _ACC[key] = torch.zeros(2, dtype=torch.float32, device=dev)
    return a


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, eps):
        x = logits.float().contiguous()
        B, C = x.shape
        y = labels.to(torch.int64).contiguous()
        dev = x.device
        lse = torch.empty(B, dtype=torch.float32, device=dev)
        st = stream_ptr(dev)
        acc = _acc(dev, st)
        correct = acc[1:].view(torch.int32)
        # per-row losses summed in a fixed order (every mode: a reproducible
        # loss value for one extra single-block launch; the hit count stays an
        # exact integer atomic)
        row_loss = torch.empty(B, dtype=torch.float32, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        hits = torch.empty((), dtype=torch.int64, device=dev)
        try:
            check(lib().zk_xent_fwd(x.data_ptr(), y.data_ptr(), lse.data_ptr(), acc.data_ptr(),
                                    correct.data_ptr(), B, C, float(eps),
                                    row_loss.data_ptr() if row_loss is not None else None, st),
                  "zk_xent_fwd")
            check(lib().zk_xent_finalize(acc.data_ptr(), loss.data_ptr(), hits.data_ptr(), B, st),
                  "zk_xent_finalize")
        except RuntimeError:
            lib().zk_zero(acc.data_ptr(), acc.numel() * 4, st)  # no partial sums leak
            raise
        ctx.save_for_backward(x, y, lse)
        ctx.eps, ctx.in_dtype = float(eps), logits.dtype
        ctx.mark_non_differentiable(hits)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the hit count
        return loss, hits

    @staticmethod
    def backward(ctx, gloss, _ghits):
        if gloss is None:
            return None, None, None
        x, y, lse = ctx.saved_tensors
        B, C = x.shape
        g = gloss.float().reshape(1).contiguous()
        dx = torch.empty_like(x)
        check(lib().zk_xent_bwd(x.data_ptr(), y.data_ptr(), lse.data_ptr(), g.data_ptr(),
                                dx.data_ptr(), B, C, ctx.eps, stream_ptr(x.device)),
              "zk_xent_bwd")
        return dx.to(ctx.in_dtype), None, None


def softmax_xent(logits: torch.Tensor, labels: torch.Tensor, label_smoothing: float = 0.0):
    """(mean sparse categorical cross-entropy, number of top-1 hits)."""
    return _SoftmaxXentFn.apply(logits, labels, label_smoothing)
