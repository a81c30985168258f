"""Fused softmax cross-entropy + top-1 correctness (``csrc/kernels/xent.hip``)."""

from __future__ import annotations

import torch

from zookeeper_amd.ops._native import check, lib, stream_ptr
from zookeeper_amd.ops.options import OPTS


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, eps):
        x = logits.float().contiguous()
        B, C = x.shape
        y = labels.to(torch.int64).contiguous()
        dev = x.device
        lse = torch.empty(B, dtype=torch.float32, device=dev)
        acc = torch.zeros(2, dtype=torch.float32, device=dev)  # [loss_sum, correct (int bits)]
        correct = acc[1:].view(torch.int32)
        # deterministic mode: per-row losses summed in a fixed order
        row_loss = torch.empty(B, dtype=torch.float32, device=dev) if OPTS.deterministic else None
        check(lib().zk_xent_fwd(x.data_ptr(), y.data_ptr(), lse.data_ptr(), acc.data_ptr(),
                                correct.data_ptr(), B, C, float(eps),
                                row_loss.data_ptr() if row_loss is not None else None,
                                stream_ptr(dev)),
              "zk_xent_fwd")
        ctx.save_for_backward(x, y, lse)
        ctx.eps, ctx.in_dtype = float(eps), logits.dtype
        loss = acc[0] / B
        hits = correct.reshape(()).to(torch.int64)
        ctx.mark_non_differentiable(hits)
        return loss, hits

    @staticmethod
    def backward(ctx, gloss, _ghits):
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
