"""Classifier head on native kernels (``csrc/kernels/head.hip``).

``classifier_head(x, weight, bias, relu)`` = ``F.linear(mean_hw(relu(x)).float(),
weight, bias)`` for a channels-last bf16 feature map: the global average pool
runs in fp32 on a per-image kernel and the dense layer is an fp32 MFMA GEMM
(``v_mfma_f32_16x16x4_f32``), forward and backward.  It replaces the
``x.mean`` reduction and the hipBLASLt GEMMs that ended the BinaryResNet-E /
QuickNet / ResNet-50 steps (the reference's models finish with Keras
``GlobalAveragePooling2D`` + an fp32 ``Dense``: larq_zoo's
``binary_resnet_e.py``/``quicknet.py`` heads; /root/reference/examples/
larq_experiment.py:95-101 for the float classifier convention).

``global_avg_pool(x)`` is the pool alone (bf16 in, bf16 out), used by
:class:`~zookeeper_amd.nn.layers.GlobalAvgPool`.

The weight gradient accumulates straight into the flat fp32 gradient buffer
when the parameter has one (:func:`~zookeeper_amd.ops._native.direct_grad`).
"""

from __future__ import annotations

import torch

from zookeeper_amd.ops._native import check, direct_grad, grad_ready, lib, stream_ptr


def head_supported(x: torch.Tensor, weight: torch.Tensor) -> bool:
    """Shapes/layouts the head kernels take (else the caller uses PyTorch)."""
    return (x.dim() == 4 and x.is_cuda and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0
            and weight.dtype == torch.float32 and weight.is_contiguous()
            and weight.shape[1] == x.shape[1] and x.numel() > 0)


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        B, C, H, W = x.shape
        N = weight.shape[0]
        dev = x.device
        pooled = torch.empty((B, C), dtype=torch.float32, device=dev)
        logits = torch.empty((B, N), dtype=torch.float32, device=dev)
        b = bias.float().contiguous() if bias is not None else None
        check(lib().zk_head_fwd(x.data_ptr(), weight.data_ptr(),
                                b.data_ptr() if b is not None else None, pooled.data_ptr(),
                                logits.data_ptr(), B, H * W, C, N, int(relu), stream_ptr(dev)),
              "zk_head_fwd")
        ctx.save_for_backward(x, weight, pooled)
        ctx.bias_param, ctx.relu = bias, bool(relu)
        ctx.weight_param = weight
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        x, weight, pooled = ctx.saved_tensors
        B, C, H, W = x.shape
        N = weight.shape[0]
        dev = x.device
        dl = dlogits.float().contiguous()
        need_x, need_w, need_b = ctx.needs_input_grad[:3]
        wp, bp = ctx.weight_param, ctx.bias_param
        dw_direct = direct_grad(wp) if need_w else None
        db_direct = direct_grad(bp) if need_b else None
        dw = dw_direct if dw_direct is not None else (
            torch.zeros((N, C), dtype=torch.float32, device=dev) if need_w else None)
        db = db_direct if db_direct is not None else (
            torch.zeros(N, dtype=torch.float32, device=dev) if need_b else None)
        dx = torch.empty_like(x) if need_x else None  # keeps channels_last
        dpooled = torch.empty((B, C), dtype=torch.float32, device=dev) if need_x else None
        # the kernel folds the bias gradient into the dW GEMM; a frozen weight
        # with a trainable bias (rare) takes the bias sum from PyTorch
        db_native = db if dw is not None else None
        if db is not None and dw is None:
            db += dl.sum(0)
        check(lib().zk_head_bwd(dl.data_ptr(), x.data_ptr(), weight.data_ptr(), pooled.data_ptr(),
                                dw.data_ptr() if dw is not None else None,
                                db_native.data_ptr() if db_native is not None else None,
                                dpooled.data_ptr() if dpooled is not None else None,
                                dx.data_ptr() if dx is not None else None,
                                B, H * W, C, N, int(ctx.relu), stream_ptr(dev)),
              "zk_head_bwd")
        if dw_direct is not None:
            grad_ready(wp)
            dw = None
        if db_direct is not None:
            grad_ready(bp)
            db = None
        if db is not None and bp is not None and bp.dtype != torch.float32:
            db = db.to(bp.dtype)
        return dx, dw, db, None


def classifier_head(x: torch.Tensor, weight: torch.Tensor, bias, relu: bool) -> torch.Tensor:
    """fp32 logits = dense(mean_hw(relu?(x))); see the module docstring."""
    return _HeadFn.apply(x, weight, bias, relu)


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        B, C, H, W = x.shape
        out = torch.empty((B, C), dtype=torch.bfloat16, device=x.device)
        check(lib().zk_gap_fwd(x.data_ptr(), out.data_ptr(), B, H * W, C, 0, 1,
                               stream_ptr(x.device)), "zk_gap_fwd")
        ctx.shape = (B, C, H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        B, C, H, W = ctx.shape
        gf = g.float().contiguous()
        dx = torch.empty((B, C, H, W), dtype=torch.bfloat16, device=g.device,
                         memory_format=torch.channels_last)
        # relu=0: the x operand is not read
        check(lib().zk_gap_bwd(gf.data_ptr(), None, dx.data_ptr(), B, H * W, C, 0,
                               stream_ptr(g.device)), "zk_gap_bwd")
        return dx


def gap_supported(x: torch.Tensor) -> bool:
    return (x.dim() == 4 and x.is_cuda and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0
            and x.numel() > 0)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """bf16 [B, C] = mean over H, W of a channels-last bf16 map."""
    return _GapFn.apply(x)
