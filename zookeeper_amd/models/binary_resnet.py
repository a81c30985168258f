"""Binary ResNet "E" family (BinaryResNetE18 and deeper variants).

Architecture as published in Larq-Zoo (Bethge et al., "Back to Simplicity:
How to Train Accurate BNNs from Scratch?", 2019) — not part of the reference
repo, which only ships BinaryNet; see SURVEY §2.4:

* float stem for ImageNet-size inputs: 7×7/2 conv (he_normal) → BN → ReLU →
  3×3/2 max-pool (``same``) → BN; for inputs < 50 px a 3×3 conv instead;
* ``2·layers`` residual blocks per stage, each ONE binary 3×3 conv
  (``ste_sign`` inputs and kernels, ``weight_clip``, ``same`` padding with
  zeros) → BN, plus its own shortcut; a stage transition strides the conv by
  2 and the shortcut is AvgPool 2×2/2 → float 1×1 conv → BN;
* ReLU → global average pool → float Dense(num_classes) (→ softmax in loss).

``num_layers`` 18 → stages of (2, 2, 2, 2) original blocks ×2 = 16 binary
convs at 64/128/256/512 channels.

Execution: the ``hip`` backend runs each binary block as ONE fused autograd
op (:func:`zookeeper_amd.ops.binary_block`): the previous BN epilogue writes
the input signs as MX-FP4 (e2m1 ±1) nibbles plus the STE mask bits, the
forward conv is an MX-FP4 MFMA implicit GEMM (``v_mfma_scale_f32_32x32x64_f8f6f4``,
exact integer outputs; measured faster than the XNOR-popcount kernel, which
remains as ``zk_bconv_fwd``) with the BN statistics fused into its epilogue,
then BN-apply + residual add, and a matching fused backward (bf16 MFMA
dgrad / wgrad, BN backward).  The ``torch`` backend is the pure-PyTorch
oracle used by the tests.
"""

from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from zookeeper_amd.core import Field, factory
from zookeeper_amd.models.base import ModelFactory
from zookeeper_amd.nn.layers import (
    _use_native,
    AvgPool2d,
    BatchNorm,
    ImageStem,
    GlobalAvgPool,
    pooled_dense,
    MaxPool2d,
    QuantConv2d,
    glorot_normal_,
)

_SPECS = {
    18: ((2, 2, 2, 2), (64, 128, 256, 512)),
    34: ((3, 4, 6, 3), (64, 128, 256, 512)),
    50: ((3, 4, 6, 3), (256, 512, 1024, 2048)),
    101: ((3, 4, 23, 3), (256, 512, 1024, 2048)),
    152: ((3, 8, 36, 3), (256, 512, 1024, 2048)),
}


class BinaryResBlock(nn.Module):
    """``out = BN(bconv(sign(x))) + shortcut(x)``."""

    def __init__(self, cin: int, cout: int, stride: int, momentum: float = 0.9,
                 eps: float = 1e-5, backend: str = "torch", pad_value: float = 0.0):
        super().__init__()
        self.cin, self.cout, self.stride, self.backend = cin, cout, stride, backend
        self.conv = QuantConv2d(cin, cout, 3, stride, "same", "ste_sign", "ste_sign",
                                "weight_clip", pad_values=pad_value)
        self.bn = BatchNorm(cout, momentum=momentum, eps=eps)
        # the next block's conv: reads this block's output sign images (set
        # by the model; decides whether the bf16 one is needed)
        self.sign_consumer = None
        # the next block pools this block's output (its downsampling
        # shortcut): the BN epilogue writes the pooled image too (set by the model)
        self.pool_out = False
        self.downsample = None
        if cin != cout:
            self.downsample = nn.Sequential(
                AvgPool2d(2, 2),
                QuantConv2d(cin, cout, 1, 1, "valid"),
                BatchNorm(cout, momentum=momentum, eps=eps),
            )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip" and x.is_cuda:
            from zookeeper_amd import ops
            from zookeeper_amd.ops import norm_pool

            handoff = None
            if self.downsample is not None:
                pool, conv, bn = self.downsample
                if (_use_native(x) and x.shape[1] % 8 == 0 and pool.pool_size == (2, 2)
                        and pool.stride == (2, 2)):
                    # x's two gradients (shortcut avg-pool + binary conv) are
                    # summed in the avg-pool backward instead of an add pass
                    handoff = norm_pool.ResidualHandoff()
                    # (BN statistics from the 1x1 GEMM's epilogue: stats_for)
                    residual = bn(conv(norm_pool.avg_pool2(x, handoff=handoff), stats_for=bn))
                else:
                    residual = self.downsample(x)
            else:
                residual = x
            return ops.binary_block(x, residual, self.conv, self.bn, dx_handoff=handoff,
                                    sign_consumer=self.sign_consumer, pool_out=self.pool_out)
        residual = self.downsample(x) if self.downsample is not None else x
        return self.bn(self.conv(x)) + residual


class BinaryResNetE(nn.Module):
    def __init__(self, input_shape, num_classes: int, num_layers: int = 18,
                 initial_filters: int = 64, backend: str = "torch"):
        super().__init__()
        h, w, c = input_shape
        blocks, filters = _SPECS[num_layers]
        if initial_filters != 64 and num_layers < 50:
            filters = tuple(initial_filters * 2**i for i in range(4))
        stem = []
        if h < 50:
            stem.append(QuantConv2d(c, initial_filters, 3, 1, "same", kernel_initializer="he_normal"))
        else:
            stem += [
                QuantConv2d(c, initial_filters, 7, 2, "same", kernel_initializer="he_normal"),
                BatchNorm(initial_filters, momentum=0.9, eps=1e-5, activation="relu"),
                MaxPool2d(3, 2, "same"),
                BatchNorm(initial_filters, momentum=0.9, eps=1e-5),
            ]
        self.stem = ImageStem(*stem)
        # the first binary block's ste_sign clip: the fused stem pre-quantises for it
        self.stem.sign_clip = 1.0
        body = []
        cin = initial_filters
        for stage, (n, f) in enumerate(zip(blocks, filters)):
            # Each original 2-conv block becomes two single-conv blocks with
            # their own shortcuts ("E" = extra shortcuts).
            for i in range(2 * n):
                stride = 1 if stage == 0 or i != 0 else 2
                body.append(BinaryResBlock(cin, f, stride, backend=backend))
                cin = f
        # (plain attributes, not submodules: no duplicate parameters / state keys)
        for blk, nxt in zip(body, body[1:]):
            object.__setattr__(blk, "sign_consumer", nxt.conv)
            ds = nxt.downsample
            blk.pool_out = (ds is not None and isinstance(ds[0], AvgPool2d)
                            and ds[0].pool_size == (2, 2) and ds[0].stride == (2, 2))
        object.__setattr__(self.stem, "sign_consumer", body[0].conv)
        self.body = nn.Sequential(*body)
        self.pool = GlobalAvgPool()
        self.fc = nn.Linear(cin, num_classes)
        glorot_normal_(self.fc.weight)
        nn.init.zeros_(self.fc.bias)
        self.input_shape, self.num_classes = tuple(input_shape), num_classes

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.stem(x)
        x = self.body(x)
        return pooled_dense(x, self.pool, self.fc, relu=True)

    def set_backend(self, backend: str) -> "BinaryResNetE":
        for m in self.modules():
            if isinstance(m, BinaryResBlock):
                m.backend = backend
        return self


@factory
class BinaryResNetE18(ModelFactory):
    """``@factory`` for BinaryResNet-E (default depth 18)."""

    num_layers: int = Field(18)
    initial_filters: int = Field(64)

    def build(self) -> nn.Module:
        return BinaryResNetE(self.input_shape, self.num_classes, self.num_layers,
                             self.initial_filters, backend=self.resolved_backend())


def stage_shapes(input_shape: Sequence[int], num_layers: int = 18):
    """(H, W, C_in, C_out, stride) of every binary conv — used by benchmarks."""
    h = input_shape[0]
    blocks, filters = _SPECS[num_layers]
    size = (h + 1) // 2
    size = (size + 1) // 2 if h >= 50 else h
    out, cin = [], 64
    for stage, (n, f) in enumerate(zip(blocks, filters)):
        for i in range(2 * n):
            stride = 1 if stage == 0 or i != 0 else 2
            out.append((size, size, cin, f, stride))
            size = (size + stride - 1) // stride
            cin = f
    return out
