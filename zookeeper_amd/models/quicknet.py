"""QuickNet / QuickNetLarge / QuickNetXL (Larq-Zoo "sota" binary networks).

Not part of the reference repo (SURVEY §2.4 lists them as north-star
workloads); definitions pinned from the published Larq-Zoo QuickNet family
(Bannink et al., "Larq Compute Engine", 2021):

* stem: 3×3/2 float conv (C/4) → BN → ReLU → 3×3/2 depthwise conv → BN →
  1×1 conv (C) → BN;
* residual block (no stride / width change): binary 3×3 conv with
  ``SteSign(clip=1.25)`` inputs and kernels, ``WeightClip(1.25)``, ``same``
  padding with **+1** pad values → ReLU → BN → + input;
* transition (when the width changes): ReLU → MaxPool 2×2/1 (valid) →
  fixed (non-trainable) blur-pool 3×3/2 depthwise → 1×1 float conv → BN;
* head: ReLU → global average pool → float dense → softmax (in the loss).

Section blocks: QuickNet (4,4,4,4), QuickNetLarge (6,8,12,6),
QuickNetXL (8,12,24,6); filters (64,128,256,512).
"""

from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from zookeeper_amd.core import Field, factory
from zookeeper_amd.models.base import ModelFactory
from zookeeper_amd.nn.layers import (BatchNorm, GlobalAvgPool, QuantConv2d, _use_native,
                                     glorot_normal_, pad_same_nhwc, pooled_dense)
from zookeeper_amd.nn.quantizers import ste_sign


class _Clip125Conv(QuantConv2d):
    """Binary conv with SteSign(clip_value=1.25) and WeightClip(1.25)."""

    def __init__(self, channels: int):
        super().__init__(channels, channels, 3, 1, "same", "ste_sign", "ste_sign", None,
                         pad_values=1.0)
        self.input_quantizer = lambda t: ste_sign(t, 1.25)
        self.kernel_quantizer = lambda t: ste_sign(t, 1.25)
        self.clip_value = 1.25

    def apply_constraints(self) -> None:
        with torch.no_grad():
            self.weight.clamp_(-self.clip_value, self.clip_value)


class QuickNetBlock(nn.Module):
    def __init__(self, channels: int, backend: str = "torch"):
        super().__init__()
        self.conv = _Clip125Conv(channels)
        self.bn = BatchNorm(channels, momentum=0.9, eps=1e-5)
        self.backend = backend
        # the next block's conv when it reads this output's sign images
        # (set by the model; ops.binary.bf16_sign_needed)
        self.sign_consumer = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.backend == "hip" and x.is_cuda:
            from zookeeper_amd import ops

            return ops.binary_block(x, x, self.conv, self.bn, act="relu",
                                    clip_value=1.25, pad_value=1.0,
                                    sign_consumer=self.sign_consumer)
        return self.bn(F.relu(self.conv(x))) + x


class BlurPool(nn.Module):
    """Fixed 3×3 stride-2 depthwise binomial blur (non-trainable)."""

    def __init__(self, channels: int):
        super().__init__()
        k = torch.tensor([1.0, 2.0, 1.0])
        k = (k[:, None] * k[None, :]) / 16.0
        self.register_buffer("kernel", k.expand(channels, 1, 3, 3).contiguous())
        self.channels = channels

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _use_native(x):
            from zookeeper_amd.ops import depthwise

            if depthwise.supported(x, self.kernel):
                return depthwise.depthwise_conv3x3(x, self.kernel, 2, "same")
        x = pad_same_nhwc(x, (3, 3), (2, 2))
        return F.conv2d(x, self.kernel.to(x.dtype), None, 2, 0, 1, self.channels)


class Transition(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.blur = BlurPool(cin)
        self.conv = QuantConv2d(cin, cout, 1, 1, "valid")
        self.bn = BatchNorm(cout, momentum=0.9, eps=1e-5)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _use_native(x) and x.shape[1] % 8 == 0:
            from zookeeper_amd.ops.norm_pool import max_pool

            x = max_pool(x, 2, 1, "valid", relu=True)  # relu∘max == max∘relu, one pass
        else:
            x = F.max_pool2d(F.relu(x), 2, 1)
        # (BN statistics from the 1x1 GEMM's epilogue where it runs one: stats_for)
        return self.bn(self.conv(self.blur(x), stats_for=self.bn))


class QuickNetModule(nn.Module):
    def __init__(self, input_shape, num_classes: int, section_blocks: Sequence[int],
                 section_filters: Sequence[int], backend: str = "torch"):
        super().__init__()
        h, w, c = input_shape
        f0 = section_filters[0]
        self.stem = nn.Sequential(
            QuantConv2d(c, f0 // 4, 3, 2, "same", kernel_initializer="he_normal"),
            BatchNorm(f0 // 4, momentum=0.9, eps=1e-5, activation="relu"),
            QuantConv2d(f0 // 4, f0 // 4, 3, 2, "same", groups=f0 // 4,
                        kernel_initializer="he_normal"),
            BatchNorm(f0 // 4, momentum=0.9, eps=1e-5),
            QuantConv2d(f0 // 4, f0, 1, 1, "valid", kernel_initializer="he_normal"),
            BatchNorm(f0, momentum=0.9, eps=1e-5),
        )
        body, cin = [], f0
        for n, f in zip(section_blocks, section_filters):
            for _ in range(n):
                if f != cin:
                    body.append(Transition(cin, f))
                    cin = f
                body.append(QuickNetBlock(cin, backend))
        # consumer links (plain attributes, not submodules)
        for blk, nxt in zip(body, body[1:]):
            if isinstance(blk, QuickNetBlock) and isinstance(nxt, QuickNetBlock):
                object.__setattr__(blk, "sign_consumer", nxt.conv)
        self.body = nn.Sequential(*body)
        self.pool = GlobalAvgPool()
        self.fc = nn.Linear(cin, num_classes)
        glorot_normal_(self.fc.weight)
        nn.init.zeros_(self.fc.bias)
        self.input_shape, self.num_classes = tuple(input_shape), num_classes

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.body(self.stem(x))
        return pooled_dense(x, self.pool, self.fc, relu=True)


class _QuickNetBase(ModelFactory):
    section_blocks: Sequence[int] = Field((4, 4, 4, 4))
    section_filters: Sequence[int] = Field((64, 128, 256, 512))

    def build(self) -> nn.Module:
        return QuickNetModule(self.input_shape, self.num_classes, self.section_blocks,
                              self.section_filters, self.resolved_backend())


@factory
class QuickNet(_QuickNetBase):
    pass


@factory
class QuickNetLarge(_QuickNetBase):
    section_blocks: Sequence[int] = Field((6, 8, 12, 6))


@factory
class QuickNetXL(_QuickNetBase):
    section_blocks: Sequence[int] = Field((8, 12, 24, 6))
