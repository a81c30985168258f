"""Float ResNet-50 (v1.5: stride on the 3×3 conv), bf16 on MFMA.

North-star config 2 of BASELINE.json ("ResNet-50 float bf16 ImageNet-shape on
1 MI355X").  Layers are NHWC (channels_last) throughout; BN momentum 0.9,
eps 1e-5; the last BN of every bottleneck starts at γ = 0.
"""

from __future__ import annotations

from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from zookeeper_amd.core import Field, factory
from zookeeper_amd.models.base import ModelFactory
from zookeeper_amd.nn.layers import (BatchNorm, GlobalAvgPool, ImageStem, MaxPool2d, QuantConv2d,
                                     _use_native, glorot_normal_, pooled_dense)


class Bottleneck(nn.Module):
    def __init__(self, cin: int, width: int, stride: int):
        super().__init__()
        cout = width * 4
        self.conv1 = QuantConv2d(cin, width, 1, 1, "valid", kernel_initializer="he_normal")
        self.bn1 = BatchNorm(width, 0.9, 1e-5, activation="relu")
        self.conv2 = QuantConv2d(width, width, 3, stride, "same", kernel_initializer="he_normal")
        self.bn2 = BatchNorm(width, 0.9, 1e-5, activation="relu")
        self.conv3 = QuantConv2d(width, cout, 1, 1, "valid", kernel_initializer="he_normal")
        self.bn3 = BatchNorm(cout, 0.9, 1e-5)
        nn.init.zeros_(self.bn3.weight)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(
                QuantConv2d(cin, cout, 1, stride, "valid", kernel_initializer="he_normal"),
                BatchNorm(cout, 0.9, 1e-5),
            )

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        handoff = give = None
        if self.down is not None:
            dconv, dbn = self.down
            if self.conv1.uses_pointwise(x) and (dconv.uses_pointwise(x)
                                                 or dconv.uses_native_conv(x)):
                from zookeeper_amd.ops import norm_pool

                # x's two gradients (conv1 + shortcut conv) summed in the
                # shortcut conv's data-gradient epilogue: conv1's backward
                # runs first and leaves its gradient there
                give = norm_pool.ResidualHandoff()
                idt = dbn(dconv(x, handoff=give, stats_for=dbn))
            else:
                idt = self.down(x)
        else:
            idt = x
            if self.conv1.uses_pointwise(x):
                from zookeeper_amd.ops import norm_pool

                if norm_pool.supported(x):  # the tail's channels = x's (identity)
                    # x's two gradients (shortcut + main path) summed in conv1's
                    # data-gradient epilogue instead of a separate add pass
                    handoff = norm_pool.ResidualHandoff()
        # stats_for: a 1x1 conv's GEMM epilogue also sums the next BN's batch
        # statistics (no separate statistics pass over its output)
        if handoff is not None:
            y = self.bn1(self.conv1(x, handoff=handoff, stats_for=self.bn1))
        elif give is not None:
            y = self.bn1(self.conv1(x, give=give, stats_for=self.bn1))
        else:
            y = self.bn1(self.conv1(x, stats_for=self.bn1))
        y = self.bn2(self.conv2(y, stats_for=self.bn2))
        y = self.conv3(y, stats_for=self.bn3)
        if _use_native(y):
            from zookeeper_amd.ops import norm_pool

            if norm_pool.supported(y):
                # relu(bn3(y) + shortcut) in one pass (and one pass back)
                return norm_pool.batch_norm(y, self.bn3, relu=True, residual=idt,
                                            handoff=handoff)
        if handoff is not None:
            raise RuntimeError("residual hand-off without the native BN tail")
        return F.relu(self.bn3(y) + idt)


class ResNetModule(nn.Module):
    def __init__(self, input_shape, num_classes: int, blocks: Sequence[int] = (3, 4, 6, 3)):
        super().__init__()
        c = input_shape[2]
        self.stem = ImageStem(
            QuantConv2d(c, 64, 7, 2, "same", kernel_initializer="he_normal"),
            BatchNorm(64, 0.9, 1e-5, activation="relu"),
            MaxPool2d(3, 2, "same"),
        )
        layers, cin = [], 64
        for stage, n in enumerate(blocks):
            width = 64 * 2**stage
            for i in range(n):
                layers.append(Bottleneck(cin, width, 2 if (i == 0 and stage > 0) else 1))
                cin = width * 4
        self.body = nn.Sequential(*layers)
        self.pool = GlobalAvgPool()
        self.fc = nn.Linear(cin, num_classes)
        glorot_normal_(self.fc.weight)
        nn.init.zeros_(self.fc.bias)
        self.input_shape, self.num_classes = tuple(input_shape), num_classes

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return pooled_dense(self.body(self.stem(x)), self.pool, self.fc, relu=False)


@factory
class ResNet50(ModelFactory):
    blocks: Sequence[int] = Field((3, 4, 6, 3))

    def build(self) -> nn.Module:
        return ResNetModule(self.input_shape, self.num_classes, self.blocks)
