"""BinaryNet (Courbariaux et al., 2016) — the reference example's model.

Layer stack of examples/larq_experiment.py:59-103 (shapes for MNIST /
CIFAR-10 in SURVEY §2.4): six 3×3 quantized convs (the first with a float
input), three 2×2 max-pools, three quantized dense layers, a
``BatchNormalization(scale=False)`` after every quantized layer, and a
softmax (fused into the loss here).
"""

from __future__ import annotations

from typing import Tuple, Union

import torch
import torch.nn as nn

from zookeeper_amd.core import Field, factory
from zookeeper_amd.models.base import ModelFactory
from zookeeper_amd.nn.layers import BatchNorm, Flatten, MaxPool2d, QuantConv2d, QuantDense, conv_out_size


class BinaryNetModule(nn.Module):
    def __init__(self, input_shape: Tuple[int, int, int], num_classes: int, filters: int = 128,
                 dense_units: int = 1024, kernel_size: Union[int, Tuple[int, int]] = 3,
                 momentum: float = 0.99, eps: float = 1e-3):
        super().__init__()
        h, w, c = input_shape
        k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        q = dict(input_quantizer="ste_sign", kernel_quantizer="ste_sign",
                 kernel_constraint="weight_clip")

        def bn(n):
            return BatchNorm(n, momentum=momentum, eps=eps, scale=False)

        layers = [
            # The first layer's input is not quantized (float pixels).
            QuantConv2d(c, filters, kernel_size, 1, "valid", None, "ste_sign", "weight_clip"),
            bn(filters),
            QuantConv2d(filters, filters, kernel_size, 1, "same", **q),
            MaxPool2d(2, 2),
            bn(filters),
            QuantConv2d(filters, 2 * filters, kernel_size, 1, "same", **q),
            bn(2 * filters),
            QuantConv2d(2 * filters, 2 * filters, kernel_size, 1, "same", **q),
            MaxPool2d(2, 2),
            bn(2 * filters),
            QuantConv2d(2 * filters, 4 * filters, kernel_size, 1, "same", **q),
            bn(4 * filters),
            QuantConv2d(4 * filters, 4 * filters, kernel_size, 1, "same", **q),
            MaxPool2d(2, 2),
            bn(4 * filters),
            Flatten(),
        ]
        hh = conv_out_size(h, k, 1, "valid") // 2 // 2 // 2
        ww = conv_out_size(w, k, 1, "valid") // 2 // 2 // 2
        flat = hh * ww * 4 * filters
        layers += [
            QuantDense(flat, dense_units, **q),
            BatchNorm(dense_units, momentum=momentum, eps=eps, scale=False),
            QuantDense(dense_units, dense_units, **q),
            BatchNorm(dense_units, momentum=momentum, eps=eps, scale=False),
            QuantDense(dense_units, num_classes, **q),
            BatchNorm(num_classes, momentum=momentum, eps=eps, scale=False),
        ]
        self.layers = nn.Sequential(*layers)
        self.input_shape, self.num_classes = tuple(input_shape), num_classes

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.layers(x).float()


@factory
class BinaryNet(ModelFactory):
    """``@factory`` building :class:`BinaryNetModule` (reference:
    examples/larq_experiment.py:40-103)."""

    filters: int = Field(128)
    dense_units: int = Field(1024)
    kernel_size: Union[int, Tuple[int, int]] = Field((3, 3))

    def build(self) -> nn.Module:
        return BinaryNetModule(self.input_shape, self.num_classes, self.filters,
                               self.dense_units, self.kernel_size)
