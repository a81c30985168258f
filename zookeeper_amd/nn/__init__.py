"""NHWC layers with Keras/Larq semantics and binarisation quantizers."""

from zookeeper_amd.nn.layers import (
    AvgPool2d,
    BatchNorm,
    Flatten,
    GlobalAvgPool,
    MaxPool2d,
    QuantConv2d,
    QuantDense,
    apply_constraints,
    same_padding,
)
from zookeeper_amd.nn.quantizers import (
    approx_sign,
    get_quantizer,
    magnitude_aware_sign,
    sign_pm1,
    ste_sign,
    swish_sign,
    weight_clip,
)

__all__ = [
    "apply_constraints",
    "approx_sign",
    "AvgPool2d",
    "BatchNorm",
    "Flatten",
    "get_quantizer",
    "GlobalAvgPool",
    "magnitude_aware_sign",
    "MaxPool2d",
    "QuantConv2d",
    "QuantDense",
    "same_padding",
    "sign_pm1",
    "ste_sign",
    "swish_sign",
    "weight_clip",
]
