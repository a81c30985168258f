"""Layers with Keras/Larq semantics on NHWC (``channels_last``) tensors.

Reference usage: the BinaryNet example builds ``lq.layers.QuantConv2D`` /
``QuantDense`` + ``BatchNormalization(scale=False)`` stacks
(examples/larq_experiment.py:59-103).  These modules reproduce those layer
semantics in PyTorch:

* ``padding="same"`` follows TensorFlow: the total padding
  ``max((out-1)*s + k - in, 0)`` is split ``total//2`` before and the rest
  after (asymmetric for even inputs with stride 2);
* quantized layers binarise inputs/kernels with the named quantizer and apply
  ``kernel_constraint`` (``weight_clip``) after each optimizer step;
* ``BatchNorm`` uses Keras' momentum convention
  (``moving = momentum*moving + (1-momentum)*batch``) and ``scale``/``center``
  switches (``scale=False`` ⇒ no γ).

Weights are stored ``[out, in, kh, kw]`` in ``channels_last`` memory format,
i.e. physically OHWI — the layout the HIP implicit-GEMM kernels consume.
"""

from __future__ import annotations

import math
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

from zookeeper_amd.nn.quantizers import CONSTRAINTS, Quantizer, get_quantizer

IntPair = Union[int, Tuple[int, int]]


def _pair(v: IntPair) -> Tuple[int, int]:
    return (v, v) if isinstance(v, int) else tuple(v)  # type: ignore[return-value]


# 1x1 convs as MFMA GEMMs (ops/pointwise.py); ``runtime.pw_gemm=False`` keeps
# them on the library convolution (A/B measurements)


def _pw_gemm() -> bool:
    from zookeeper_amd.ops.options import OPTS

    return OPTS.pw_gemm


def _use_native(x: torch.Tensor) -> bool:
    """HIP kernels run for bf16 tensors on the GPU when the library is loaded."""
    if not (x.is_cuda and x.dtype == torch.bfloat16):
        return False
    from zookeeper_amd.ops import _native

    if _native.available():
        return True
    if _native.load_error() == "disabled by ZK_NATIVE=0":
        return False
    # A GPU tensor without the kernels is a broken install, not a fallback.
    raise RuntimeError(f"zookeeper_amd native library unavailable: {_native.load_error()}")


def same_padding(size: int, kernel: int, stride: int, dilation: int = 1) -> Tuple[int, int]:
    """TensorFlow ``SAME`` padding (before, after) for one spatial dim."""
    eff = (kernel - 1) * dilation + 1
    out = math.ceil(size / stride)
    total = max((out - 1) * stride + eff - size, 0)
    return total // 2, total - total // 2


def conv_out_size(size: int, kernel: int, stride: int, padding: str) -> int:
    if padding == "same":
        return math.ceil(size / stride)
    return (size - kernel) // stride + 1


def pad_same_nhwc(x: torch.Tensor, kernel: Tuple[int, int], stride: Tuple[int, int],
                  value: float = 0.0) -> torch.Tensor:
    """Pad an NCHW-shaped (channels_last-strided) tensor TF-``SAME`` style."""
    ph = same_padding(x.shape[2], kernel[0], stride[0])
    pw = same_padding(x.shape[3], kernel[1], stride[1])
    if ph == (0, 0) and pw == (0, 0):
        return x
    return F.pad(x, (pw[0], pw[1], ph[0], ph[1]), value=value)


def glorot_normal_(w: torch.Tensor) -> torch.Tensor:
    """Keras ``glorot_normal`` (truncated normal, std = sqrt(2/(fan_in+fan_out)))."""
    receptive = w[0][0].numel() if w.dim() > 2 else 1
    fan_in, fan_out = w.shape[1] * receptive, w.shape[0] * receptive
    std = math.sqrt(2.0 / (fan_in + fan_out)) / 0.87962566103423978
    with torch.no_grad():
        return nn.init.trunc_normal_(w, 0.0, std, -2 * std, 2 * std)


def he_normal_(w: torch.Tensor) -> torch.Tensor:
    receptive = w[0][0].numel() if w.dim() > 2 else 1
    fan_in = w.shape[1] * receptive
    std = math.sqrt(2.0 / fan_in) / 0.87962566103423978
    with torch.no_grad():
        return nn.init.trunc_normal_(w, 0.0, std, -2 * std, 2 * std)


INITIALIZERS = {"glorot_normal": glorot_normal_, "he_normal": he_normal_}


class QuantConv2d(nn.Module):
    """2-D convolution with optional input/kernel quantizers (Larq
    ``QuantConv2D`` semantics).  With both quantizers ``None`` this is a plain
    float convolution."""

    def __init__(
        self,
        in_channels: int,
        out_channels: int,
        kernel_size: IntPair,
        stride: IntPair = 1,
        padding: str = "valid",
        input_quantizer: Quantizer = None,
        kernel_quantizer: Quantizer = None,
        kernel_constraint: Optional[str] = None,
        use_bias: bool = False,
        groups: int = 1,
        pad_values: float = 0.0,
        kernel_initializer: str = "glorot_normal",
    ):
        super().__init__()
        if padding not in ("same", "valid"):
            raise ValueError(f"padding must be 'same' or 'valid', got {padding!r}")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride = _pair(kernel_size), _pair(stride)
        self.padding, self.groups, self.pad_values = padding, groups, pad_values
        self.input_quantizer_name = input_quantizer if isinstance(input_quantizer, str) else None
        self.kernel_quantizer_name = kernel_quantizer if isinstance(kernel_quantizer, str) else None
        self.input_quantizer = get_quantizer(input_quantizer)
        self.kernel_quantizer = get_quantizer(kernel_quantizer)
        self.kernel_constraint = kernel_constraint
        w = torch.empty(out_channels, in_channels // groups, *self.kernel_size)
        INITIALIZERS[kernel_initializer](w)
        self.weight = nn.Parameter(w.contiguous(memory_format=torch.channels_last))
        self.bias = nn.Parameter(torch.zeros(out_channels)) if use_bias else None

    def extra_repr(self) -> str:
        return (
            f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
            f"stride={self.stride}, padding={self.padding!r}, "
            f"input_quantizer={self.input_quantizer_name}, "
            f"kernel_quantizer={self.kernel_quantizer_name}"
        )

    def quantized_weight(self) -> torch.Tensor:
        w = self.weight
        return self.kernel_quantizer(w) if self.kernel_quantizer is not None else w

    def _is_depthwise3x3(self) -> bool:
        return (self.groups == self.in_channels == self.out_channels and self.kernel_size == (3, 3)
                and self.stride[0] == self.stride[1] and self.input_quantizer is None
                and self.kernel_quantizer is None and self.bias is None and self.pad_values == 0.0)

    def uses_pointwise(self, x: torch.Tensor) -> bool:
        """True when ``forward(x)`` runs on the native 1×1 GEMM path
        (``ops/pointwise.py``), which can take a residual-gradient hand-off."""
        if not (self.input_quantizer is None and self.kernel_quantizer is None
                and self.kernel_size == (1, 1) and _pw_gemm() and _use_native(x)):
            return False
        from zookeeper_amd.ops import pointwise

        return pointwise.supported(x, self.weight, self.stride, self.groups, self.bias)

    def uses_native_conv(self, x: torch.Tensor) -> bool:
        """True when ``forward(x)`` runs on the native float-conv path
        (``ops/conv.py``, any stride), which can consume a gradient hand-off."""
        if not (self.input_quantizer is None and self.kernel_quantizer is None
                and _use_native(x)):
            return False
        from zookeeper_amd.ops import conv as conv_op

        return conv_op.supported(x, self.weight, self.stride, self.padding, self.groups,
                                 self.bias, self.pad_values)

    def forward(self, x: torch.Tensor, handoff=None, give=None, stats_for=None) -> torch.Tensor:
        """``stats_for``: the BatchNorm that normalises the output next (its
        statistics then come from the 1x1 GEMM's epilogue, ops/pointwise.py);
        ignored by the other paths."""
        if handoff is not None or give is not None:
            # gradient hand-off (norm_pool.ResidualHandoff); the caller checked
            # uses_pointwise(x) / uses_native_conv(x) (see models/resnet.py)
            if self.uses_pointwise(x):
                from zookeeper_amd.ops import pointwise

                return pointwise.conv1x1(x, self.weight, handoff, give, stats_for)
            if give is None and self.uses_native_conv(x):
                from zookeeper_amd.ops import conv as conv_op

                return conv_op.conv2d(x, self.weight, self.stride[0], self.padding,
                                      handoff=handoff)
            raise RuntimeError("gradient hand-off needs the native 1x1 / conv path")
        if self.groups > 1 and self._is_depthwise3x3() and _use_native(x):
            from zookeeper_amd.ops import depthwise

            if depthwise.supported(x, self.weight):
                return depthwise.depthwise_conv3x3(x, self.weight, self.stride[0], self.padding)
        if (self.input_quantizer is None and self.kernel_quantizer is None
                and self.kernel_size == (1, 1) and _pw_gemm() and _use_native(x)):
            from zookeeper_amd.ops import pointwise

            if pointwise.supported(x, self.weight, self.stride, self.groups, self.bias):
                return pointwise.conv1x1(x, self.weight, stats_for=stats_for)
        if (self.input_quantizer is None and self.kernel_quantizer is None
                and self.kernel_size == (3, 3) and _use_native(x)):
            from zookeeper_amd.ops import conv3x3

            if conv3x3.supported(x, self.weight, self.stride, self.padding, self.groups,
                                 self.bias, self.pad_values):
                return conv3x3.conv3x3(x, self.weight, stats_for=stats_for)
        if self._binary() and _use_native(x):
            from zookeeper_amd.ops import bconv

            if bconv.conv_supported(x, self.weight, self.stride, self.padding, self.groups,
                                    self.bias, self.pad_values):
                clip = getattr(self, "clip_value", 1.0)
                return bconv.binary_conv(x, self.weight, self.stride[0], self.padding, clip,
                                         clip, self.pad_values, owner=self)
        if (self.input_quantizer is None and self.kernel_quantizer is None
                and _use_native(x)):
            from zookeeper_amd.ops import conv as conv_op

            if conv_op.supported(x, self.weight, self.stride, self.padding, self.groups,
                                 self.bias, self.pad_values):
                return conv_op.conv2d(x, self.weight, self.stride[0], self.padding)
        if (self.input_quantizer is None and self.kernel_quantizer_name in (None, "ste_sign")
                and (self.kernel_quantizer is None or self.kernel_quantizer_name == "ste_sign")
                and _use_native(x)):
            from zookeeper_amd.ops import smallconv

            if smallconv.supported(x, self.weight, self.stride, self.padding, self.groups,
                                   self.bias, self.pad_values):
                kclip = getattr(self, "clip_value", 1.0) if self.kernel_quantizer else None
                return smallconv.small_conv(x, self.weight, self.stride[0], self.padding, kclip)
        if self.input_quantizer is not None:
            x = self.input_quantizer(x)
        if self.padding == "same":
            x = pad_same_nhwc(x, self.kernel_size, self.stride, self.pad_values)
        w = self.quantized_weight().to(x.dtype)
        b = self.bias.to(x.dtype) if self.bias is not None else None
        return F.conv2d(x, w, b, self.stride, 0, 1, self.groups)

    def _binary(self) -> bool:
        """ste_sign on both the input and the kernel (Larq's binary layer)."""
        return self.input_quantizer_name == "ste_sign" and self.kernel_quantizer_name == "ste_sign"

    def apply_constraints(self) -> None:
        if self.kernel_constraint is not None:
            CONSTRAINTS[self.kernel_constraint](self.weight)


class QuantDense(nn.Module):
    """Fully-connected layer with optional quantizers (Larq ``QuantDense``)."""

    def __init__(
        self,
        in_features: int,
        out_features: int,
        input_quantizer: Quantizer = None,
        kernel_quantizer: Quantizer = None,
        kernel_constraint: Optional[str] = None,
        use_bias: bool = False,
        kernel_initializer: str = "glorot_normal",
    ):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.input_quantizer_name = input_quantizer if isinstance(input_quantizer, str) else None
        self.kernel_quantizer_name = kernel_quantizer if isinstance(kernel_quantizer, str) else None
        self.input_quantizer = get_quantizer(input_quantizer)
        self.kernel_quantizer = get_quantizer(kernel_quantizer)
        self.kernel_constraint = kernel_constraint
        w = torch.empty(out_features, in_features)
        INITIALIZERS[kernel_initializer](w)
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(torch.zeros(out_features)) if use_bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (self.input_quantizer_name == "ste_sign" and self.kernel_quantizer_name == "ste_sign"
                and _use_native(x)):
            from zookeeper_amd.ops import bconv

            if bconv.dense_supported(x, self.weight, self.bias):
                clip = getattr(self, "clip_value", 1.0)
                return bconv.binary_dense(x, self.weight, clip, clip, owner=self)
        if self.input_quantizer is not None:
            x = self.input_quantizer(x)
        w = self.weight
        if self.kernel_quantizer is not None:
            w = self.kernel_quantizer(w)
        b = self.bias.to(x.dtype) if self.bias is not None else None
        return F.linear(x, w.to(x.dtype), b)

    def apply_constraints(self) -> None:
        if self.kernel_constraint is not None:
            CONSTRAINTS[self.kernel_constraint](self.weight)


class BatchNorm(nn.Module):
    """Batch normalisation over the channel dim with Keras conventions.

    ``momentum`` is Keras' (0.99 default ⇒ torch momentum 0.01); ``scale=False``
    drops γ, ``center=False`` drops β.  Works on ``[N, C]`` and NCHW-shaped
    (channels_last) tensors; statistics are computed in fp32.
    """

    def __init__(self, num_features: int, momentum: float = 0.99, eps: float = 1e-3,
                 scale: bool = True, center: bool = True, activation: Optional[str] = None):
        super().__init__()
        if activation not in (None, "relu"):
            raise ValueError("BatchNorm activation must be None or 'relu'")
        self.num_features, self.momentum, self.eps = num_features, momentum, eps
        self.activation = activation
        self.weight = nn.Parameter(torch.ones(num_features)) if scale else None
        self.bias = nn.Parameter(torch.zeros(num_features)) if center else None
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))

    def extra_repr(self) -> str:
        return (f"{self.num_features}, momentum={self.momentum}, eps={self.eps}, "
                f"scale={self.weight is not None}, center={self.bias is not None}")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        relu = self.activation == "relu"
        if _use_native(x):
            from zookeeper_amd.ops import norm_pool

            if norm_pool.supported(x):
                return norm_pool.batch_norm(x, self, relu)
            y = self._formula(x.float())  # e.g. a 10-way classifier's BN: tiny
            return (F.relu(y) if relu else y).to(x.dtype)
        if x.is_cuda:
            # the fp32 oracle on the GPU: explicit arithmetic, not the library
            # BN (MIOpen's backward mis-shapes the bias gradient when scale=False)
            y = self._formula(x.float()).to(x.dtype)
            return F.relu(y) if relu else y
        w = self.weight
        b = self.bias
        if x.dtype != torch.float32:
            # Oracle path: compute in fp32, return in the input dtype.
            y = F.batch_norm(x.float(), self.running_mean, self.running_var, w, b,
                             self.training, 1.0 - self.momentum, self.eps)
            y = y.to(x.dtype)
        else:
            y = F.batch_norm(x, self.running_mean, self.running_var, w, b, self.training,
                             1.0 - self.momentum, self.eps)
        return F.relu(y) if relu else y


    def _formula(self, x: torch.Tensor) -> torch.Tensor:
        """Batch norm as plain fp32 tensor arithmetic (no library BN kernel)."""
        dims = [0] + list(range(2, x.dim()))
        shape = [1, -1] + [1] * (x.dim() - 2)
        if self.training:
            mean = x.mean(dim=dims)
            var = x.var(dim=dims, unbiased=False)
            n = x.numel() // x.shape[1]
            with torch.no_grad():
                m = 1.0 - self.momentum
                self.running_mean.mul_(1 - m).add_(mean.detach(), alpha=m)
                self.running_var.mul_(1 - m).add_(var.detach() * n / max(n - 1, 1), alpha=m)
        else:
            mean, var = self.running_mean, self.running_var
        y = (x - mean.view(shape)) * torch.rsqrt(var.view(shape) + self.eps)
        if self.weight is not None:
            y = y * self.weight.view(shape)
        if self.bias is not None:
            y = y + self.bias.view(shape)
        return y


class MaxPool2d(nn.Module):
    """Max pooling with TF ``same``/``valid`` padding semantics."""

    def __init__(self, pool_size: IntPair = 2, stride: Optional[IntPair] = None,
                 padding: str = "valid"):
        super().__init__()
        self.pool_size = _pair(pool_size)
        self.stride = _pair(stride if stride is not None else pool_size)
        self.padding = padding

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        k, s = self.pool_size, self.stride
        if _use_native(x) and x.dim() == 4 and x.shape[1] % 8 == 0 and k[0] == k[1] and s[0] == s[1]:
            from zookeeper_amd.ops import norm_pool

            return norm_pool.max_pool(x, k[0], s[0], self.padding)
        if self.padding == "same":
            x = pad_same_nhwc(x, self.pool_size, self.stride, float("-inf"))
        return F.max_pool2d(x, self.pool_size, self.stride)


class AvgPool2d(nn.Module):
    """Average pooling (``valid`` padding, the only form the model zoo uses)."""

    def __init__(self, pool_size: IntPair = 2, stride: Optional[IntPair] = None):
        super().__init__()
        self.pool_size = _pair(pool_size)
        self.stride = _pair(stride if stride is not None else pool_size)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (_use_native(x) and x.dim() == 4 and x.shape[1] % 8 == 0
                and self.pool_size == (2, 2) and self.stride == (2, 2)):
            from zookeeper_amd.ops import norm_pool

            return norm_pool.avg_pool2(x)
        return F.avg_pool2d(x, self.pool_size, self.stride)


class GlobalAvgPool(nn.Module):
    """Keras ``GlobalAveragePooling2D``; channels-last bf16 maps on the GPU run
    the native pool kernel (``ops/head.py``), fp32 accumulation."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _use_native(x):
            from zookeeper_amd.ops.head import gap_supported, global_avg_pool

            if gap_supported(x):
                return global_avg_pool(x)
        return x.mean(dim=(2, 3))


def pooled_dense(x: torch.Tensor, pool: nn.Module, fc: nn.Linear, relu: bool) -> torch.Tensor:
    """fp32 logits of the ImageNet models' head: ``fc(pool(relu?(x)).float())``.

    Native path (bf16 channels-last on the GPU): one fused ReLU + average-pool
    kernel and fp32 MFMA GEMMs for the dense layer, forward and backward
    (``ops/head.py``) -- no library kernel.  Else the PyTorch ops."""
    if _use_native(x):
        from zookeeper_amd.ops.head import classifier_head, head_supported

        if head_supported(x, fc.weight):
            return classifier_head(x, fc.weight, fc.bias, relu)
    if relu:
        x = F.relu(x)
    return F.linear(pool(x).float(), fc.weight, fc.bias)


class Flatten(nn.Module):
    """Flatten in NHWC order (Keras ``Flatten`` on channels-last tensors)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


def apply_constraints(model: nn.Module) -> None:
    """Apply every layer's kernel constraint (call after the optimizer step)."""
    for m in model.modules():
        fn = getattr(m, "apply_constraints", None)
        if fn is not None and m is not model:
            fn()


class ImageStem(nn.Sequential):
    """``conv → BN(+ReLU) → MaxPool [→ BN]`` ImageNet stem as an
    ``nn.Sequential`` (parameter names ``0.weight``, ``1.weight``, ...).

    On bf16 GPU tensors the whole stem runs as the fused HIP pipeline of
    :mod:`zookeeper_amd.ops.stem` (MFMA conv with BN statistics in its
    epilogue, BN+ReLU+pool in one pass, sparse pool backward); otherwise
    the modules run one after the other.

    ``sign_clip``: when set (by a model whose next layer is a binary block
    quantising its input with this clip value), the fused stem also emits
    that block's sign image / STE mask in its final BN pass.
    """

    sign_clip: Optional[float] = None
    # ... and that block's conv (decides whether a bf16 sign image is needed)
    sign_consumer = None

    def _fusable(self, x: torch.Tensor) -> bool:
        if not _use_native(x) or len(self) not in (3, 4):
            return False
        conv, bn1, pool = self[0], self[1], self[2]
        bn2 = self[3] if len(self) == 4 else None
        if not (isinstance(conv, QuantConv2d) and isinstance(bn1, BatchNorm)
                and isinstance(pool, MaxPool2d) and bn1.activation == "relu"
                and pool.padding == "same" and (bn2 is None or (isinstance(bn2, BatchNorm)
                                                               and bn2.activation is None))):
            return False
        k, s = _pair(pool.pool_size), _pair(pool.stride)
        if k[0] != k[1] or s[0] != s[1]:
            return False
        # the fused backward assumes batch statistics whenever it runs
        if torch.is_grad_enabled() and not (bn1.training and (bn2 is None or bn2.training)):
            return False
        from zookeeper_amd.ops import stem

        return stem.supported(x, conv, bn1, k[0], s[0])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._fusable(x):
            from zookeeper_amd.ops.stem import fused_stem

            pool = self[2]
            return fused_stem(x, self[0], self[1], _pair(pool.pool_size)[0],
                              _pair(pool.stride)[0], self[3] if len(self) == 4 else None,
                              sign_clip=self.sign_clip, sign_consumer=self.sign_consumer)
        return super().forward(x)
