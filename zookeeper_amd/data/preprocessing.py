"""Preprocessing components (batched, on the device).

Parity with zookeeper/tf/preprocessing.py:11-75: a ``Preprocessing`` has
``decoders`` and ``input_shape`` fields, subclasses override
``input(data, training)`` / ``output(data, training)``, and ``__call__``
returns ``(input, output)``, forwarding ``training`` only to overrides that
accept it (the example's ``output(self, data)`` omits it,
examples/larq_experiment.py:36).

Difference by design: the reference maps preprocessing per example on TF's
host thread pool (HOT LOOP #1 in SURVEY §3.4).  Here ``data`` is a *batch*
already on the GPU (``{"image": uint8[B,H,W,C], "label": int64[B]}``) and the
ops are batched tensor ops, so the host never touches pixels after the
pinned copy; ImageNet-style normalisation + flip is one fused HIP kernel when
the extension is available.
"""

from __future__ import annotations

import functools
import inspect
from typing import Any, Callable, Dict, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from zookeeper_amd.core.component import component
from zookeeper_amd.core.field import Field

TensorDict = Dict[str, torch.Tensor]


def pass_training_kwarg(fn, training: bool = False):
    if "training" in inspect.signature(fn).parameters:
        return functools.partial(fn, training=training)
    return fn


class Preprocessing:
    """Batch preprocessing; subclasses implement ``input`` and ``output``."""

    decoders: Optional[Dict[str, Any]] = Field(None)
    # The (H, W, C) shape of one processed input example.
    input_shape: Tuple[int, int, int] = Field()

    def input(self, data: TensorDict, training: bool) -> torch.Tensor:
        raise NotImplementedError("Must be implemented in subclasses.")

    def output(self, data: TensorDict, training: bool) -> torch.Tensor:
        raise NotImplementedError("Must be implemented in subclasses.")

    def device_transform(self, training: bool) -> Optional[Callable[[TensorDict], None]]:
        """Optional: a function the :class:`~zookeeper_amd.data.loader.DeviceLoader`
        runs on its copy stream right after a batch's H2D copy.  It stores the
        model input under ``data["input"]`` (reusing that buffer from the
        slot's previous batch), so the input pipeline's kernels overlap the
        previous step instead of opening the next one on the compute stream;
        :meth:`__call__` then passes ``data["input"]`` through.  ``None`` (the
        default): preprocess in :meth:`input` on the consumer's stream."""
        return None

    def __call__(self, data: TensorDict, training: bool = False):
        output_fn = pass_training_kwarg(self.output, training=training)
        if "input" in data:  # already preprocessed by the loader (device_transform)
            return data["input"], output_fn(data)
        input_fn = pass_training_kwarg(self.input, training=training)
        return input_fn(data), output_fn(data)


def nhwc_to_model(x: torch.Tensor) -> torch.Tensor:
    """``[B,H,W,C]`` (contiguous) → NCHW-shaped ``channels_last`` view (no copy)."""
    return x.permute(0, 3, 1, 2)


def _resize_with_crop_or_pad(img: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """Centre crop / zero-pad ``[B,H,W,C]`` to ``h × w`` (TF semantics)."""
    B, H, W, C = img.shape
    out = img
    if H > h or W > w:
        top, left = max((H - h) // 2, 0), max((W - w) // 2, 0)
        out = out[:, top:top + min(h, H), left:left + min(w, W)]
    H2, W2 = out.shape[1], out.shape[2]
    if H2 < h or W2 < w:
        pt, pl = (h - H2) // 2, (w - W2) // 2
        out = F.pad(out, (0, 0, pl, w - W2 - pl, pt, h - H2 - pt))
    return out


def _random_crop(img: torch.Tensor, h: int, w: int, gen: Optional[torch.Generator]) -> torch.Tensor:
    B, H, W, C = img.shape
    if (H, W) == (h, w):
        return img
    dev = img.device
    tops = torch.randint(0, H - h + 1, (B,), device=dev, generator=gen)
    lefts = torch.randint(0, W - w + 1, (B,), device=dev, generator=gen)
    rows = tops[:, None] + torch.arange(h, device=dev)[None]
    cols = lefts[:, None] + torch.arange(w, device=dev)[None]
    b = torch.arange(B, device=dev)[:, None, None]
    return img[b, rows[:, :, None], cols[:, None, :]]


def _random_flip(img: torch.Tensor, gen: Optional[torch.Generator]) -> torch.Tensor:
    flip = torch.rand(img.shape[0], device=img.device, generator=gen) < 0.5
    return torch.where(flip[:, None, None, None], img.flip(2), img)


@component
class PadCropAndFlip(Preprocessing):
    """CIFAR/MNIST-style augmentation (examples/larq_experiment.py:20-37):
    training pads to ``pad_size``, random-crops to ``input_shape`` and flips;
    evaluation centre-crops/pads.  Pixels are mapped to [-1, 1]."""

    pad_size: int = Field()
    dtype: str = Field("bfloat16")

    def input(self, data: TensorDict, training: bool) -> torch.Tensor:
        image = data["image"]
        h, w = self.input_shape[:2]
        if training:
            image = _resize_with_crop_or_pad(image, self.pad_size, self.pad_size)
            image = _random_crop(image, h, w, None)
            image = _random_flip(image, None)
        else:
            image = _resize_with_crop_or_pad(image, h, w)
        x = image.to(torch.float32) / (255.0 / 2.0) - 1.0
        return nhwc_to_model(x.to(getattr(torch, self.dtype)).contiguous())

    def output(self, data: TensorDict) -> torch.Tensor:
        return data["label"]


@component
class ImageNetPreprocessing(Preprocessing):
    """ImageNet-shape preprocessing: centre crop/pad to ``input_shape``,
    random horizontal flip when training, per-channel ``(x - mean) / std``.

    When the HIP extension is loaded the whole thing (uint8 NHWC → bf16,
    normalise, flip) is a single fused kernel (``ops.normalize_flip``).
    """

    mean: Sequence[float] = Field((0.485 * 255, 0.456 * 255, 0.406 * 255))
    std: Sequence[float] = Field((0.229 * 255, 0.224 * 255, 0.225 * 255))
    flip: bool = Field(True)
    dtype: str = Field("bfloat16")

    def input(self, data: TensorDict, training: bool) -> torch.Tensor:
        image = data["image"]
        h, w = self.input_shape[:2]
        if image.shape[1:3] != (h, w):
            image = _resize_with_crop_or_pad(image, h, w)
        from zookeeper_amd import ops

        if ops.available() and image.is_cuda and self.dtype == "bfloat16":
            return nhwc_to_model(
                ops.normalize_flip(image.contiguous(), self.mean, self.std,
                                   training and self.flip)
            )
        x = image.to(torch.float32)
        if training and self.flip:
            x = _random_flip(x, None)
        mean = torch.tensor(self.mean, device=x.device, dtype=torch.float32)
        std = torch.tensor(self.std, device=x.device, dtype=torch.float32)
        x = (x - mean) / std
        return nhwc_to_model(x.to(getattr(torch, self.dtype)).contiguous())

    def output(self, data: TensorDict) -> torch.Tensor:
        return data["label"]

    def device_transform(self, training: bool) -> Optional[Callable[[TensorDict], None]]:
        """The fused normalise + flip kernel on the loader's copy stream, into a
        per-slot bf16 buffer (0.2 ms per E18 step at batch 1536 off the compute
        stream).  Only when no resize is needed and the kernel is available."""
        from zookeeper_amd import ops

        if not ops.available() or self.dtype != "bfloat16":
            return None
        h, w = self.input_shape[:2]
        flip = training and self.flip

        from zookeeper_amd.ops.stem import PACK_SPECS

        def transform(data: TensorDict) -> None:
            image = data["image"]
            if not image.is_cuda or image.shape[1:3] != (h, w) or image.shape[3] != 3:
                return  # left to input() on the consumer's stream
            buf = data.get("input")
            base = buf.permute(0, 2, 3, 1) if buf is not None else None
            if base is not None and (base.shape != image.shape or not base.is_contiguous()):
                base = None
            spec = PACK_SPECS.get((h, w, 3))
            if spec is None:
                data["input"] = nhwc_to_model(
                    ops.normalize_flip(image, self.mean, self.std, flip, out=base))
                return
            # a fused stem ran on this shape: also write its padded input, in
            # the same pass (the stem then skips its pack kernel)
            xp = data.get("input_xp")
            if xp is not None and xp.shape != (image.shape[0], spec[0], spec[1], 4):
                xp = None
            out, xp = ops.normalize_flip_pack(image, self.mean, self.std, flip, spec,
                                              out=base, xp=xp)
            x = nhwc_to_model(out)
            x._zk_stem_xp = (xp, spec, x._version)
            data["input"], data["input_xp"] = x, xp

        return transform
