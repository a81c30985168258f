"""Common base for model @factory components.

Mirrors the structure of the reference example's ``BinaryNet`` factory
(examples/larq_experiment.py:40-49): a model factory declares ``dataset`` and
``input_shape`` fields that it normally *inherits* from the enclosing
experiment (scoped inheritance), and reads ``num_classes`` from the dataset.

Models output **logits**; the trailing ``softmax`` of the Keras models is fused
into the loss (softmax-cross-entropy, ``zookeeper_amd.train.losses``).
"""

from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn

from zookeeper_amd.core.field import ComponentField, Field
from zookeeper_amd.data.dataset import Dataset


class ModelFactory:
    """Fields shared by every model factory (subclass + ``@factory``)."""

    dataset: Dataset = ComponentField()
    input_shape: Tuple[int, int, int] = Field()

    # "auto": the fused HIP kernels on a GPU, the pure-PyTorch oracle path on
    # the CPU.  On a GPU a missing / stale native library raises instead of
    # quietly running the library (MIOpen / hipBLASLt) path; "torch" (or
    # ZK_NATIVE=0) selects that path deliberately.
    backend: str = Field("auto")

    @Field
    def num_classes(self) -> int:
        return self.dataset.num_classes

    def resolved_backend(self) -> str:
        if self.backend != "auto":
            if self.backend not in ("hip", "torch"):
                raise ValueError(f"backend must be 'auto', 'hip' or 'torch', got {self.backend!r}")
            return self.backend
        from zookeeper_amd import ops

        if not torch.cuda.is_available():
            return "torch"
        if ops.available():
            return "hip"
        if ops.native_disabled():
            return "torch"
        raise RuntimeError(
            "backend='auto' on a GPU needs the native library, which did not load: "
            f"{ops.load_error()} (set model.backend='torch' or ZK_NATIVE=0 to run the "
            "PyTorch path on purpose)")


def count_parameters(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())


def summary(model: nn.Module) -> str:
    """A compact parameter summary (the role of ``lq.models.summary``)."""
    lines = [f"{'layer':<48}{'type':<20}{'params':>12}"]
    total = 0
    for name, mod in model.named_modules():
        own = sum(p.numel() for p in mod.parameters(recurse=False))
        if own:
            lines.append(f"{name:<48}{type(mod).__name__:<20}{own:>12,}")
            total += own
    lines.append(f"{'total':<68}{total:>12,}")
    return "\n".join(lines)
