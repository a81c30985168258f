"""Losses.  Models emit logits; Keras' ``softmax`` activation + the
``sparse_categorical_crossentropy`` loss of the reference example
(examples/larq_experiment.py:101,117) are fused into one softmax-CE that
also yields top-1 correctness, so metrics need no second pass over logits.
"""

from __future__ import annotations

from typing import Callable, Tuple, Union

import torch
import torch.nn.functional as F


def softmax_cross_entropy(logits: torch.Tensor, labels: torch.Tensor,
                          label_smoothing: float = 0.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mean sparse categorical cross-entropy and the number of top-1 hits."""
    from zookeeper_amd import ops

    if logits.is_cuda and ops.available() and hasattr(ops, "softmax_xent"):
        return ops.softmax_xent(logits, labels, label_smoothing)
    logits = logits.float()
    loss = F.cross_entropy(logits, labels, label_smoothing=label_smoothing)
    correct = (logits.argmax(dim=1) == labels).sum()
    return loss, correct


LOSSES = {
    "sparse_categorical_crossentropy": softmax_cross_entropy,
    "softmax_cross_entropy": softmax_cross_entropy,
}

LossSpec = Union[str, Callable]


def get_loss(spec: LossSpec) -> Callable:
    if callable(spec):
        return spec
    try:
        return LOSSES[spec]
    except KeyError:
        raise ValueError(f"Unknown loss '{spec}'. Known: {sorted(LOSSES)}") from None
