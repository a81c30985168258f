"""The training step: forward → fused softmax-CE → backward with bucketed
RCCL all-reduce overlapped → fused optimizer (+ ``weight_clip``) on the flat
buffers.

This is the hot loop that the reference delegates to ``keras.Model.fit``
(HOT LOOP #2).  Nothing in :meth:`Trainer.train_step` touches a
component field or synchronises with the host: losses and hit counts stay on
the device until the metrics logger flushes.
"""

from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.nn as nn

from zookeeper_amd.ops import streams
from zookeeper_amd.parallel import dist as zdist
from zookeeper_amd.parallel.ddp import GradBucketer
from zookeeper_amd.parallel.flat import FlatParams
from zookeeper_amd.train.losses import get_loss
from zookeeper_amd.train.optimizers import OptimizerSpec


def prepare_model(model: nn.Module, device: torch.device) -> nn.Module:
    """Move to the device with NHWC (channels_last) conv kernels."""
    model = model.to(device)
    for m in model.modules():
        for name, p in list(m.named_parameters(recurse=False)):
            if p.dim() == 4 and not p.is_contiguous(memory_format=torch.channels_last):
                p.data = p.data.contiguous(memory_format=torch.channels_last)
    return model


class Trainer:
    def __init__(self, model: nn.Module, loss, optimizer: OptimizerSpec,
                 info: Optional[zdist.DistInfo] = None, bucket_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, grad_dtype: Optional[torch.dtype] = None):
        self.info = info or zdist.info()
        self.device = self.info.device
        self.model = prepare_model(model, self.device)
        self.model.train()
        self.loss_fn: Callable = get_loss(loss)
        self.flat = FlatParams(self.model, self.device)
        if self.info.world > 1:
            # One broadcast of the flat parameter buffer + the BN buffers.
            zdist.broadcast_(self.flat.data)
            for b in self.model.buffers():
                zdist.broadcast_(b)
        self.bucketer = GradBucketer(self.flat, self.info.world, bucket_mb, first_bucket_mb,
                                     grad_dtype=grad_dtype)
        self.optimizer = optimizer.create(self.flat, grad_scale=1.0 / self.info.world)

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        self.flat.zero_grad()
        logits = self.model(x)
        loss, correct = self.loss_fn(logits, y)
        # binary-conv weight gradients on a side stream, ordered by events
        with streams.session(self.device):
            loss.backward()
        self.bucketer.finish()
        self.optimizer.step()
        return loss.detach(), correct

    @torch.no_grad()
    def eval_step(self, x: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        was = self.model.training
        self.model.eval()
        try:
            logits = self.model(x)
            return self.loss_fn(logits, y)
        finally:
            self.model.train(was)
