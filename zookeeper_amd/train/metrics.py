"""Metrics accumulated on the device and flushed every ``log_every`` steps.

Per step the trainer only adds loss and top-1 hit counts into device scalars
(no host synchronisation); a flush does one ``.item()`` round-trip, averages
across data-parallel ranks, and appends a JSON line to ``metrics.jsonl`` on
rank 0 (loss, top-1 accuracy, images/sec per GPU and for the whole job,
step time).  The reference relied on Keras' progress bar.
"""

from __future__ import annotations

import json
import os
import time
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


class MetricsLogger:
    def __init__(self, device: torch.device, path: Optional[str] = None, rank: int = 0,
                 world: int = 1, echo: bool = True):
        self.device, self.path, self.rank, self.world, self.echo = device, path, rank, world, echo
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=device)
        self.correct = torch.zeros((), dtype=torch.float32, device=device)
        self.examples = 0
        self.steps = 0
        self._t0 = time.perf_counter()
        if path and rank == 0:
            os.makedirs(os.path.dirname(path), exist_ok=True)

    def update(self, loss: torch.Tensor, correct: torch.Tensor, batch: int) -> None:
        self.loss_sum += loss.detach().float()
        self.correct += correct.detach().float()
        self.examples += batch
        self.steps += 1

    def flush(self, step: int, extra: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        if self.steps == 0:
            return {}
        vals = torch.stack([self.loss_sum, self.correct]).double()
        if self.world > 1 and dist.is_initialized():
            dist.all_reduce(vals)
        loss_sum, correct = vals.tolist()
        dt = time.perf_counter() - self._t0
        global_examples = self.examples * self.world
        rec = {
            "step": step,
            "loss": loss_sum / (self.steps * self.world),
            "top1": correct / max(global_examples, 1),
            "images_per_sec": global_examples / dt,
            "images_per_sec_per_gpu": self.examples / dt,
            "step_ms": 1000 * dt / self.steps,
            **(extra or {}),
        }
        if self.rank == 0:
            if self.path:
                with open(self.path, "a") as f:
                    f.write(json.dumps(rec) + "\n")
            if self.echo:
                print(" ".join(f"{k}={v:.5g}" if isinstance(v, float) else f"{k}={v}"
                               for k, v in rec.items()), flush=True)
        self.loss_sum.zero_()
        self.correct.zero_()
        self.examples = self.steps = 0
        self._t0 = time.perf_counter()
        return rec
