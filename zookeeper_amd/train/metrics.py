"""Metrics accumulated on the device and flushed every ``log_every`` steps.

Per step the trainer only adds loss and hit counts into device scalars (no
host synchronisation); a flush does one ``.item()`` round-trip, averages
across data-parallel ranks, and appends a JSON line to ``metrics.jsonl`` on
rank 0 (loss, the configured metrics, images/sec per GPU and for the whole
job, step time, and under data parallelism the per-step all-reduce time and
the part of it exposed after backward).  The reference relied on Keras' progress bar and
``compile(metrics=...)`` (examples/larq_experiment.py:118,142).

Configured metric names follow Keras: ``accuracy`` /
``sparse_categorical_accuracy`` (top-1, taken from the fused softmax-CE's
hit count — no second pass over the logits) and
``sparse_top_k_categorical_accuracy`` / ``top5`` / ``top<k>`` (top-k hits
computed on the logits inside the step).  Unknown names raise at set-up.
"""

from __future__ import annotations

import json
import os
import re
import time
from typing import Any, Callable, Dict, Optional, Sequence

import torch
import torch.distributed as dist

_TOP1 = {"accuracy", "acc", "sparse_categorical_accuracy", "top1", "top_1"}
_TOPK = re.compile(r"^top_?(\d+)$")


def topk_hits(k: int) -> Callable[[torch.Tensor, torch.Tensor], torch.Tensor]:
    def fn(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        kk = min(k, logits.shape[1])
        top = logits.topk(kk, dim=1).indices
        return (top == labels.view(-1, 1)).any(dim=1).sum()

    return fn


def comm_summary(timings: Sequence[Dict[str, float]]) -> Dict[str, float]:
    """Median per-step communication of a logging window, from
    ``GradBucketer.pop_timings()``: ``comm_ms`` (first collective start ->
    last end), ``exposed_ms`` (how long communication ran past the end of
    backward).  Empty without data parallelism / timing."""
    if not timings:
        return {}

    def med(key):
        xs = sorted(t[key] for t in timings)
        return xs[len(xs) // 2]

    return {"comm_ms": med("comm_ms"), "exposed_ms": med("exposed_ms"),
            "exposed_ms_max": max(t["exposed_ms"] for t in timings)}


def resolve_metrics(names: Optional[Sequence[str]]) -> Dict[str, Optional[Callable]]:
    """``{record key: None (from the loss) | fn(logits, labels) -> hits}``."""
    out: Dict[str, Optional[Callable]] = {}
    for name in names or ():
        n = str(name).lower()
        if n in _TOP1:
            out["top1"] = None
        elif n == "sparse_top_k_categorical_accuracy":
            out["top5"] = topk_hits(5)
        elif _TOPK.match(n):
            k = int(_TOPK.match(n).group(1))
            out[f"top{k}"] = None if k == 1 else topk_hits(k)
        elif n in ("loss", "crossentropy", "sparse_categorical_crossentropy"):
            continue  # the loss is always logged
        else:
            raise ValueError(
                f"Unknown metric '{name}'. Known: accuracy, sparse_categorical_accuracy, "
                "sparse_top_k_categorical_accuracy, top<k>.")
    return out


class MetricsLogger:
    def __init__(self, device: torch.device, path: Optional[str] = None, rank: int = 0,
                 world: int = 1, echo: bool = True,
                 metrics: Optional[Sequence[str]] = ("accuracy",)):
        self.device, self.path, self.rank, self.world, self.echo = device, path, rank, world, echo
        self.metric_fns = resolve_metrics(metrics)
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=device)
        self.hits = {k: torch.zeros((), dtype=torch.float32, device=device)
                     for k in self.metric_fns}
        self.examples = 0
        self.steps = 0
        self._t0 = time.perf_counter()
        if path and rank == 0:
            os.makedirs(os.path.dirname(path), exist_ok=True)

    @property
    def logit_metrics(self) -> Dict[str, Callable]:
        """The metrics that need the logits (computed by the trainer)."""
        return {k: f for k, f in self.metric_fns.items() if f is not None}

    def update(self, loss: torch.Tensor, correct: torch.Tensor, batch: int,
               extra: Optional[Dict[str, torch.Tensor]] = None) -> None:
        self.loss_sum += loss.detach().float()
        for k, acc in self.hits.items():
            if self.metric_fns[k] is None:
                acc += correct.detach().float()
            elif extra is not None and k in extra:
                acc += extra[k].detach().float()
        self.examples += batch
        self.steps += 1

    def exclude(self, seconds: float) -> None:
        """Leave ``seconds`` (validation, checkpoints) out of the next flush's
        throughput."""
        self._t0 += seconds

    def flush(self, step: int, extra: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        if self.steps == 0:
            return {}
        keys = list(self.hits)
        vals = torch.stack([self.loss_sum] + [self.hits[k] for k in keys]).double()
        if self.world > 1 and dist.is_initialized():
            dist.all_reduce(vals)
        vals = vals.tolist()
        dt = time.perf_counter() - self._t0
        global_examples = self.examples * self.world
        rec = {"step": step, "loss": vals[0] / (self.steps * self.world)}
        for k, v in zip(keys, vals[1:]):
            rec[k] = v / max(global_examples, 1)
        rec.update({
            "images_per_sec": global_examples / dt,
            "images_per_sec_per_gpu": self.examples / dt,
            "step_ms": 1000 * dt / self.steps,
            **(extra or {}),
        })
        if self.rank == 0:
            if self.path:
                with open(self.path, "a") as f:
                    f.write(json.dumps(rec) + "\n")
            if self.echo:
                print(" ".join(f"{k}={v:.5g}" if isinstance(v, float) else f"{k}={v}"
                               for k, v in rec.items()), flush=True)
        self.loss_sum.zero_()
        for acc in self.hits.values():
            acc.zero_()
        self.examples = self.steps = 0
        self._t0 = time.perf_counter()
        return rec
