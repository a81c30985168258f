"""Optimizer components and the fused flat-buffer optimizer.

The reference builds a Keras optimizer in a ``@Field`` from
``self.learning_rate`` (examples/larq_experiment.py:120-122) and applies
Larq's ``weight_clip`` kernel constraint inside Keras' update.  Here an
optimizer is a ``@component`` *spec* (hyper-parameters, schedule) whose
``create(flat, grad_scale)`` returns a :class:`FlatOptimizer` acting on the
flat parameter/gradient buffers (``zookeeper_amd.parallel.flat``):

* one fused kernel updates every parameter (Adam/AdamW/SGD-momentum) and
  applies ``weight_clip`` to binary kernels in the same pass (per-parameter
  attribute table), with the data-parallel ``1/world`` averaging folded into
  ``grad_scale`` — no separate scaling, clipping or constraint passes;
* on CPU the same math runs as a handful of vectorised torch ops.

``learning_rate`` has no default on the spec, so it is inherited from the
enclosing experiment's ``learning_rate`` field (scoped inheritance), exactly
like the reference's ``Adam(self.learning_rate)``.
"""

from __future__ import annotations

import math
from typing import Any, Dict, Optional

import torch

from zookeeper_amd.core import Field, component
from zookeeper_amd.parallel.flat import FlatParams


class OptimizerSpec:
    learning_rate: float = Field()
    weight_decay: float = Field(0.0)
    # "constant" | "cosine" | "linear" | "step"
    schedule: str = Field("constant")
    warmup_steps: int = Field(0)
    # Total steps for decaying schedules (None → set by the trainer).
    decay_steps: Optional[int] = Field(None)
    min_lr_ratio: float = Field(0.0)
    # For "step": multiply by `step_gamma` every `step_every` steps.
    step_every: int = Field(30)
    step_gamma: float = Field(0.1)

    kind = "base"

    def lr_at(self, step: int, total: Optional[int] = None) -> float:
        base = self.learning_rate
        if self.warmup_steps and step < self.warmup_steps:
            return base * (step + 1) / self.warmup_steps
        total = self.decay_steps or total
        if self.schedule == "constant" or not total:
            return base
        t = min(max(step - self.warmup_steps, 0), max(total - self.warmup_steps, 1))
        span = max(total - self.warmup_steps, 1)
        if self.schedule == "cosine":
            f = 0.5 * (1 + math.cos(math.pi * t / span))
        elif self.schedule == "linear":
            f = 1 - t / span
        elif self.schedule == "step":
            f = self.step_gamma ** (step // max(self.step_every, 1))
            return base * f
        else:
            raise ValueError(f"unknown schedule {self.schedule!r}")
        return base * (self.min_lr_ratio + (1 - self.min_lr_ratio) * f)

    def create(self, flat: FlatParams, grad_scale: float = 1.0) -> "FlatOptimizer":
        return FlatOptimizer(self, flat, grad_scale)


@component
class Adam(OptimizerSpec):
    """Adam (decoupled weight decay ⇒ AdamW when ``weight_decay > 0``).

    ``epsilon_form="keras"`` (default) is the update of the reference's
    ``tf.keras.optimizers.Adam`` (examples/larq_experiment.py:120-122):
    ``p -= lr·√(1-β₂ᵗ)/(1-β₁ᵗ) · m/(√v + ε)``, i.e. ε is added to the raw
    √v ("epsilon hat").  ``"textbook"`` is Kingma & Ba's / PyTorch's
    ``p -= lr · m̂/(√v̂ + ε)`` with bias-corrected moments.  The two differ
    only in how large ε acts during the first steps (by √(1-β₂ᵗ)), which
    matters for binary networks with tiny latent-weight gradients.  The
    fused kernel computes the textbook form; the Keras form is the same
    kernel with ε/√(1-β₂ᵗ)."""

    beta_1: float = Field(0.9)
    beta_2: float = Field(0.999)
    epsilon: float = Field(1e-7)  # Keras' default
    epsilon_form: str = Field("keras")

    kind = "adam"

    def eps_effective(self, t: int) -> float:
        """ε to use in the textbook form at step ``t`` so that it equals the
        configured form."""
        if self.epsilon_form == "textbook":
            return self.epsilon
        if self.epsilon_form == "keras":
            return self.epsilon / math.sqrt(1.0 - self.beta_2 ** t)
        raise ValueError(f"epsilon_form must be 'keras' or 'textbook', got {self.epsilon_form!r}")


@component
class SGD(OptimizerSpec):
    """SGD with (optionally Nesterov) momentum and L2 weight decay."""

    momentum: float = Field(0.9)
    nesterov: bool = Field(False)

    kind = "sgd"


class FlatOptimizer:
    """Fused optimizer over :class:`FlatParams`."""

    def __init__(self, spec: OptimizerSpec, flat: FlatParams, grad_scale: float = 1.0):
        self.spec, self.flat, self.grad_scale = spec, flat, grad_scale
        self.step_count = 0
        self.total_steps: Optional[int] = None
        dev = flat.data.device
        self.m = torch.zeros_like(flat.data)
        self.v = torch.zeros_like(flat.data) if spec.kind == "adam" else None
        self.table = flat.table().to(dev)
        # Per-element constraint / decay vectors for the torch path only.
        self._clip_vec = None
        self._decay_vec = None

    # -- torch reference implementation ------------------------------------ #

    def _vectors(self):
        if self._clip_vec is None:
            clip = torch.zeros_like(self.flat.data)
            decay = torch.zeros_like(self.flat.data)
            for s in self.flat.slots:
                clip[s.offset:s.offset + s.numel] = s.clip
                decay[s.offset:s.offset + s.numel] = 1.0 if s.decay else 0.0
            self._clip_vec, self._decay_vec = clip, decay
        return self._clip_vec, self._decay_vec

    def _step_torch(self, lr: float) -> None:
        sp, p, g = self.spec, self.flat.data, self.flat.grad
        clip, decay = self._vectors()
        t = self.step_count
        with torch.no_grad():
            g = g * self.grad_scale
            if sp.kind == "adam":
                b1, b2 = sp.beta_1, sp.beta_2
                self.m.mul_(b1).add_(g, alpha=1 - b1)
                self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
                mhat = self.m / (1 - b1**t)
                vhat = self.v / (1 - b2**t)
                upd = mhat / (vhat.sqrt() + sp.eps_effective(t))
                if sp.weight_decay:
                    upd = upd + sp.weight_decay * decay * p
                p.sub_(lr * upd)
            else:
                if sp.weight_decay:
                    g = g + sp.weight_decay * decay * p
                self.m.mul_(sp.momentum).add_(g)
                d = g + sp.momentum * self.m if sp.nesterov else self.m
                p.sub_(lr * d)
            clipped = torch.maximum(torch.minimum(p, clip), -clip)
            p.copy_(torch.where(clip > 0, clipped, p))

    # -- public -------------------------------------------------------------- #

    def step(self) -> float:
        self.step_count += 1
        lr = self.spec.lr_at(self.step_count - 1, self.total_steps)
        from zookeeper_amd import ops

        if self.flat.data.is_cuda and ops.available():
            ops.fused_optimizer_step(self, lr)
        else:
            self._step_torch(lr)
            reg = getattr(self.flat, "images", None)
            if reg is not None:
                reg.invalidate()  # parameters changed without their weight images
        return lr

    def state_dict(self) -> Dict[str, Any]:
        out = {"step_count": self.step_count, "m": self.m}
        if self.v is not None:
            out["v"] = self.v
        return out

    def load_state_dict(self, state: Dict[str, Any]) -> None:
        self.step_count = int(state["step_count"])
        self.m.copy_(state["m"])
        if self.v is not None:
            self.v.copy_(state["v"])
