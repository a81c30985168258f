"""Checkpoint / resume.

The reference has no checkpointing; this defines the layout::

    <output_dir>/<TaskName>/<run_id>/
        config.json                 flattened config + str(task) tree
        metrics.jsonl               one JSON object per log step
        checkpoints/step_00001234/
            model.pt                parameters + buffers (state_dict)
            optimizer.pt            optimizer state (flat moments, step count)
            rng_rank<r>.pt          per-rank RNG states (CPU + GPU)
            meta.json               step, epoch, world size, wall time

Writes go to a ``.tmp`` directory that is renamed into place, so a crash
never leaves a half-written checkpoint that :func:`latest` would pick up.
Only rank 0 writes model/optimizer state (replicated under data
parallelism); every rank writes its RNG state.  Loading uses
``torch.load(weights_only=True)`` — nothing in a checkpoint is executed.
"""

from __future__ import annotations

import json
import os
import re
import shutil
import time
from typing import Any, Dict, Optional

import torch

_STEP_DIR = re.compile(r"^step_(\d{8})$")


def step_dir(root: str, step: int) -> str:
    return os.path.join(root, "checkpoints", f"step_{step:08d}")


def latest(root: str) -> Optional[str]:
    d = os.path.join(root, "checkpoints")
    if not os.path.isdir(d):
        return None
    steps = sorted(int(m.group(1)) for m in map(_STEP_DIR.match, os.listdir(d)) if m)
    for s in reversed(steps):
        p = step_dir(root, s)
        if os.path.exists(os.path.join(p, "meta.json")):
            return p
    return None


def _rng_state() -> Dict[str, Any]:
    state = {"cpu": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        state["cuda"] = torch.cuda.get_rng_state()
    return state


def save(root: str, step: int, model: torch.nn.Module, optimizer, rank: int = 0,
         extra: Optional[Dict[str, Any]] = None, keep: int = 3, barrier=None) -> str:
    final = step_dir(root, step)
    tmp = final + ".tmp"
    if rank == 0:
        shutil.rmtree(tmp, ignore_errors=True)
        os.makedirs(tmp, exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()},
                   os.path.join(tmp, "model.pt"))
        if optimizer is not None:
            torch.save({k: (v.detach().cpu() if torch.is_tensor(v) else v)
                        for k, v in optimizer.state_dict().items()},
                       os.path.join(tmp, "optimizer.pt"))
    if barrier is not None:
        barrier()
    target = tmp if rank == 0 else final + ".tmp"
    os.makedirs(target, exist_ok=True)
    torch.save(_rng_state(), os.path.join(target, f"rng_rank{rank}.pt"))
    if barrier is not None:
        barrier()
    if rank == 0:
        meta = {"step": step, "time": time.time(), **(extra or {})}
        with open(os.path.join(tmp, "meta.json"), "w") as f:
            json.dump(meta, f, indent=2)
        if os.path.exists(final):
            shutil.rmtree(final)
        os.replace(tmp, final)
        _prune(root, keep)
    if barrier is not None:
        barrier()
    return final


def _prune(root: str, keep: int) -> None:
    if keep <= 0:
        return
    d = os.path.join(root, "checkpoints")
    steps = sorted(int(m.group(1)) for m in map(_STEP_DIR.match, os.listdir(d)) if m)
    for s in steps[:-keep]:
        shutil.rmtree(step_dir(root, s), ignore_errors=True)


def load(path: str, model: torch.nn.Module, optimizer=None, rank: int = 0) -> Dict[str, Any]:
    state = torch.load(os.path.join(path, "model.pt"), map_location="cpu", weights_only=True)
    with torch.no_grad():
        own = model.state_dict()
        for k, v in state.items():
            own[k].copy_(v)
    from zookeeper_amd.ops.weight_images import invalidate_model

    invalidate_model(model)  # the bf16 weight images no longer match
    if optimizer is not None and os.path.exists(os.path.join(path, "optimizer.pt")):
        ostate = torch.load(os.path.join(path, "optimizer.pt"), map_location="cpu",
                            weights_only=True)
        optimizer.load_state_dict(ostate)
    rng = os.path.join(path, f"rng_rank{rank}.pt")
    if os.path.exists(rng):
        r = torch.load(rng, weights_only=True)
        torch.set_rng_state(r["cpu"])
        if "cuda" in r and torch.cuda.is_available():
            torch.cuda.set_rng_state(r["cuda"])
    with open(os.path.join(path, "meta.json")) as f:
        return json.load(f)


def _jsonable(v: Any) -> Any:
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    return repr(v)


def write_config(root: str, task: Any, config: Dict[str, Any]) -> None:
    """``config.json``: the resolved dotted-key config (``flatten_config``
    of the task) and the ``str(task)`` tree."""
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "config.json"), "w") as f:
        json.dump({"task": type(task).__name__,
                   "config": {k: _jsonable(v) for k, v in config.items()},
                   "tree": str(task)}, f, indent=2)


def read_config(root: str) -> Dict[str, Any]:
    with open(os.path.join(root, "config.json")) as f:
        return json.load(f)
