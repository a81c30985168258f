"""Multi-experiment sweeps: run a grid of @task configurations concurrently
on disjoint GPU sets of one node.

The reference runs exactly one task per CLI invocation
(zookeeper/core/task.py:55-59); this is new (BASELINE.json config 5: "lr×wd
grid, 4 concurrent @task runs across 8 GPUs").

CLI (added to every @task command)::

    python train.py TrainImageNet --grid learning_rate=[1e-3,2e-3] \\
        --grid optimizer.weight_decay=[0.0,5e-5] --gpus-per-run 2 epochs=1

* each ``--grid key=[v1,...]`` is one axis; runs are the cartesian product;
  ordinary ``key=value`` arguments are shared by every run (a list value on
  a normal argument still means a list);
* runs are scheduled ``max_parallel`` at a time (default: GPUs ÷
  ``gpus_per_run``); each run gets ``HIP_VISIBLE_DEVICES`` restricted to its
  own GPUs and, if ``gpus_per_run > 1``, is launched data-parallel with
  ``--nproc gpus_per_run``;
* ``--runs-per-gpu k`` packs k concurrent runs onto every GPU set (small
  models that leave most of a 288 GB MI355X idle): the slots are the GPU
  sets repeated k times, filled set by set round-robin;
* every run gets ``ZK_RUN_ID=<run_name>``, the default ``run_id`` of a
  training experiment, so runs sharing ``output_dir`` checkpoint into their
  own ``<output_dir>/<Task>/<run_name>/``;
* every run writes ``<sweep_dir>/<run_name>/stdout.log`` and (training
  experiments, via ``ZK_RESULT_JSON``) ``result.json``; the sweep writes
  ``<sweep_dir>/sweep.json`` (config, exit code, wall time, images/sec, final
  loss and validation metrics per run); a failing
  run does not stop the others, the sweep exits non-zero if any run failed.

The parent process never touches the GPU (device counting only reads the
environment / sysfs), so no HIP runtime is initialised before children start.
"""

from __future__ import annotations

import itertools
import json
import os
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

from zookeeper_amd.core.utils import parse_value_from_string
from zookeeper_amd.parallel.devices import visible_gpu_count, visible_gpu_ids


def parse_grid(specs: Sequence[str]) -> List[Tuple[str, List[Any]]]:
    """``["lr=[0.1,0.01]", "wd=[0,1e-4]"]`` → ``[("lr", [0.1, 0.01]), ...]``."""
    axes = []
    for spec in specs:
        if "=" not in spec:
            raise ValueError(f"--grid expects key=[v1,v2,...], got {spec!r}")
        key, raw = spec.split("=", 1)
        values = parse_value_from_string(raw)
        if not isinstance(values, (list, tuple)):
            values = [values]
        axes.append((key, list(values)))
    return axes


def expand(axes: Sequence[Tuple[str, List[Any]]]) -> List[Dict[str, Any]]:
    keys = [k for k, _ in axes]
    return [dict(zip(keys, combo)) for combo in itertools.product(*[v for _, v in axes])]


def run_name(overrides: Dict[str, Any]) -> str:
    parts = []
    for k, v in overrides.items():
        parts.append(f"{k.replace('.', '-')}_{v}")
    return "__".join(parts).replace("/", "-") or "run"


def count_gpus() -> int:
    """Visible GPUs without initialising HIP in this process (environment and
    the KFD sysfs topology only, ``parallel/devices.py``)."""
    return visible_gpu_count()


def visible_ids() -> List[str]:
    return visible_gpu_ids()


@dataclass
class Run:
    name: str
    overrides: Dict[str, Any]
    argv: List[str]
    devices: List[str] = field(default_factory=list)
    proc: Optional[subprocess.Popen] = None
    start: float = 0.0
    end: float = 0.0
    code: Optional[int] = None


def _token(k: str, v: Any) -> str:
    return f"{k}={v!r}" if isinstance(v, str) else f"{k}={v}"


def run_sweep(base_argv: Sequence[str], axes, gpus_per_run: int = 1,
              max_parallel: int = 0, sweep_dir: str = "sweeps/latest",
              poll_s: float = 0.5, env: Optional[Dict[str, str]] = None,
              runs_per_gpu: int = 1) -> int:
    """Run the grid.  ``base_argv`` is the full command of one run *without*
    the grid values (e.g. ``[python, train.py, TrainImageNet, epochs=1]``)."""
    combos = expand(axes)
    devices = visible_ids()
    slots: List[List[str]] = []
    if devices:
        per = max(gpus_per_run, 1)
        for i in range(0, len(devices) - per + 1, per):
            slots.append(devices[i:i + per])
        # k runs per GPU set: one pass over the sets per k, so the first
        # len(sets) runs still land on distinct GPUs
        slots = [list(sl) for _ in range(max(runs_per_gpu, 1)) for sl in slots]
    if not slots:  # CPU-only: concurrency without device partitioning
        slots = [[] for _ in range(max(max_parallel, 1))]
    if max_parallel > 0:
        slots = slots[:max_parallel]
    os.makedirs(sweep_dir, exist_ok=True)
    pending = [Run(run_name(c), c, list(base_argv) + [_token(k, v) for k, v in c.items()])
               for c in combos]
    running: List[Run] = []
    done: List[Run] = []
    free = list(range(len(slots)))
    base_env = dict(os.environ if env is None else env)
    base_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    while pending or running:
        while pending and free:
            run = pending.pop(0)
            slot = free.pop(0)
            run.devices = slots[slot]
            e = dict(base_env)
            if run.devices:
                e["HIP_VISIBLE_DEVICES"] = ",".join(run.devices)
            e["ZK_RUN_ID"] = run.name  # default run_id: separate checkpoint dirs
            for var in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_PORT"):
                e.pop(var, None)
            argv = list(run.argv)
            if gpus_per_run > 1:
                argv.append(f"--nproc={gpus_per_run}")
            rdir = os.path.join(sweep_dir, run.name)
            os.makedirs(rdir, exist_ok=True)
            e["ZK_RESULT_JSON"] = os.path.abspath(os.path.join(rdir, "result.json"))
            out = open(os.path.join(rdir, "stdout.log"), "w")
            run.start = time.time()
            run.proc = subprocess.Popen(argv, env=e, stdout=out, stderr=subprocess.STDOUT)
            run.proc._zk_slot = slot  # type: ignore[attr-defined]
            run.proc._zk_out = out  # type: ignore[attr-defined]
            running.append(run)
            print(f"[sweep] start {run.name} on devices {run.devices or 'cpu'}", flush=True)
        for run in list(running):
            rc = run.proc.poll()
            if rc is None:
                continue
            run.code, run.end = rc, time.time()
            run.proc._zk_out.close()  # type: ignore[attr-defined]
            free.append(run.proc._zk_slot)  # type: ignore[attr-defined]
            running.remove(run)
            done.append(run)
            print(f"[sweep] done  {run.name} rc={rc} ({run.end - run.start:.1f}s)", flush=True)
        time.sleep(poll_s)
    summary = []
    for r in done:
        rec = {"name": r.name, "overrides": {k: repr(v) for k, v in r.overrides.items()},
               "devices": r.devices, "exit_code": r.code, "wall_s": round(r.end - r.start, 3)}
        res = _read_result(os.path.join(sweep_dir, r.name, "result.json"))
        for key in ("images_per_sec", "final_loss", "steps", "validation"):
            if key in res:
                rec[key] = res[key]
        summary.append(rec)
    with open(os.path.join(sweep_dir, "sweep.json"), "w") as f:
        json.dump(summary, f, indent=2)
    failed = [r for r in done if r.code != 0]
    return 1 if failed else 0


def _read_result(path: str) -> Dict[str, Any]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _strip_sweep_args(argv: Sequence[str]) -> List[str]:
    out, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in ("--grid", "--gpus-per-run", "--max-parallel", "--runs-per-gpu"):
            skip = True
            continue
        if a.startswith(("--grid=", "--gpus-per-run=", "--max-parallel=", "--runs-per-gpu=")):
            continue
        out.append(a)
    return out


def run_sweep_from_cli(task_name: str, grid: Sequence[str], gpus_per_run: int,
                       max_parallel: int, runs_per_gpu: int = 1) -> int:
    """Entry point used by the @task command when ``--grid`` is given."""
    axes = parse_grid(grid)
    base = [sys.executable] + _strip_sweep_args(sys.argv)
    stamp = time.strftime("%Y%m%d-%H%M%S")
    sweep_dir = os.environ.get("ZK_SWEEP_DIR", os.path.join("sweeps", f"{task_name}-{stamp}"))
    return run_sweep(base, axes, gpus_per_run, max_parallel, sweep_dir,
                     runs_per_gpu=runs_per_gpu)
