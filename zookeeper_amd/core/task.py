"""The ``@task`` decorator: a component with an argument-less ``run()`` that is
registered as a CLI sub-command.

Parity: zookeeper/core/task.py:10-61 (``run`` validation, snake-case naming
conflicts, the ``-i/--interactive`` flag and variadic ``key=value`` config).

Additions (never passed to ``configure``):

* ``--nproc N`` launches N local data-parallel ranks of the task (one process
  per GPU, ``torch.distributed`` env contract), see
  :mod:`zookeeper_amd.parallel.launch`;
* ``--grid key=[v1,v2,...]`` (repeatable) with ``--gpus-per-run G`` runs the
  cartesian product of the grids as concurrent runs on disjoint GPU sets, see
  :mod:`zookeeper_amd.sweep`.
"""

from __future__ import annotations

import inspect
from typing import Any, Dict, Tuple

import click

from zookeeper_amd.core.cli import ConfigParam, cli
from zookeeper_amd.core.component import component, configure
from zookeeper_amd.core.utils import convert_to_snake_case


def _check_run(cls: type) -> None:
    run = getattr(cls, "run", None)
    if run is None or not callable(run):
        raise TypeError("Classes decorated with @task must define a `run` method.")
    params = inspect.signature(run).parameters
    if len(params) > 1 or (len(params) == 1 and "self" not in params):
        raise TypeError(
            "A @task class must define a `run` method taking no arguments except "
            f"`self`, which runs the task, but `{cls.__name__}.run` accepts arguments "
            f"{tuple(params)}."
        )


def run_task(cls: type, config: Dict[str, Any], interactive: bool = False) -> Any:
    """Instantiate, configure and run a task class in-process."""
    instance = cls()
    configure(instance, config, interactive=interactive)
    return instance.run()


def task(cls: type) -> type:
    """Turn a class with an argument-less ``run`` into a runnable task."""
    cls = component(cls)
    _check_run(cls)

    snake = convert_to_snake_case(cls.__name__)
    if snake in (convert_to_snake_case(c) for c in cli.commands):
        raise ValueError(
            f"Task naming conflict. Task with name '{cls.__name__}' (or similar) "
            "already registered. Note that the task name is the name of the class that "
            "the @task decorator is applied to."
        )

    @cli.command(cls.__name__, context_settings=dict(ignore_unknown_options=True))
    @click.option(
        "-i", "--interactive", is_flag=True, default=False, help="Interactively configure task."
    )
    @click.option(
        "--nproc",
        type=int,
        default=1,
        show_default=True,
        help="Number of local data-parallel ranks (one process per GPU).",
    )
    @click.option(
        "--grid",
        multiple=True,
        help="Sweep axis `key=[v1,v2,...]` (repeatable); runs the cartesian product.",
    )
    @click.option(
        "--gpus-per-run", type=int, default=1, show_default=True, help="GPUs per sweep run."
    )
    @click.option(
        "--max-parallel",
        type=int,
        default=0,
        help="Concurrent sweep runs (default: all GPUs / gpus-per-run).",
    )
    @click.option(
        "--runs-per-gpu",
        type=int,
        default=1,
        show_default=True,
        help="Concurrent sweep runs sharing each GPU set.",
    )
    @click.argument("config", type=ConfigParam(), nargs=-1)
    def command(
        config: Tuple[Tuple[str, Any], ...],
        interactive: bool,
        nproc: int,
        grid: Tuple[str, ...],
        gpus_per_run: int,
        max_parallel: int,
        runs_per_gpu: int,
    ):
        conf = {k: v for k, v in config}
        if grid:
            from zookeeper_amd.sweep import run_sweep_from_cli

            raise SystemExit(
                run_sweep_from_cli(cls.__name__, grid, gpus_per_run, max_parallel,
                                   runs_per_gpu)
            )
        if nproc > 1:
            from zookeeper_amd.parallel.launch import maybe_relaunch

            code = maybe_relaunch(nproc)
            if code is not None:
                raise SystemExit(code)
        run_task(cls, conf, interactive=interactive)

    return cls
