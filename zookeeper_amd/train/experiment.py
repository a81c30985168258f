"""Experiment base classes.

``Experiment`` is the field bundle of the reference (zookeeper/tf/experiment.py:10-27):
``dataset``, ``preprocessing`` and ``model`` sub-components plus ``epochs``,
``batch_size``, ``loss`` and ``optimizer``.  Like the reference it is an
undecorated base; users subclass it and apply ``@task``.

``TrainingExperiment`` adds a complete ``run()`` — the PyTorch-ROCm
replacement for the example's ``model.compile`` / ``model.fit``
(examples/larq_experiment.py:124-153): device input pipeline, data-parallel
training over RCCL, fused optimizer, metrics, checkpoint/resume and
validation.

``batch_size`` is **per GPU**; the global batch is ``batch_size × world``.
"""

from __future__ import annotations

import os
import time
from typing import Any, Callable, Optional, Sequence, Union

import torch
import torch.nn as nn

from zookeeper_amd.core.component import base_getattr
from zookeeper_amd.core.field import ComponentField, Field
from zookeeper_amd.data.dataset import Dataset
from zookeeper_amd.data.loader import DeviceLoader
from zookeeper_amd.data.preprocessing import Preprocessing
from zookeeper_amd.train.optimizers import OptimizerSpec
from zookeeper_amd.train.runtime import Runtime


class Experiment:
    """Field bundle; subclasses implement ``run``."""

    dataset: Dataset = ComponentField()
    preprocessing: Preprocessing = ComponentField()
    model: nn.Module = ComponentField()

    epochs: int = Field()
    batch_size: int = Field()
    loss: Union[str, Callable] = Field()
    optimizer: OptimizerSpec = ComponentField()


class TrainingExperiment(Experiment):
    """A ready-made classification training task (decorate a subclass with
    ``@task``)."""

    loss: Union[str, Callable] = Field("sparse_categorical_crossentropy")
    # Keras-style metric names (``compile(metrics=...)``,
    # examples/larq_experiment.py:118,142): accuracy, top5, top<k>, ...
    metrics: Sequence[str] = Field(lambda: ["accuracy"])
    learning_rate: float = Field(1e-3)
    seed: int = Field(0)
    # None → examples // global batch.
    steps_per_epoch: Optional[int] = Field(None)
    validation_steps: Optional[int] = Field(None)
    validate: bool = Field(True)
    log_every: int = Field(50)
    # Checkpointing: every N steps (0 = only at the end); output_dir None = off.
    output_dir: Optional[str] = Field(None)
    # A sweep (zookeeper_amd/sweep.py) sets ZK_RUN_ID to each run's name so
    # concurrent runs sharing output_dir keep separate run directories.
    run_id: str = Field(lambda: os.environ.get("ZK_RUN_ID", "run"))
    checkpoint_every: int = Field(0)
    keep_checkpoints: int = Field(3)
    resume: bool = Field(True)
    # Keep this many batches resident on the device and cycle them (synthetic
    # benchmarking); 0 = stream from the host through the pinned ring.
    device_pool: int = Field(0)
    bucket_mb: float = Field(10.0)
    print_summary: bool = Field(True)
    # kernel variants and schedule (side stream, graph replay, deterministic
    # reductions, ...): typed, recorded in config.json, sweepable
    runtime: Runtime = ComponentField(Runtime)

    def run_dir(self) -> Optional[str]:
        if self.output_dir is None:
            return None
        return os.path.join(self.output_dir, type(self).__name__, self.run_id)

    def run(self) -> dict:
        from zookeeper_amd.core.component import flatten_config
        from zookeeper_amd.models.base import summary
        from zookeeper_amd.parallel import dist as zdist
        from zookeeper_amd.parallel.ddp import all_reduce_buffers
        from zookeeper_amd.train import checkpoint as ckpt
        from zookeeper_amd.train.metrics import MetricsLogger, comm_summary, resolve_metrics
        from zookeeper_amd.train.trainer import Trainer

        logit_metrics = {k: f for k, f in resolve_metrics(self.metrics).items() if f is not None}
        rt = self.runtime
        rt.apply()
        info = zdist.init(single_group=rt.force_dp, comm=rt.comm_config())
        torch.manual_seed(self.seed)
        if info.is_main:
            print(self, flush=True)

        train_src, n_train = self.dataset.train(self.preprocessing.decoders)
        global_batch = self.batch_size * info.world
        steps_per_epoch = self.steps_per_epoch or max(n_train // global_batch, 1)
        total_steps = steps_per_epoch * self.epochs

        model = self.model
        if info.is_main and self.print_summary:
            print(summary(model), flush=True)
        dp = info.world > 1 or rt.force_dp
        trainer = Trainer(model, self.loss, base_getattr(self, "optimizer"), info,
                          bucket_mb=self.bucket_mb, metric_fns=logit_metrics,
                          graph=rt.trainer_graph(), force_dp=rt.force_dp,
                          comm_timing=dp and rt.comm_timing and info.device.type == "cuda")
        trainer.optimizer.total_steps = total_steps

        run_dir = self.run_dir()
        start_step = 0
        if run_dir is not None:
            if info.is_main:
                ckpt.write_config(run_dir, self, flatten_config(self))
            last = ckpt.latest(run_dir) if self.resume else None
            if last is not None:
                meta = ckpt.load(last, trainer.model, trainer.optimizer, info.rank)
                start_step = int(meta["step"])
                if info.is_main:
                    print(f"resumed from {last} at step {start_step}", flush=True)

        result = {"steps": start_step, "total_steps": total_steps}
        if total_steps == 0 or start_step >= total_steps:
            return result

        loader = DeviceLoader(train_src, self.batch_size, info.device, shuffle=True,
                              seed=self.seed, rank=info.rank, world=info.world,
                              device_pool=self.device_pool, start_step=start_step,
                              transform=(self.preprocessing.device_transform(training=True)
                                         if rt.loader_preprocess else None))
        metrics = MetricsLogger(info.device,
                                os.path.join(run_dir, "metrics.jsonl") if run_dir else None,
                                info.rank, info.world, metrics=self.metrics)
        it = iter(loader)
        step = start_step
        t_start = time.perf_counter()
        t_other = 0.0  # validation, checkpoints, BN buffer sync: not training throughput
        last_rec = {}
        while step < total_steps:
            batch = next(it)
            x, y = self.preprocessing(batch, training=True)
            loss, correct = trainer.train_step(x, y)
            metrics.update(loss, correct, x.shape[0], trainer.last_metrics)
            step += 1
            epoch_end = step % steps_per_epoch == 0
            if step % self.log_every == 0 or epoch_end or step == total_steps:
                extra = {"epoch": step / steps_per_epoch,
                         "lr": trainer.optimizer.spec.lr_at(step - 1, total_steps)}
                extra.update(comm_summary(trainer.bucketer.pop_timings()))
                last_rec = metrics.flush(step, extra)
            t_o = time.perf_counter()
            save_now = run_dir is not None and (
                (self.checkpoint_every and step % self.checkpoint_every == 0)
                or step == total_steps)
            if save_now or (epoch_end and self.validate):
                # BN running statistics: cross-rank mean before they are
                # evaluated or saved (each rank's drift apart otherwise)
                all_reduce_buffers(trainer.model)
            if save_now:
                ckpt.save(run_dir, step, trainer.model, trainer.optimizer, info.rank,
                          {"epoch": step / steps_per_epoch, "world": info.world},
                          keep=self.keep_checkpoints, barrier=zdist.barrier)
            if epoch_end and self.validate:
                val = self.evaluate(trainer, info)
                if val and info.is_main:
                    print(f"validation step={step} " +
                          " ".join(f"{k}={v:.5g}" for k, v in val.items()), flush=True)
                    result["validation"] = val
            dt_other = time.perf_counter() - t_o
            t_other += dt_other
            metrics.exclude(dt_other)
        loader.close()
        wall = time.perf_counter() - t_start
        train_s = max(wall - t_other, 1e-9)
        result.update(steps=step, train=last_rec, wall_s=wall, train_s=train_s,
                      final_loss=last_rec.get("loss"),
                      # training steps only (validation / checkpoint time excluded)
                      images_per_sec=(step - start_step) * global_batch / train_s,
                      end_to_end_images_per_sec=(step - start_step) * global_batch / max(wall, 1e-9),
                      runtime=rt.as_dict())
        # a sweep (zookeeper_amd/sweep.py) collects every run's result here
        out = os.environ.get("ZK_RESULT_JSON")
        if out and info.is_main:
            import json

            with open(out, "w") as f:
                json.dump(result, f, indent=2, default=repr)
        return result

    def evaluate(self, trainer, info) -> dict:
        try:
            src, n = self.dataset.validation(self.preprocessing.decoders)
        except ValueError:
            return {}
        if n < self.batch_size * info.world:
            return {}
        steps = self.validation_steps or n // (self.batch_size * info.world)
        loader = DeviceLoader(src, self.batch_size, info.device, shuffle=False,
                              rank=info.rank, world=info.world)
        it = iter(loader)
        from zookeeper_amd.train.metrics import resolve_metrics

        keys = list(resolve_metrics(self.metrics))
        tot_loss = torch.zeros((), device=info.device)
        tot_hits = {k: torch.zeros((), device=info.device) for k in keys}
        for _ in range(steps):
            batch = next(it)
            x, y = self.preprocessing(batch, training=False)
            loss, hits = trainer.eval_step(x, y)
            tot_loss += loss.float()
            for k in keys:
                tot_hits[k] += (trainer.eval_metrics[k] if k in trainer.eval_metrics
                                else hits).float()
        loader.close()
        vals = torch.stack([tot_loss] + [tot_hits[k] for k in keys]).double()
        if info.world > 1:
            import torch.distributed as dist

            dist.all_reduce(vals)
        vals = vals.tolist()
        out = {"val_loss": vals[0] / (steps * info.world)}
        for k, v in zip(keys, vals[1:]):
            out[f"val_{k}"] = v / (steps * self.batch_size * info.world)
        return out
