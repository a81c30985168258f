"""The training step: forward → fused softmax-CE → backward with bucketed
RCCL all-reduce overlapped → fused optimizer (+ ``weight_clip``) on the flat
buffers.

This is the hot loop that the reference delegates to ``keras.Model.fit``
(HOT LOOP #2).  Nothing in :meth:`Trainer.train_step` touches a
component field or synchronises with the host: losses and hit counts stay on
the device until the metrics logger flushes.
"""

from __future__ import annotations

import dataclasses
import sys
import time
from typing import Callable, Optional, Tuple, Union

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
                 info: Optional[zdist.DistInfo] = None, bucket_mb: float = 10.0,
                 first_bucket_mb: float = 1.0, grad_dtype: Optional[torch.dtype] = None,
                 graph: Union[bool, str] = False, graph_warmup: int = 3,
                 comm_timing: bool = False, metric_fns: Optional[dict] = None,
                 force_dp: bool = False):
        self.info = info or zdist.info()
        if info is None and self.info.world == 1 and self.info.device.type == "cpu" \
                and torch.cuda.is_available():
            # single process without zdist.init(): train on the current GPU
            # rather than silently moving the model to the host
            self.info = dataclasses.replace(
                self.info, device=torch.device("cuda", torch.cuda.current_device()))
        self.device = self.info.device
        self.model = prepare_model(model, self.device)
        self.model.train()
        self.loss_fn: Callable = get_loss(loss)
        # metrics that need the logits (top-k): device hit counts per step,
        # exposed as ``last_metrics`` (graph mode: static graph outputs)
        self.metric_fns = dict(metric_fns or {})
        self.last_metrics: dict = {}
        self.eval_metrics: dict = {}  # eval_step's (kept apart: graph replays reuse last_metrics)
        self.flat = FlatParams(self.model, self.device)
        if self.device.type == "cuda":
            # bf16 GEMM-layout images of the float conv weights, kept current
            # by the fused optimizer (ops/weight_images.py)
            from zookeeper_amd.ops.weight_images import WeightImages

            self.flat.images = WeightImages(self.flat)
            self.flat.images.attach()
        # force_dp: the bucketed all-reduce stays on with one rank (a 1-rank
        # RCCL group), so one GPU runs the exact data-parallel code path
        comm = self.info.comm
        native = None
        if (comm.backend in ("native", "auto") and self.device.type == "cuda"
                and self.info.backend == "nccl" and (self.info.world > 1 or force_dp)):
            native = self._native_comm(comm.backend == "auto")
        self.native_comm = native
        if self.info.world > 1:
            # One broadcast of the flat parameter buffer + the BN buffers
            # (through the native communicator when it is the transport: then
            # the rank holds one RCCL communicator for its collectives)
            for t in [self.flat.data] + list(self.model.buffers()):
                if native is not None and t.is_cuda and t.is_contiguous():
                    native.broadcast_(t, 0)
                else:
                    zdist.broadcast_(t)
            if getattr(self.flat, "images", None) is not None:
                self.flat.images.invalidate()
        self.bucketer = GradBucketer(self.flat, self.info.world, bucket_mb, first_bucket_mb,
                                     grad_dtype=grad_dtype, timing=comm_timing, force=force_dp,
                                     high_priority=comm.high_priority,
                                     check_order=comm.check_bucket_order, native_comm=native)
        self.optimizer = optimizer.create(self.flat, grad_scale=1.0 / self.info.world)
        # HIP-graph replay of zero-grad + forward + loss + backward: one graph
        # launch instead of ~300 kernel launches and the Python / autograd
        # work behind them.  The optimizer (host-side step count and
        # learning-rate schedule) runs eagerly after each replay.  Under data
        # parallelism the collectives stay OUTSIDE the graph: readiness
        # signals are ignored during capture and every bucket is all-reduced
        # on the comm stream right after the replay (no overlap with
        # backward, but no host enqueue cost either — the trade is only worth
        # it when the step is host-bound).
        # ``graph="auto"`` decides on the last warmup step: replay only when
        # the host cannot enqueue a step faster than the GPU runs it (small
        # per-GPU batches); a GPU-bound step keeps the eager path, whose
        # side-stream weight gradients and overlapped all-reduce win.
        auto = isinstance(graph, str) and graph == "auto"
        if isinstance(graph, str) and not auto:
            raise ValueError(f"graph must be a bool or 'auto', got {graph!r}")
        self.graph = (auto or bool(graph)) and self.device.type == "cuda"
        self._graph_auto = auto and self.graph
        self.graph_probe: Optional[Tuple[float, float]] = None  # (host s, GPU s) of the probe
        self.graph_warmup = max(1, graph_warmup)
        self._eager_steps = 0
        self._graph = None
        self._static_in = None
        self._static_out = None

    def _native_comm(self, fallback: bool):
        """The in-tree RCCL communicator for the gradient all-reduce
        (:func:`~zookeeper_amd.parallel.rccl.connect`: load, rendezvous,
        ``ncclCommInitRank`` under a deadline and a canary all-reduce, each
        phase agreed through the store).  With ``fallback``
        (``runtime.comm_backend="auto"``) a failure on any rank makes every
        rank return ``None`` together: ProcessGroupNCCL carries the buckets."""
        from zookeeper_amd.parallel.rccl import connect

        return connect(self.info.rank, self.info.world, fallback=fallback)

    def _forward_backward(self, x: torch.Tensor, y: torch.Tensor):
        self.flat.zero_grad()
        logits = self.model(x)
        loss, correct = self.loss_fn(logits, y)
        if self.metric_fns:
            with torch.no_grad():
                self.last_metrics = {k: f(logits.detach(), y) for k, f in self.metric_fns.items()}
        # binary-conv weight gradients on a side stream, ordered by events
        with streams.session(self.device):
            if loss.is_cuda:
                # a persistent seed gradient: no fill kernel for ones_like(loss)
                one = getattr(self, "_one", None)
                if one is None or one.device != loss.device or one.dtype != loss.dtype:
                    one = self._one = torch.ones((), dtype=loss.dtype, device=loss.device)
                torch.autograd.backward(loss, one)
            else:
                loss.backward()
        return loss.detach(), correct

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """One training step.  In graph mode the returned tensors are the
        graph's static outputs: overwritten by the next step (consume or
        clone them before)."""
        if not self.graph or self._eager_steps < self.graph_warmup:
            probe = self._graph_auto and self._eager_steps == self.graph_warmup - 1
            if probe:
                # empty queue, then one step: the events' span is max(host
                # enqueue, GPU time)
                torch.cuda.synchronize(self.device)
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
                t0 = time.perf_counter()
            self._eager_steps += 1  # eager warmup initialises lazy state (kernel attributes, scratch)
            out = self._forward_backward(x, y)
            self.bucketer.finish()
            self.optimizer.step()
            if probe:
                t_host = time.perf_counter() - t0
                ev[1].record()
                ev[1].synchronize()
                t_gpu = ev[0].elapsed_time(ev[1]) / 1e3
                if self.bucketer.enabled:
                    # every rank must take the same path: replayed graphs issue
                    # the bucket collectives after the replay in index order,
                    # eager steps during backward in readiness order -- mixed,
                    # the ranks' collectives would not match
                    t_host, t_gpu = zdist.all_reduce_max_values([t_host, t_gpu], self.device)
                self.graph_probe = (t_host, t_gpu)
                self.graph = t_host > 0.85 * t_gpu  # host-bound: replay
            return out
        capture_comm = self.bucketer.enabled and self.bucketer.capturable
        images = getattr(self.flat, "images", None)
        if images is not None:
            # the replay reads the bf16 weight images as captured: rebuild them
            # if a parameter changed outside the fused optimizer (checkpoint
            # restore, an in-place edit) -- eagerly, before the replay
            images.ensure_current(torch.cuda.current_stream(self.device).cuda_stream)
        if self._graph is None:
            self._static_in = (x.clone(), y.clone())  # clone keeps x's channels_last strides
            self._graph = torch.cuda.CUDAGraph()
            # thread_local capture: other threads keep their HIP calls -- the
            # RCCL process group's watchdog queries its work events while we
            # capture, which a global-mode capture turns into
            # hipErrorStreamCaptureUnsupported (found on the 1-rank RCCL test)
            torch.cuda.synchronize(self.device)
            if capture_comm:
                # native communicator: the bucketed all-reduce is captured with
                # the backward (same overlap as eager, one graph launch)
                with self.bucketer.untimed(), torch.cuda.graph(
                        self._graph, capture_error_mode="thread_local"):
                    self._static_out = self._forward_backward(*self._static_in)
                    self.bucketer.finish()
            else:
                with self.bucketer.suspended(), torch.cuda.graph(
                        self._graph, capture_error_mode="thread_local"):
                    self._static_out = self._forward_backward(*self._static_in)
            if capture_comm and self.bucketer.check_order:
                # the captured launch order is what every replay issues:
                # compare it across ranks once, outside the capture
                self.bucketer.compare_order(self.bucketer.last_order)
        else:
            self._static_in[0].copy_(x)
            self._static_in[1].copy_(y)
        if capture_comm:
            # a communicator the watchdog aborted must not be replayed: the
            # captured RCCL kernels are bound to its (freed) resources
            self.bucketer.native.check()
        self._graph.replay()
        if capture_comm:
            self.bucketer.watch_replay()  # watchdog over the captured collectives
        else:
            self.bucketer.finish()  # DP: all buckets all-reduced after the replay
        self.optimizer.step()
        return self._static_out

    @torch.no_grad()
    def eval_step(self, x: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        was = self.model.training
        self.model.eval()
        try:
            logits = self.model(x)
            if self.metric_fns:
                self.eval_metrics = {k: f(logits, y) for k, f in self.metric_fns.items()}
            return self.loss_fn(logits, y)
        finally:
            self.model.train(was)
