"""Bucketed gradient all-reduce overlapped with backward.

Mechanism:

* gradients already live in one flat fp32 buffer in reverse registration
  order (:class:`~zookeeper_amd.parallel.flat.FlatParams`);
* the buffer is cut into contiguous **buckets** (``bucket_mb``, the first —
  holding the last layers — kept small so communication starts early);
* a ``post_accumulate_grad`` hook on every parameter counts arrivals; when a
  bucket's last gradient lands, its range is all-reduced asynchronously.
  With the ``nccl`` (= RCCL) backend the collective runs on RCCL's own HIP
  stream, ordered after the producing backward kernels by an event, so it
  overlaps the rest of backward on the compute stream;
* :meth:`finish` waits for the outstanding work before the optimizer reads
  the buffer.  The ``1/world`` averaging is folded into the optimizer's
  gradient scale (no extra pass over the gradients).

xGMI sizing: on MI355X every GPU has 7 point-to-point links of ≈153 GB/s, a
ring uses one link per hop, so a bucket of S bytes costs ≈ 2·(N-1)/N · S /
153 GB/s per ring (RCCL spreads channels over several links).  BinaryResNet-E18
has ≈47 MB of fp32 gradients → 2–3 buckets of 25 MB (≈0.3 ms each at N=8),
far below the backward pass they hide under.
"""

from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from zookeeper_amd.parallel.flat import FlatParams


class GradBucketer:
    def __init__(self, flat: FlatParams, world: int, bucket_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, group=None, grad_dtype: Optional[torch.dtype] = None):
        self.flat, self.world, self.group = flat, world, group
        self.grad_dtype = grad_dtype
        limit0 = int(first_bucket_mb * 2**20 / 4)
        limit = int(bucket_mb * 2**20 / 4)
        buckets: List[List[int]] = []  # slot indices
        cur, cur_elems = [], 0
        for i, s in enumerate(flat.slots):
            cap = limit0 if not buckets else limit
            if cur and cur_elems + s.numel > cap:
                buckets.append(cur)
                cur, cur_elems = [], 0
            cur.append(i)
            cur_elems += s.numel
        if cur:
            buckets.append(cur)
        self.buckets = buckets
        self.ranges = []
        for b in buckets:
            lo = flat.slots[b[0]].offset
            last = flat.slots[b[-1]]
            hi = last.offset + last.numel
            self.ranges.append((lo, hi))
        self.slot_bucket = {}
        for bi, b in enumerate(buckets):
            for i in b:
                self.slot_bucket[i] = bi
        self._pending = [len(b) for b in buckets]
        self._works: List = []
        self._launched = [False] * len(buckets)
        self._hooks = []
        self._seen = [False] * len(flat.slots)
        self.enabled = world > 1
        # gloo on GPU tensors (tests, 1-GPU rehearsals) stages through host
        # copies on its own streams; order them with a host sync instead of
        # relying on its stream events (RCCL orders on the device).
        self._host_sync = (self.enabled and flat.grad.is_cuda
                           and dist.get_backend(group) != "nccl")
        if self.enabled:
            for i, s in enumerate(flat.slots):
                hook = self._make_hook(i)
                self._hooks.append(s.param.register_post_accumulate_grad_hook(hook))
                # Fused kernels that write gradients in place (bypassing
                # autograd accumulation) signal completion through this.
                s.param._zk_grad_ready = lambda h=hook: h(None)

    @property
    def num_buckets(self) -> int:
        return len(self.buckets)

    def _make_hook(self, slot_index: int):
        def hook(_param):
            if self._seen[slot_index]:
                return
            self._seen[slot_index] = True
            b = self.slot_bucket[slot_index]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)

        return hook

    def _launch(self, b: int) -> None:
        lo, hi = self.ranges[b]
        view = self.flat.grad[lo:hi]
        if self._host_sync:
            torch.cuda.current_stream(view.device).synchronize()
        if self.grad_dtype is not None and self.grad_dtype != view.dtype:
            tmp = view.to(self.grad_dtype)
            work = dist.all_reduce(tmp, group=self.group, async_op=True)
            self._works.append((work, view, tmp))
        else:
            self._works.append((dist.all_reduce(view, group=self.group, async_op=True), None, None))
        self._launched[b] = True

    def finish(self) -> None:
        """Launch any bucket whose hooks did not fire (unused params) and wait."""
        if not self.enabled:
            return
        for b, done in enumerate(self._launched):
            if not done:
                self._launch(b)
        for work, view, tmp in self._works:
            work.wait()
            if view is not None:
                view.copy_(tmp)
        if self._host_sync:
            torch.cuda.synchronize(self.flat.grad.device)
        self._works.clear()
        self._pending = [len(b) for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._seen = [False] * len(self.flat.slots)

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        for s in self.flat.slots:
            if hasattr(s.param, "_zk_grad_ready"):
                del s.param._zk_grad_ready


def broadcast_module(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Broadcast parameters and buffers from ``src`` (initial sync)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src, group=group)


def all_reduce_buffers(module: torch.nn.Module, group=None) -> None:
    """Average floating-point buffers (BN running statistics) across ranks."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    with torch.no_grad():
        for b in module.buffers():
            if b.is_floating_point():
                dist.all_reduce(b, group=group)
                b.div_(world)
