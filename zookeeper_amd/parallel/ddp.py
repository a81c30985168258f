"""Bucketed gradient all-reduce overlapped with backward.

Mechanism:

* gradients already live in one flat fp32 buffer in reverse registration
  order (:class:`~zookeeper_amd.parallel.flat.FlatParams`);
* the buffer is cut into contiguous **buckets** (``bucket_mb``, the first —
  holding the last layers — kept small so communication starts early).
  Default 10 MB, sized for xGMI: each ring all-reduce of 10 MB over 8 GPUs
  is a few tens of microseconds of per-link time, and only the LAST bucket
  (the gradients that complete at the very end of backward) is exposed —
  for BinaryResNet-E18 (44.6 MB of fp32 gradients) 25 MB buckets cut
  [2 | 20 | 24.6 MB], leaving 24.6 MB after backward; 10 MB buckets cut
  [2 | 9 | 9 | 9.5 | 9 | 6.1 MB];
* a ``post_accumulate_grad`` hook on every parameter (and the ``grad_ready``
  callback of the fused kernels that write gradients in place) counts
  arrivals; when a bucket's last gradient lands, its range is all-reduced
  asynchronously.

Stream ordering is explicit and backend-independent (no host
synchronisation anywhere on the GPU path):

* at bucket-ready an event is recorded on the **compute** stream;
* a dedicated **comm** HIP stream waits on that event and issues the
  collective under itself (``torch.distributed`` — backend ``"nccl"`` is
  RCCL — orders its internal stream after the comm stream; gloo's CUDA work
  orders its staging copies the same way);
* :meth:`GradBucketer.finish` makes the comm stream wait on every
  outstanding work, then the compute stream waits on the comm stream once,
  before the optimizer reads the buffer.  The ``1/world`` averaging is folded
  into the optimizer's gradient scale (no extra pass over the gradients).

With ``timing=True`` each bucket's collective is bracketed by timing events
on the comm stream, and an event marks the end of backward on the compute
stream; :meth:`GradBucketer.pop_timings` returns per step the comm span, the
sum of per-bucket times and the **exposed** communication (how long the last
collective ran past the end of backward).

xGMI sizing: on MI355X every GPU has 7 point-to-point links of ≈153 GB/s, a
ring uses one link per hop, so a bucket of S bytes costs ≈ 2·(N-1)/N · S /
153 GB/s per ring (RCCL spreads channels over several links).  BinaryResNet-E18
has ≈45 MB of fp32 gradients → six buckets of ≤10 MB (≈0.1 ms each at N=8),
far below the backward pass they hide under (23 ms at 1024 images per GPU);
what stays exposed is the last bucket, ≈6 MB.
"""

from __future__ import annotations

import contextlib
import os
import queue
import sys
import threading
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from zookeeper_amd.ops import streams as side_streams
from zookeeper_amd.parallel.flat import FlatParams


# buckets smaller than this are folded into the next one (bench JSON: no
# sub-0.1 MB bucket)
MIN_BUCKET_BYTES = 256 * 1024

# ZK_COMM_DEBUG_EVENTS=1: log, per bucket launch and per staged copy, whether
# the side-stream events it depends on report complete (ordering diagnostics)
_DEBUG_EVENTS = os.environ.get("ZK_COMM_DEBUG_EVENTS", "0") == "1"


class GradBucketer:
    def __init__(self, flat: FlatParams, world: int, bucket_mb: float = 10.0,
                 first_bucket_mb: float = 1.0, group=None, grad_dtype: Optional[torch.dtype] = None,
                 timing: bool = False, force: bool = False, high_priority: bool = False,
                 check_order: bool = False, native_comm=None):
        """``force``: stay enabled with one rank (needs an initialised
        process group, e.g. a 1-rank RCCL communicator from
        ``zdist.init(single_group=True)``), so a single-GPU run exercises the
        exact multi-GPU path: comm stream, events, RCCL kernels.
        ``high_priority``: the comm stream is a high-priority HIP stream.
        ``check_order``: every step, compare the launched bucket sequence
        across ranks (a MAX and a MIN all-reduce of its hash; raises on a
        mismatch) -- a debug check that costs a host sync per step.
        ``native_comm``: a :class:`~zookeeper_amd.parallel.rccl.NativeComm`
        that issues the all-reduces onto the comm stream itself (instead of
        ProcessGroupNCCL); the collectives are then graph-capturable
        (:attr:`capturable`)."""
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
        # fold buckets below MIN_BUCKET_BYTES (at most a quarter of the cap)
        # into their successor: a 4 KB classifier-bias bucket (the head
        # weight alone exceeds the first-bucket cap) would otherwise cost a
        # whole collective's latency
        fold_bytes = min(MIN_BUCKET_BYTES, limit)
        merged: List[List[int]] = []
        carry: List[int] = []
        for bi, b in enumerate(buckets):
            b = carry + b
            if (sum(flat.slots[i].numel for i in b) * 4 < fold_bytes
                    and bi != len(buckets) - 1):
                carry = b
                continue
            carry = []
            merged.append(b)
        if carry:
            if merged:
                merged[-1] = merged[-1] + carry
            else:
                merged.append(carry)
        buckets = merged
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
        # id() of each bucket's parameters: the side-stream weight gradients a
        # bucket's collective must wait for
        self._bucket_pids = [[id(flat.slots[i].param) for i in b] for b in buckets]
        self._pending = [len(b) for b in buckets]
        self._works: List = []
        self._launched = [False] * len(buckets)
        self._hooks = []
        self._seen = [False] * len(flat.slots)
        self._suspended = False
        self.enabled = world > 1 or bool(force)
        if self.enabled and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("GradBucketer needs an initialised process group "
                               "(zookeeper_amd.parallel.dist.init(single_group=True) for one rank)")
        self.cuda = flat.grad.is_cuda
        self.comm_stream = (torch.cuda.Stream(flat.grad.device, priority=-1 if high_priority else 0)
                            if (self.enabled and self.cuda) else None)
        self.check_order = bool(check_order) and self.enabled
        self.native = native_comm if (self.enabled and self.cuda) else None
        self._order: List[int] = []  # bucket ids in launch order (this step)
        self.order_checks = 0        # steps whose order was compared across ranks
        self.last_order: List[int] = []
        self.timing = bool(timing) and self.comm_stream is not None
        # debugging hook only: ZK_COMM_HOST_SYNC=1 synchronises the device
        # before each collective and after the last (isolates stream-ordering
        # bugs)
        hs = os.environ.get("ZK_COMM_HOST_SYNC", "0") if self.cuda else "0"
        self._sync_launch = hs in ("1", "launch")
        self._sync_finish = hs in ("1", "finish")
        self._step_events: Optional[Dict] = None
        self._timings: List[Dict] = []
        # gloo with GPU tensors (rehearsals on one GPU): explicit host
        # staging instead of handing device tensors to gloo (its internal
        # staging streams raced with the compute stream on this ROCm build,
        # tools/dp_order_diag.py)
        self._stager = None
        if (self.enabled and self.cuda and self.native is None
                and dist.get_backend(group) != "nccl"):
            self._stager = _HostStager(flat.total, group)
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

    @property
    def capturable(self) -> bool:
        """The collectives can be captured into a HIP graph with the backward
        (native communicator: plain stream work, no work objects)."""
        return self.native is not None

    @contextlib.contextmanager
    def untimed(self):
        """No timing events (they cannot be recorded inside a graph capture)."""
        old = self.timing
        self.timing = False
        try:
            yield
        finally:
            self.timing = old

    @contextlib.contextmanager
    def suspended(self):
        """Ignore readiness signals (HIP-graph capture of forward+backward:
        the collectives are issued eagerly after the replay instead)."""
        old = self._suspended
        self._suspended = True
        try:
            yield
        finally:
            self._suspended = old
            self._seen = [False] * len(self.flat.slots)
            self._pending = [len(b) for b in self.buckets]
            self._clear_claims()

    def _clear_claims(self) -> None:
        for s in self.flat.slots:
            if getattr(s.param, "_zk_direct_claim", False):
                s.param._zk_direct_claim = False

    def _make_hook(self, slot_index: int):
        def hook(_param):
            if _DEBUG_EVENTS:
                print(f"[bucketer {os.getpid()}] ready {self.flat.slots[slot_index].name} "
                      f"(bucket {self.slot_bucket[slot_index]}, seen {self._seen[slot_index]}, "
                      f"{'autograd' if _param is not None else 'direct'})",
                      file=sys.stderr, flush=True)
            if self._suspended or self._seen[slot_index]:
                return
            if _param is not None and getattr(_param, "_zk_direct_claim", False):
                # autograd's post-accumulate call for a gradient a kernel writes
                # straight into the flat buffer: the op returned None for it,
                # yet the hook still runs, possibly before the write is even
                # ordered (a side-stream weight gradient is deferred).  Its
                # writer signals readiness itself (``_zk_grad_ready``).
                return
            self._seen[slot_index] = True
            b = self.slot_bucket[slot_index]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)

        return hook

    def _events(self) -> Dict:
        if self._step_events is None:
            mk = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
            self._step_events = {"start": {}, "end": {}, "bwd_end": mk(), "mk": mk}
        return self._step_events

    def _launch(self, b: int) -> None:
        self._order.append(b)
        lo, hi = self.ranges[b]
        view = self.flat.grad[lo:hi]
        if self.comm_stream is None:  # CPU tensors (gloo): plain async collective
            self._works.append((self._issue(view), view, b))
            self._launched[b] = True
            return
        if self._sync_launch:
            torch.cuda.synchronize(view.device)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(view.device))
        self.comm_stream.wait_event(ready)
        # this bucket's weight gradients still running on the side stream
        # (ops/streams.py); the other buckets' are not waited for
        for ev in side_streams.unwaited_events_for(self._bucket_pids[b]):
            self.comm_stream.wait_event(ev)
        if _DEBUG_EVENTS:
            print(f"[bucketer {os.getpid()}] launch {b}: side events "
                  f"{[(id(e) % 10007, e.query()) for e in side_streams.unwaited_events()]}",
                  file=sys.stderr, flush=True)
        with torch.cuda.stream(self.comm_stream):
            if self.timing:
                ev = self._events()
                ev["start"][b] = ev["mk"]()
                ev["start"][b].record(self.comm_stream)
            if self._stager is not None:
                self._works.append((self._stager.submit(b, lo, hi, view, self.comm_stream,
                                                        list(side_streams.unwaited_events())),
                                    view, b))
            else:
                work, tmp = self._issue(view)
                # RCCL: order the comm stream after this collective right away
                # (a stream wait, the host does not block), so the bucket's
                # end event marks the collective's own completion instead of
                # the end of backward (finish() would otherwise record every
                # end event behind the last bucket's launch)
                work.wait()
                if tmp is not None:
                    view.copy_(tmp, non_blocking=True)
                if self.timing:
                    ev = self._events()
                    ev["end"][b] = ev["mk"]()
                    ev["end"][b].record(self.comm_stream)
                self._works.append(((_DoneWork(), None), view, b))
        self._launched[b] = True

    def _issue(self, view: torch.Tensor):
        if self.native is not None:
            # onto the comm stream (current here): ordered by the stream alone
            buf = view if self.grad_dtype in (None, view.dtype) else view.to(self.grad_dtype)
            self.native.all_reduce_(buf, stream=self.comm_stream)
            return (_DoneWork(), buf if buf is not view else None)
        if self.grad_dtype is not None and self.grad_dtype != view.dtype:
            tmp = view.to(self.grad_dtype)
            return (dist.all_reduce(tmp, group=self.group, async_op=True), tmp)
        return (dist.all_reduce(view, group=self.group, async_op=True), None)

    def watch_replay(self) -> None:
        """After a graph replay that contains the collectives (native
        communicator): the watchdog follows them through an event on the
        current stream."""
        if self.native is not None:
            done = torch.cuda.Event()
            done.record(torch.cuda.current_stream(self.flat.grad.device))
            self.native.watch(done, "captured gradient all-reduce (graph replay)")

    def launch_all(self) -> None:
        """Issue every bucket not yet launched (after a graph replay, or for
        parameters whose hooks never fired)."""
        if not self.enabled:
            return
        for b, done in enumerate(self._launched):
            if not done:
                self._launch(b)

    def finish(self) -> None:
        """Launch any bucket whose hooks did not fire (unused params) and make
        the compute stream wait for every collective."""
        if not self.enabled:
            return
        if self.native is not None:
            self.native.check()  # the watchdog found an earlier step's collectives hung
        if self.timing:
            self._events()["bwd_end"].record(torch.cuda.current_stream(self.flat.grad.device))
        self.launch_all()
        if self.comm_stream is None:
            for (work, tmp), view, _ in self._works:
                work.wait()
                if tmp is not None:
                    view.copy_(tmp)
        else:
            with torch.cuda.stream(self.comm_stream):
                for (work, tmp), view, b in self._works:
                    work.wait()  # comm stream waits on the collective's stream
                    if tmp is not None:
                        view.copy_(tmp, non_blocking=True)
                    if self.timing and b not in self._events()["end"]:
                        ev = self._events()
                        ev["end"][b] = ev["mk"]()
                        ev["end"][b].record(self.comm_stream)
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(self.comm_stream)
            if self.native is not None and not torch.cuda.is_current_stream_capturing():
                # watchdog: this step's collectives must complete within the timeout
                done = torch.cuda.Event()
                done.record(self.comm_stream)
                self.native.watch(done, "bucketed gradient all-reduce")
            if self._sync_finish:
                torch.cuda.synchronize(self.flat.grad.device)
        if self.timing and self._step_events is not None:
            self._timings.append(self._step_events)
            self._step_events = None
        self.last_order = list(self._order)
        self._order.clear()
        if self.check_order and not (self.cuda and torch.cuda.is_current_stream_capturing()):
            self.compare_order(self.last_order)
        self._works.clear()
        self._pending = [len(b) for b in self.buckets]
        self._launched = [False] * len(self.buckets)
        self._seen = [False] * len(self.flat.slots)
        self._clear_claims()

    def compare_order(self, order: List[int]) -> None:
        h = order_hash(order)
        dev = self.flat.grad.device if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([h, -h], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        hmax, hmin = int(t[0].item()), -int(t[1].item())
        self.order_checks += 1
        if hmax != hmin:
            raise RuntimeError(
                f"bucket launch order differs across ranks (this rank: {order}, hash {h}; "
                f"max {hmax}, min {hmin})")

    def pop_timings(self) -> List[Dict[str, float]]:
        """Per recorded step: ``comm_ms`` (first collective start → last end),
        ``bucket_sum_ms`` and ``exposed_ms`` (last end − backward end, ≥0).
        Synchronises on the recorded events; call outside timed regions."""
        out = []
        for ev in self._timings:
            starts, ends = ev["start"], ev["end"]
            if not ends:
                continue
            # every event read below (a bucket's end can complete before the
            # compute stream reaches bwd_end; bench --warmup 5 hit this)
            for e in (*ends.values(), *starts.values(), ev["bwd_end"]):
                e.synchronize()
            first = min(starts.values(), key=lambda e: ev["bwd_end"].elapsed_time(e))
            last = max(ends.values(), key=lambda e: ev["bwd_end"].elapsed_time(e))
            out.append({
                "comm_ms": first.elapsed_time(last),
                "bucket_sum_ms": sum(starts[b].elapsed_time(ends[b]) for b in ends if b in starts),
                "exposed_ms": max(0.0, ev["bwd_end"].elapsed_time(last)),
            })
        self._timings.clear()
        return out

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        for s in self.flat.slots:
            if hasattr(s.param, "_zk_grad_ready"):
                del s.param._zk_grad_ready


def order_hash(order: List[int]) -> int:
    """Position-sensitive hash of a bucket sequence (fits in int64)."""
    h = 1469598103934665603 % (2**61 - 1)
    for i, b in enumerate(order):
        h = (h * 1099511628211 + (b + 1) * 1000003 + i) % (2**61 - 1)
    return h


class _DoneWork:
    """A collective the comm stream is already ordered after."""

    def wait(self):
        return True


class _StagedWork:
    def __init__(self, done: threading.Event, box: list):
        self.done, self.box = done, box

    def wait(self):
        self.done.wait()
        if self.box:
            raise self.box[0]


class _HostStager:
    """gloo all-reduce of GPU gradient ranges through a pinned host mirror.

    The main thread records an event on the comm stream after the bucket's
    readiness waits and queues the range.  A worker thread (one, so every
    rank issues the collectives in the same bucket order) orders its own
    copy stream after that event, copies the range D2H into the mirror with
    a BLOCKING copy, all-reduces the host range over gloo and signals;
    the compute stream never blocks.  :meth:`GradBucketer.finish` then copies
    the result back H2D on the comm stream, which the compute stream waits
    on; next step's D2H of the range is ordered after that H2D (its event is
    recorded on the comm stream later).

    The copy used to be an async D2H on the comm stream followed by an event
    the worker synchronised on.  With the comm stream at high priority the
    worker then all-reduced host data that did not yet hold the whole copy
    in ~1 of 3 two-rank runs (tests/gpu/test_dp_gpu.py, deterministic mode,
    side stream on: a partially stale weight gradient, identical on both
    ranks); with the blocking copy: 0 of 12 (scripts/lease/diag_dp.py)."""

    def __init__(self, total: int, group):
        self.host = torch.empty(total, dtype=torch.float32, pin_memory=True)
        self.group = group
        self.copy_stream = None  # created by the worker on first use
        self.q: "queue.Queue" = queue.Queue()
        self.thread = threading.Thread(target=self._run, daemon=True)
        self.thread.start()

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                return
            lo, hi, view, ready, done, box, deps = item
            try:
                if self.copy_stream is None:
                    self.copy_stream = torch.cuda.Stream(view.device)
                self.copy_stream.wait_event(ready)
                if _DEBUG_EVENTS:
                    print(f"[stager {os.getpid()}] {time.perf_counter():.6f} copy [{lo}:{hi}] ready="
                          f"{ready.query()} side={[(id(e) % 10007, e.query()) for e in deps]}",
                          file=sys.stderr, flush=True)
                with torch.cuda.stream(self.copy_stream):
                    self.host[lo:hi].copy_(view, non_blocking=False)
                dist.all_reduce(self.host[lo:hi], group=self.group)
            except Exception as e:  # surfaced by wait()
                box.append(e)
            done.set()

    def submit(self, b: int, lo: int, hi: int, view: torch.Tensor, stream, deps=()) -> tuple:
        host = self.host[lo:hi]
        ready = torch.cuda.Event()
        ready.record(stream)  # after the bucket's readiness waits
        done, box = threading.Event(), []
        self.q.put((lo, hi, view, ready, done, box, deps))
        return _StagedWork(done, box), host


def broadcast_module(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Broadcast parameters and buffers from ``src`` (initial sync)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src, group=group)


def all_reduce_buffers(module: torch.nn.Module, group=None) -> None:
    """Average the floating-point buffers (BN running statistics) across
    ranks with ONE coalesced all-reduce.  Called before evaluation and before
    every checkpoint so eval and the saved model use the cross-rank mean
    (each rank's statistics otherwise drift apart after the initial
    broadcast)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    bufs = [b for b in module.buffers() if b.is_floating_point()]
    if not bufs:
        return
    with torch.no_grad():
        flat = torch.cat([b.detach().reshape(-1).float() for b in bufs])
        dist.all_reduce(flat, group=group)
        flat.div_(world)
        off = 0
        for b in bufs:
            n = b.numel()
            b.copy_(flat[off:off + n].view_as(b))
            off += n
