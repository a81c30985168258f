"""Weight-gradient side stream: binary-conv weight gradients run
concurrently with the data-gradient chain.

In a backward pass only the data gradients are on the critical path: block
``k``'s BN backward and dgrad feed block ``k-1``, while its weight gradient is
consumed by nobody until the optimizer (or the bucket all-reduce).  With the
side stream on, ``ops.binary_block``'s backward enqueues the split-K wgrad
on a second HIP stream right after ``dy`` is ready, so it overlaps the dgrad
of the same block and the BN backward / dgrad of the next one — filling the
CUs that the small deep-stage grids leave idle and pairing memory-bound BN
passes with MFMA-bound GEMMs.

Ordering is explicit with HIP events:

* the side stream waits for an event recorded on the compute stream once
  ``dy`` is written;
* the gradient's readiness (``grad_ready`` → the data-parallel bucketer's
  RCCL all-reduce) is *deferred*: the next block's backward signals it and
  hands the wgrad's event to the bucketer, whose comm stream waits for it
  before the all-reduce (``unwaited_events``); the compute stream itself
  waits only once, at the end of the backward (``session`` exit), so a slow
  weight gradient never stalls the data-gradient chain (measured: ~0.6 ms
  per E18 step of compute-stream stalls behind the stage-4 weight gradients
  when every block waited).

The float 1x1 / 3x3 / strided convs (ResNet-50) put their weight gradients
on the same stream through :func:`side_wgrad` (``runtime.float_wgrad_side_stream``):
the compute stream joins each one ``SIDE_LAG`` launches later, which releases
its inputs and bounds the backlog.

Only active inside :func:`session` (the trainer opens one per step and
flushes at its end), so direct callers of the ops keep single-stream
semantics.  ``runtime.wgrad_side_stream=False`` disables it.
"""

from __future__ import annotations

import contextlib
import os
import sys
from typing import Callable, Dict, List, Tuple

import torch

from zookeeper_amd.ops._native import grad_ready
from zookeeper_amd.ops.options import OPTS

_active = False
_streams: Dict[int, torch.cuda.Stream] = {}
_pending: List[Tuple[torch.cuda.Event, object]] = []
# side-stream events whose gradients were signalled ready without the
# compute stream waiting for them (flush(wait=False)); joined at session exit
_unwaited: List[torch.cuda.Event] = []
# the same events by parameter (id): a bucket's all-reduce waits only for the
# weight gradients inside its own range
_unwaited_by_param: Dict[int, torch.cuda.Event] = {}
# compute-stream tensors the side stream reads: held until the compute stream
# has waited for the side stream (flush(wait=True)), then released on their
# own stream.  (record_stream instead made the caching allocator treat their
# blocks as busy until the side-stream event completed, as seen by the host,
# which runs a step ahead of the GPU: ~2.5 fresh device allocations per E18
# step, memory growth and multi-second hipMalloc stalls.)
_keep: List[torch.Tensor] = []


def active() -> bool:
    return _active


def side_stream(device: torch.device) -> torch.cuda.Stream:
    """The weight-gradient side stream of ``device`` (default priority: a
    higher-priority side stream and a CU-masked one both measured slower,
    profiles/r4/removed_variants.md)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=idx)
        _streams[idx] = s
    return s


def keep(*tensors: torch.Tensor) -> None:
    """Keep ``tensors`` (allocated on the compute stream, read by queued
    side-stream work) alive until the compute stream joins the side stream."""
    _keep.extend(tensors)


# ZK_COMM_DEBUG_EVENTS=1: log deferrals and flushes (ordering diagnostics)
_DEBUG = os.environ.get("ZK_COMM_DEBUG_EVENTS", "0") == "1"


# side_wgrad: the compute stream joins a float-conv weight gradient this many
# launches later and releases its inputs then (bounds the memory kept alive
# and the side stream's backlog)
SIDE_LAG = 4
_lagged: List[Tuple[torch.cuda.Event, tuple]] = []


def side_wgrad(device: torch.device, launch: Callable[[int], None], param,
               keep_alive: tuple = ()) -> bool:
    """Float-conv weight gradient on the side stream: ``launch(stream)``
    enqueues it (``stream`` = the raw ``hipStream_t``) after everything the
    compute stream has queued so far; ``param``'s readiness is signalled at
    the next :func:`flush`.  ``keep_alive``: compute-stream tensors the launch
    reads, released once the compute stream has joined it (``SIDE_LAG``
    launches later).  Returns False (nothing launched) when the side stream
    is off (outside a :func:`session` or ``runtime.float_wgrad_side_stream``)."""
    if not (_active and OPTS.float_wgrad_side_stream):
        return False
    s = side_stream(device)
    ready = torch.cuda.Event()
    ready.record()
    s.wait_event(ready)
    with torch.cuda.stream(s):
        launch(s.cuda_stream)
        done = torch.cuda.Event()
        done.record(s)
    _lagged.append((done, keep_alive))
    if len(_lagged) > SIDE_LAG:
        ev, _ = _lagged.pop(0)
        torch.cuda.current_stream(device).wait_event(ev)
    flush(wait=False)
    defer_ready(done, param)
    return True


def defer_ready(event: torch.cuda.Event, param) -> None:
    """``param``'s gradient is complete once ``event`` (side stream) fires."""
    if _DEBUG:
        print(f"[streams {os.getpid()}] defer {tuple(param.shape)} event {id(event) % 10007}",
              file=sys.stderr, flush=True)
    _pending.append((event, param))


def unwaited_events() -> List[torch.cuda.Event]:
    """Events of weight gradients already signalled ready that the compute
    stream has not waited for: a consumer on another stream (the bucketer's
    comm stream) must wait for them before reading the gradients."""
    return _unwaited


def unwaited_events_for(param_ids) -> List[torch.cuda.Event]:
    """The unwaited events of the parameters ``param_ids`` (``id(param)``):
    what a consumer of just those gradients must wait for."""
    out = []
    for pid in param_ids:
        ev = _unwaited_by_param.get(pid)
        if ev is not None:
            out.append(ev)
    return out


def flush(wait: bool = True) -> None:
    """Signal the readiness of every deferred weight gradient (bucketed
    all-reduce).  ``wait``: order the compute stream after them (and after
    every earlier unwaited one); otherwise only record their events for
    :func:`unwaited_events`."""
    cur = torch.cuda.current_stream()
    items = list(_pending)
    _pending.clear()
    if _DEBUG:
        print(f"[streams {os.getpid()}] flush wait={wait}: {[id(ev) % 10007 for ev, _ in items]}",
              file=sys.stderr, flush=True)
    if wait:
        for ev in _unwaited:
            cur.wait_event(ev)
        _unwaited.clear()
        _unwaited_by_param.clear()
        for ev, _ in items:
            cur.wait_event(ev)
        # every side-stream reader of these is now ordered before the compute
        # stream's next use of their memory
        _keep.clear()
        _lagged.clear()
    else:
        _unwaited.extend(ev for ev, _ in items)
        for ev, p in items:
            _unwaited_by_param[id(p)] = ev
    for _, p in items:
        grad_ready(p)


@contextlib.contextmanager
def session(device: torch.device):
    """Enable the side stream for one training step's backward; everything
    deferred is flushed (compute stream ordered after it) on exit."""
    global _active
    use = OPTS.wgrad_side_stream and device.type == "cuda"
    _pending.clear()
    _unwaited.clear()
    _unwaited_by_param.clear()
    _keep.clear()
    _lagged.clear()
    _active = use
    try:
        yield
    finally:
        _active = False
        if use:
            flush()
