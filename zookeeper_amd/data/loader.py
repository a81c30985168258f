"""Host → device input pipeline.

Replaces the reference's ``tf.data`` chain
(``cache → shuffle → repeat → map → batch``, examples/larq_experiment.py:124-139).

Design (MI355X-first):

* a per-epoch seeded permutation, sharded across data-parallel ranks
  (rank r takes every world-th index) — no sample is seen twice per epoch;
* batches are gathered into a ring of **pinned** host slots by the native
  C++ gather pool when available (``zookeeper_amd/csrc/runtime/host_ring.cpp``,
  multi-threaded row gather straight into pinned memory) or by a Python
  thread otherwise;
* each filled slot is copied with ``non_blocking`` H2D on a **side HIP
  stream** into one of a ring of preallocated device batches and published
  with an event; the compute stream waits on the event only when it consumes
  the batch, so the copy of batch *i+1* overlaps compute on batch *i*
  (double/triple buffering), and the steady state allocates no device memory;
* slots are recycled through an event-carrying free list: the consumer never
  blocks on a copy — the producer thread waits for a slot's last copy event
  before it refills that slot;
* ``device_pool`` mode keeps a few batches resident on the GPU and cycles
  them — the benchmark mode for synthetic data (zero host work per step).
"""

from __future__ import annotations

import queue
import threading
from typing import Dict, Iterator, Optional, Tuple

import numpy as np
import torch

from zookeeper_amd.data.dataset import Source


class IndexSampler:
    """Epoch permutations sharded by rank, ``drop_last`` semantics."""

    def __init__(self, n: int, batch_size: int, shuffle: bool, seed: int = 0,
                 rank: int = 0, world: int = 1):
        self.n, self.batch_size, self.shuffle = n, batch_size, shuffle
        self.seed, self.rank, self.world = seed, rank, world
        self.per_rank = n // world
        self.steps_per_epoch = self.per_rank // batch_size
        if self.steps_per_epoch == 0:
            raise ValueError(
                f"Split of {n} examples is too small for batch {batch_size} x {world} ranks."
            )

    def epoch_indices(self, epoch: int) -> np.ndarray:
        if self.shuffle:
            order = np.random.default_rng((self.seed, epoch)).permutation(self.n)
        else:
            order = np.arange(self.n)
        mine = order[self.rank::self.world][: self.steps_per_epoch * self.batch_size]
        return mine.reshape(self.steps_per_epoch, self.batch_size)

    def batches(self, start_step: int = 0) -> Iterator[np.ndarray]:
        """Infinite stream of index batches (``repeat()``), resumable at a step."""
        step = start_step
        while True:
            epoch, within = divmod(step, self.steps_per_epoch)
            idx = self.epoch_indices(epoch)
            for b in range(within, self.steps_per_epoch):
                yield idx[b]
            step = (epoch + 1) * self.steps_per_epoch


def _native_ring():
    try:
        from zookeeper_amd.ops import _native

        return _native.lib() if _native.available() else None
    except Exception:
        return None


class DeviceLoader:
    """Iterator of device batches ``{"image": uint8[B,H,W,C], "label": int64[B]}``.

    Parameters
    ----------
    source: map-style source of the split.
    batch_size: per-rank batch size.
    device: target device (``cuda:N`` or ``cpu``).
    slots: pinned ring depth (≥2 for overlap).
    device_pool: if >0, materialise that many batches on the device once and
        cycle them forever (synthetic benchmarking).
    transform: optional ``f(batch)`` run on the copy stream right after each
        batch's H2D copy (streaming path), e.g.
        :meth:`~zookeeper_amd.data.preprocessing.Preprocessing.device_transform`:
        it may add keys to the batch (reusing the buffers the device slot held
        for its previous batch); the compute stream's wait on the copy event
        then covers them too.
    """

    def __init__(self, source: Source, batch_size: int, device: torch.device,
                 shuffle: bool = True, seed: int = 0, rank: int = 0, world: int = 1,
                 slots: int = 4, device_pool: int = 0, start_step: int = 0,
                 gather_threads: int = 8, transform=None):
        self.source, self.batch_size, self.device = source, batch_size, torch.device(device)
        self.sampler = IndexSampler(len(source), batch_size, shuffle, seed, rank, world)
        self.steps_per_epoch = self.sampler.steps_per_epoch
        self.slots, self.device_pool = max(3, slots), device_pool
        self.gather_threads = gather_threads
        self.transform = transform
        self._start_step = start_step
        self._pool = None
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._free_q = None

    # -- device-resident pool ----------------------------------------------- #

    def _build_pool(self):
        it = self.sampler.batches(self._start_step)
        pool = []
        for _ in range(self.device_pool):
            host = self.source.get_batch(next(it))
            pool.append({k: torch.from_numpy(np.ascontiguousarray(v)).to(self.device)
                         for k, v in host.items()})
        return pool

    # -- streaming path ----------------------------------------------------- #

    def _producer(self, free_q: "queue.Queue", full_q: "queue.Queue", pinned, idx_iter):
        native = _native_ring()
        try:
            while not self._stop.is_set():
                item = free_q.get()
                if item is None:
                    break
                slot, copied = item
                if copied is not None:
                    # the slot's previous H2D copy must have landed before it
                    # is overwritten (waits in this thread, not the consumer)
                    copied.synchronize()
                idx = next(idx_iter)
                plan = self.source.gather_plan(idx) if native is not None else None
                if plan is not None:
                    # native multi-threaded gather of whole rows into pinned memory
                    from zookeeper_amd.ops import _native

                    rows, row_idx, labels = plan
                    _native.gather_rows(rows, row_idx, pinned[slot]["image"],
                                        threads=self.gather_threads)
                    pinned[slot]["label"].numpy()[:] = labels
                else:
                    host = self.source.get_batch(idx)
                    for k, v in host.items():
                        pinned[slot][k].numpy()[...] = v
                full_q.put(slot)
        except Exception as e:  # surface loader errors in the consumer
            full_q.put(e)

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        if self.device_pool > 0:
            if self._pool is None:
                self._pool = self._build_pool()
            i = 0
            while True:
                yield self._pool[i % len(self._pool)]
                i += 1

        probe = self.source.get_batch(np.arange(min(self.batch_size, len(self.source))))
        use_pin = self.device.type == "cuda"
        pinned = []
        for _ in range(self.slots):
            slot = {}
            for k, v in probe.items():
                t = torch.empty((self.batch_size,) + v.shape[1:],
                                dtype=torch.from_numpy(v[:1]).dtype, pin_memory=use_pin)
                slot[k] = t
            pinned.append(slot)
        free_q: "queue.Queue" = queue.Queue()
        full_q: "queue.Queue" = queue.Queue()
        self._free_q = free_q
        for s in range(self.slots):
            free_q.put((s, None))
        idx_iter = self.sampler.batches(self._start_step)
        self._stop.clear()
        self._thread = threading.Thread(
            target=self._producer, args=(free_q, full_q, pinned, idx_iter), daemon=True
        )
        self._thread.start()

        copy_stream = torch.cuda.Stream(self.device) if use_pin else None
        ahead = max(1, self.slots - 2)  # H2D copies kept in flight ahead of the consumer
        # A ring of preallocated device batches, reused round-robin: no device
        # allocation (and no record_stream, which made the caching allocator
        # hold blocks a step longer) per batch.  Each device slot carries two
        # reusable events: `copied` (its H2D landed, recorded on the copy
        # stream; the compute stream waits for it) and `consumed` (recorded on
        # the compute stream when the consumer asks for the following batch,
        # i.e. after it enqueued every use of this one; the copy stream waits
        # for it before overwriting the slot).  A yielded batch therefore stays
        # valid until the consumer has requested two more.
        ndev = ahead + 2 if copy_stream is not None else 0
        dev_slots = [{k: torch.empty(v.shape, dtype=v.dtype, device=self.device)
                      for k, v in pinned[0].items()} for _ in range(ndev)]
        copied = [torch.cuda.Event() for _ in range(ndev)]
        consumed = [torch.cuda.Event() for _ in range(ndev)]
        used = [False] * ndev
        free_dev = list(range(ndev))
        in_flight: list = []  # (pinned slot, device slot or batch, event)
        try:
            while True:
                while len(in_flight) < ahead:
                    item = full_q.get()
                    if isinstance(item, Exception):
                        raise item
                    slot = item
                    if copy_stream is not None:
                        d = free_dev.pop(0)
                        with torch.cuda.stream(copy_stream):
                            if used[d]:
                                copy_stream.wait_event(consumed[d])
                            for k, v in pinned[slot].items():
                                dev_slots[d][k].copy_(v, non_blocking=True)
                            if self.transform is not None:
                                self.transform(dev_slots[d])
                            copied[d].record(copy_stream)
                        used[d] = True
                        in_flight.append((slot, d, copied[d]))
                    else:
                        in_flight.append((slot, {k: v.clone() for k, v in pinned[slot].items()},
                                          None))
                slot, d, ev = in_flight.pop(0)
                if ev is not None:
                    # the compute stream (not the host) waits for the copy
                    cur = torch.cuda.current_stream(self.device)
                    cur.wait_event(ev)
                    # recycled through the free list with its copy event: the
                    # producer thread waits on it before refilling the slot
                    free_q.put((slot, ev))
                    yield dev_slots[d]
                    # the consumer is back for the next batch: every use of
                    # this one is enqueued on its stream
                    consumed[d].record(torch.cuda.current_stream(self.device))
                    free_dev.append(d)
                else:
                    free_q.put((slot, None))
                    yield d
        finally:
            self.close()

    def close(self) -> None:
        """Stop and join the producer thread (idempotent)."""
        self._stop.set()
        q = getattr(self, "_free_q", None)
        if q is not None:
            q.put(None)
        if self._thread is not None and self._thread.is_alive():
            self._thread.join(timeout=10)
        self._thread = None


def make_device_pool_batches(n_batches: int, batch: int, shape: Tuple[int, int, int],
                             num_classes: int, device: torch.device, seed: int = 0):
    """Random uint8 image batches generated directly on the device (N10)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = []
    for _ in range(n_batches):
        img = torch.randint(0, 256, (batch,) + tuple(shape), device=device, dtype=torch.uint8,
                            generator=g)
        lab = torch.randint(0, num_classes, (batch,), device=device, generator=g)
        out.append({"image": img, "label": lab})
    return out
