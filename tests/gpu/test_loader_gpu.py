"""Streaming input path on the GPU (N9): native row gather into pinned
slots, H2D on a side HIP stream, event hand-off to the compute stream and
slot recycling through the event-carrying free list.  Streamed batches must
be bit-identical to ``get_batch`` of the sampler's indices, and the copies
must really be issued on the side stream (the consumer never blocks)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.timeout(120)
@pytest.mark.parametrize("kind", ["synthetic", "array"])
def test_streamed_batches_bit_identical(kind):
    from zookeeper_amd.data.dataset import ArraySource, SyntheticSource
    from zookeeper_amd.data.loader import DeviceLoader, IndexSampler

    if kind == "synthetic":
        src = SyntheticSource(600, (64, 64, 3), 100, seed=3, pool=32)
    else:
        arr = np.random.default_rng(0).integers(0, 255, (600, 32, 32, 3), dtype=np.uint8)
        src = ArraySource(arr, np.arange(600) % 17)
    dev = torch.device("cuda", 0)
    loader = DeviceLoader(src, 64, dev, shuffle=True, seed=4, slots=4)
    sampler = IndexSampler(len(src), 64, True, 4)
    it, ref = iter(loader), sampler.batches()
    for _ in range(20):  # > 2 epochs of 9 steps: every slot recycled several times
        got, idx = next(it), next(ref)
        # consume on the compute stream (as the trainer does) before comparing
        img = got["image"].float().sum()
        want = src.get_batch(idx)
        assert got["image"].is_cuda and got["image"].dtype == torch.uint8
        assert torch.equal(got["image"].cpu(), torch.from_numpy(np.ascontiguousarray(want["image"])))
        assert torch.equal(got["label"].cpu(), torch.from_numpy(want["label"]))
        assert torch.isfinite(img)
    loader.close()


@pytest.mark.timeout(120)
def test_stream_overlaps_compute():
    """With a long kernel queued on the compute stream, fetching the next
    batch returns without waiting for it (no host synchronisation)."""
    import time

    from zookeeper_amd.data.dataset import SyntheticSource
    from zookeeper_amd.data.loader import DeviceLoader

    src = SyntheticSource(4096, (224, 224, 3), 1000, seed=1, pool=16)
    loader = DeviceLoader(src, 128, torch.device("cuda", 0), shuffle=True, slots=4)
    it = iter(loader)
    next(it)
    torch.cuda.synchronize()
    a = torch.randn(8192, 8192, device="cuda")
    for _ in range(10):  # ~10+ ms of queued GPU work
        a = a @ a
        a = a / a.norm()
    t0 = time.perf_counter()
    b = next(it)
    t_next = time.perf_counter() - t0
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    t1 = time.perf_counter()
    ev.synchronize()
    t_gpu = time.perf_counter() - t1
    loader.close()
    assert b["image"].shape == (128, 224, 224, 3)
    # the GPU work was still running when next() returned
    assert t_gpu > 0.002, (t_next, t_gpu)


@pytest.mark.timeout(120)
def test_device_slots_reused_under_slow_consumer():
    """The device batches come from a preallocated ring (no allocation per
    batch), and a slot is not overwritten while a slow consumer's queued work
    still reads it: each batch is summed on the compute stream only after a
    long sleep kernel, and every sum must equal its host reference."""
    from zookeeper_amd.data.dataset import ArraySource
    from zookeeper_amd.data.loader import DeviceLoader, IndexSampler

    arr = np.random.default_rng(5).integers(0, 255, (512, 32, 32, 3), dtype=np.uint8)
    src = ArraySource(arr, np.arange(512) % 11)
    dev = torch.device("cuda", 0)
    loader = DeviceLoader(src, 32, dev, shuffle=True, seed=2, slots=4)
    sampler = IndexSampler(len(src), 32, True, 2)
    it, ref = iter(loader), sampler.batches()
    sums, want, ptrs = [], [], set()
    for i in range(24):
        got, idx = next(it), next(ref)
        if i == 4:
            torch.cuda.synchronize()
            allocs0 = torch.cuda.memory_stats(dev).get("num_device_alloc", 0)
        ptrs.add(got["image"].data_ptr())
        torch.cuda._sleep(2_000_000)  # the consumer's "step": the copy stream runs ahead
        sums.append(got["image"].sum(dtype=torch.int64))
        want.append(int(src.get_batch(idx)["image"].astype(np.int64).sum()))
    torch.cuda.synchronize()
    allocs1 = torch.cuda.memory_stats(dev).get("num_device_alloc", 0)
    loader.close()
    assert [int(s) for s in sums] == want
    assert len(ptrs) <= 4  # ahead + 2 device slots, round-robin
    # (the sum results are the only allocations; the caching allocator reuses them)
    assert allocs1 == allocs0


@pytest.mark.timeout(120)
def test_preprocessing_on_the_loader_stream_matches_the_consumer_path():
    """``Preprocessing.device_transform`` (runtime.loader_preprocess): the fused
    normalise kernel runs on the copy stream into a per-slot buffer; under a
    slow consumer every batch's model input must equal ``input()`` of the same
    uint8 batch on the compute stream (no flip: seed-independent), and the
    buffers must be reused (one per device slot)."""
    from zookeeper_amd.core import configure
    from zookeeper_amd.data import ImageNetPreprocessing
    from zookeeper_amd.data.dataset import ArraySource
    from zookeeper_amd.data.loader import DeviceLoader

    arr = np.random.default_rng(6).integers(0, 255, (256, 32, 32, 3), dtype=np.uint8)
    src = ArraySource(arr, np.arange(256) % 7)
    prep = ImageNetPreprocessing()
    configure(prep, {"input_shape": (32, 32, 3)})
    tf = prep.device_transform(training=False)
    assert tf is not None
    loader = DeviceLoader(src, 32, torch.device("cuda", 0), shuffle=True, seed=3, slots=4,
                          transform=tf)
    it = iter(loader)
    ptrs = set()
    for _ in range(20):
        batch = next(it)
        torch.cuda._sleep(2_000_000)
        x, y = prep(batch, training=False)
        want = prep.input({"image": batch["image"].clone()}, training=False)
        assert x.shape == want.shape and x.dtype == torch.bfloat16
        assert torch.equal(x, want)
        assert torch.equal(y, batch["label"])
        ptrs.add(x.data_ptr())
    loader.close()
    assert len(ptrs) <= 4
