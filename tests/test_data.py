"""Datasets, split handling, samplers and the host→device loader (CPU)."""

import numpy as np
import pytest
import torch

from zookeeper_amd.core import configure
from zookeeper_amd.data import (ArraySource, ConcatSource, DeviceLoader, IndexSampler,
                                MultiDataset, SyntheticCIFAR10, SyntheticImageNet,
                                SyntheticMNIST, base_splits)
from zookeeper_amd.data.dataset import slice_range


def test_base_splits_and_slices():
    assert base_splits("train+validation") == ["train", "validation"]
    assert base_splits("train") == ["train"]
    assert slice_range("train[:10%]", 200) == ("train", 0, 20)
    assert slice_range("train[50:]", 200) == ("train", 50, 200)
    assert slice_range("test[-10:]", 100) == ("test", 90, 100)


def test_synthetic_dataset_components():
    ds = SyntheticCIFAR10()
    configure(ds, {"num_train_examples": 100, "num_validation_examples": 20})
    src, n = ds.train()
    assert n == 100 and len(src) == 100
    b = src.get_batch(np.array([0, 5, 99]))
    assert b["image"].shape == (3, 32, 32, 3) and b["image"].dtype == np.uint8
    assert b["label"].dtype == np.int64 and b["label"].max() < 10
    # deterministic per index
    b2 = src.get_batch(np.array([5]))
    assert (b2["image"][0] == b["image"][1]).all() and b2["label"][0] == b["label"][1]
    v, nv = ds.validation()
    assert nv == 20
    with pytest.raises(ValueError, match="not configured with a test split"):
        ds.test()
    src, n = ds.load("train[:10]+validation[:5]"), ds.num_examples("train[:10]+validation[:5]")
    assert n == 15 and len(src) == 15


def test_imagenet_defaults():
    ds = SyntheticImageNet()
    configure(ds, {})
    assert ds.num_classes == 1000 and ds.image_shape == (224, 224, 3)
    assert ds.train()[1] == 1281167


def test_multi_dataset_concatenates_and_raises_on_empty():
    a, b = SyntheticMNIST(), SyntheticMNIST()
    configure(a, {"num_train_examples": 30, "seed": 1})
    configure(b, {"num_train_examples": 20, "seed": 2})
    from zookeeper_amd.core import component

    @component
    class Both(MultiDataset):  # like the reference, the base is undecorated
        pass

    m = Both()
    configure(m, {"datasets": {"a": a, "b": b}, "train_split": {"a": "train", "b": "train[:10]"}})
    src, n = m.train()
    assert n == 40 and len(src) == 40
    got = src.get_batch(np.array([29, 30]))
    assert (got["image"][0] == a.train()[0].get_batch(np.array([29]))["image"][0]).all()
    assert (got["image"][1] == b.train()[0].get_batch(np.array([0]))["image"][0]).all()
    with pytest.raises(ValueError, match="not configured with a validation split"):
        m.validation()


def test_sampler_shards_and_resumes():
    s0 = IndexSampler(103, 10, True, seed=3, rank=0, world=2)
    s1 = IndexSampler(103, 10, True, seed=3, rank=1, world=2)
    e0, e1 = s0.epoch_indices(0), s1.epoch_indices(0)
    assert e0.shape == (5, 10)
    assert not set(e0.ravel()) & set(e1.ravel())  # disjoint shards
    it = s0.batches(0)
    seq = [next(it) for _ in range(12)]
    it2 = s0.batches(7)  # resume at step 7
    assert all((next(it2) == seq[i]).all() for i in range(7, 12))


def test_concat_source():
    a = ArraySource(np.arange(6).reshape(3, 2, 1, 1).astype(np.uint8), np.arange(3))
    b = ArraySource(np.arange(10, 14).reshape(2, 2, 1, 1).astype(np.uint8), np.arange(3, 5))
    c = ConcatSource([a, b])
    got = c.get_batch(np.array([4, 0, 3]))
    assert got["label"].tolist() == [4, 0, 3]


def test_device_loader_cpu_stream():
    imgs = np.random.default_rng(0).integers(0, 255, (40, 4, 4, 3), dtype=np.uint8)
    labels = np.arange(40)
    src = ArraySource(imgs, labels)
    loader = DeviceLoader(src, 8, torch.device("cpu"), shuffle=False)
    it = iter(loader)
    batches = [next(it) for _ in range(6)]
    loader.close()
    assert [int(b["label"][0]) for b in batches] == [0, 8, 16, 24, 32, 0]
    assert torch.equal(batches[1]["image"], torch.from_numpy(imgs[8:16]))


def test_device_pool_mode():
    src = ArraySource(np.zeros((16, 2, 2, 1), np.uint8), np.arange(16))
    loader = DeviceLoader(src, 4, torch.device("cpu"), shuffle=False, device_pool=2)
    it = iter(loader)
    a, b, c = next(it), next(it), next(it)
    assert a is c and a is not b


def test_native_gather_rows():
    from zookeeper_amd.ops import _native

    if not _native.available():
        pytest.skip("native library not built")
    src = np.random.default_rng(1).integers(0, 255, (300, 64, 3), dtype=np.uint8)
    idx = np.random.default_rng(2).permutation(300)[:100]
    dst = torch.empty(100, 64, 3, dtype=torch.uint8)
    _native.gather_rows(src, idx, dst)
    assert (dst.numpy() == src[idx]).all()


def test_stream_gather_plan_matches_get_batch():
    """The streaming loader gathers rows natively through ``gather_plan``;
    its batches must be bit-identical to ``get_batch`` of the sampler's
    indices (synthetic, array and sliced sources), over several epochs."""
    from zookeeper_amd.data.dataset import SyntheticSource, _SubsetSource
    from zookeeper_amd.data.loader import IndexSampler

    arr = np.random.default_rng(3).integers(0, 255, (48, 5, 5, 3), dtype=np.uint8)
    for src in (SyntheticSource(40, (6, 6, 3), 10, seed=5, pool=7),
                ArraySource(arr, np.arange(48) % 9),
                _SubsetSource(ArraySource(arr, np.arange(48)), 8, 40)):
        loader = DeviceLoader(src, 8, torch.device("cpu"), shuffle=True, seed=11)
        sampler = IndexSampler(len(src), 8, True, 11)
        it, ref = iter(loader), sampler.batches()
        for _ in range(11):  # wraps past an epoch boundary
            got, idx = next(it), next(ref)
            want = src.get_batch(idx)
            assert torch.equal(got["image"], torch.from_numpy(np.ascontiguousarray(want["image"])))
            assert torch.equal(got["label"], torch.from_numpy(want["label"]))
        loader.close()
