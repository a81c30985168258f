"""Parallel image decode for real-data sources (data/dataset.py): an
ImageFolder batch and a HuggingFace ``Image``-feature batch decoded on a
thread pool give exactly the serial result, and the pool is actually used.
The throughput of both paths is printed (CPU-only measurement, not
asserted: shared CI hosts make timing bounds flaky)."""

import os
import time

import numpy as np
import pytest

from zookeeper_amd import component, configure
from zookeeper_amd.data import dataset as ds_mod
from zookeeper_amd.data.dataset import HFDataset, ImageFolderDataset

PIL = pytest.importorskip("PIL.Image")


@component
class Folder(ImageFolderDataset):
    pass


@component
class Hub(HFDataset):
    pass


def _write_folder(root, n_per_class=24, size=96):
    rng = np.random.default_rng(0)
    for split in ("train",):
        for c in ("cat", "dog"):
            d = os.path.join(root, split, c)
            os.makedirs(d)
            for i in range(n_per_class):
                a = rng.integers(0, 256, (size, size + 16, 3), dtype=np.uint8)
                PIL.fromarray(a).save(os.path.join(d, f"{i:03d}.jpg"), quality=90)


def _source(root, threads):
    ds = Folder()
    configure(ds, {"root": str(root), "image_size": (64, 64), "decode_threads": threads,
                   "validation_split": None})
    src, n = ds.train()
    return src, n


def test_imagefolder_parallel_decode_matches_serial(tmp_path, monkeypatch):
    _write_folder(tmp_path)
    src1, n = _source(tmp_path, 1)
    src4, _ = _source(tmp_path, 4)
    idx = np.arange(n)[::-1].copy()
    calls = []
    real = ds_mod.decode_pool

    def spy(threads):
        calls.append(threads)
        return real(threads)

    monkeypatch.setattr(ds_mod, "decode_pool", spy)
    t0 = time.perf_counter()
    b1 = src1.get_batch(idx)
    t1 = time.perf_counter()
    b4 = src4.get_batch(idx)
    t4 = time.perf_counter()
    assert b1["image"].shape == (n, 64, 64, 3) and b1["image"].dtype == np.uint8
    np.testing.assert_array_equal(b1["image"], b4["image"])
    np.testing.assert_array_equal(b1["label"], b4["label"])
    assert calls and set(calls) == {4}  # the 4-thread source used the pool; 1 thread did not
    print(f"ImageFolder decode: 1 thread {n / (t1 - t0):.0f} img/s, "
          f"4 threads {n / (t4 - t1):.0f} img/s")


def test_hf_image_feature_decoded_on_pool(tmp_path):
    hf = pytest.importorskip("datasets")
    rng = np.random.default_rng(1)
    imgs = [PIL.fromarray(rng.integers(0, 256, (32, 32, 3), dtype=np.uint8)) for _ in range(20)]
    d = hf.Dataset.from_dict({"image": imgs, "label": list(range(20))})
    d = d.cast_column("image", hf.Image())
    d = d.cast_column("label", hf.ClassLabel(num_classes=20))
    hf.DatasetDict({"train": d}).save_to_disk(str(tmp_path / "tiny"))

    def make(threads):
        ds = Hub()
        configure(ds, {"name": "tiny", "data_dir": str(tmp_path), "decode_threads": threads,
                       "train_split": "train"})
        return ds.train()[0]

    serial, par = make(1), make(4)
    assert par._encoded and not serial._encoded
    idx = np.array([3, 1, 4, 15, 9, 2, 6])
    a, b = serial.get_batch(idx), par.get_batch(idx)
    np.testing.assert_array_equal(a["image"], b["image"])
    np.testing.assert_array_equal(a["label"], b["label"])
    np.testing.assert_array_equal(b["image"][0], np.asarray(imgs[3]))
