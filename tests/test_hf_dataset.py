"""``HFDataset`` — the TFDS role of the reference (zookeeper/tf/dataset.py:69-166)
— fully offline: a ``datasets.DatasetDict`` written with ``save_to_disk``
under ``data_dir``.  Covers split loading, slicing and ``+`` merging with
summed example counts (``base_splits``), ``num_classes`` auto-detection from
a ``ClassLabel`` feature, batches through the loader, and ``download=False``
refusing to fetch a dataset that is not on disk."""

import numpy as np
import pytest
import torch

datasets = pytest.importorskip("datasets")

from zookeeper_amd import component, configure  # noqa: E402
from zookeeper_amd.data import HFDataset  # noqa: E402
from zookeeper_amd.data.loader import DeviceLoader  # noqa: E402


@component
class TinyHF(HFDataset):
    pass


def _write(tmp_path, name="tiny_digits", n_train=40, n_test=12, classes=7):
    rng = np.random.default_rng(0)
    feats = datasets.Features({
        "image": datasets.Array3D((6, 5, 3), "uint8"),
        "label": datasets.ClassLabel(num_classes=classes),
    })

    def split(n):
        return datasets.Dataset.from_dict(
            {"image": rng.integers(0, 255, (n, 6, 5, 3), dtype=np.uint8).tolist(),
             "label": (np.arange(n) % classes).tolist()}, features=feats)

    dd = datasets.DatasetDict({"train": split(n_train), "test": split(n_test)})
    dd.save_to_disk(str(tmp_path / name))
    return dd


def _make(tmp_path, **conf):
    ds = TinyHF()
    configure(ds, {"name": "tiny_digits", "data_dir": str(tmp_path), "train_split": "train",
                   **conf})
    return ds


def test_splits_counts_and_classes(tmp_path):
    dd = _write(tmp_path)
    ds = _make(tmp_path, validation_split="test[:50%]", test_split="test[50%:]+train[:4]")
    assert ds.num_classes == 7
    src, n = ds.train()
    assert n == 40 and len(src) == 40
    vsrc, vn = ds.validation()
    assert vn == 6 and len(vsrc) == 6
    tsrc, tn = ds.test()
    assert tn == 6 + 4 and len(tsrc) == 10
    b = src.get_batch(np.array([3, 0, 39]))
    assert b["image"].shape == (3, 6, 5, 3) and b["image"].dtype == np.uint8
    assert b["label"].tolist() == [3, 0, 4]
    np.testing.assert_array_equal(b["image"][1], np.asarray(dd["train"][0]["image"], np.uint8))
    # the sliced validation split starts at test[0]; the merged test split ends in train[:4]
    assert vsrc.get_batch(np.array([0]))["label"].tolist() == [0]
    assert tsrc.get_batch(np.array([9]))["label"].tolist() == [3]


def test_batches_through_the_loader(tmp_path):
    _write(tmp_path)
    ds = _make(tmp_path)
    src, n = ds.train()
    loader = DeviceLoader(src, 8, torch.device("cpu"), shuffle=True, seed=1)
    it = iter(loader)
    batch = next(it)
    loader.close()
    assert batch["image"].shape == (8, 6, 5, 3) and batch["label"].dtype == torch.int64


def test_no_validation_split_raises(tmp_path):
    _write(tmp_path)
    ds = _make(tmp_path)
    with pytest.raises(ValueError, match="not configured with a validation split"):
        ds.validation()


def test_download_false_refuses_to_fetch(tmp_path, capsys):
    ds = TinyHF()
    configure(ds, {"name": "zk-amd/definitely-not-a-local-dataset", "data_dir": str(tmp_path),
                   "train_split": "train"})
    with pytest.raises(Exception):
        ds.train()
    err = capsys.readouterr().err
    assert "WARNING: Field 'download' of component TinyHF is False." in err


def test_mixed_gray_and_rgb_images_decode_to_one_channel_layout(tmp_path):
    """Encoded images decoded on the pool (``Image`` feature): a dataset that
    starts with an RGB image decodes every image -- grayscale ones too -- to
    H x W x 3, whatever the order of the batch (the batch buffer
    used to take its shape from whichever image came first)."""
    from PIL import Image

    rng = np.random.default_rng(1)
    imgs = []
    for k in range(6):
        a = rng.integers(0, 255, (6, 5, 3), dtype=np.uint8)
        im = Image.fromarray(a, "RGB")
        imgs.append(im if k % 2 == 0 else im.convert("L"))
    feats = datasets.Features({"image": datasets.Image(),
                               "label": datasets.ClassLabel(num_classes=2)})
    d = datasets.Dataset.from_dict({"image": imgs, "label": [k % 2 for k in range(6)]},
                                   features=feats)
    datasets.DatasetDict({"train": d}).save_to_disk(str(tmp_path / "mixed"))
    ds = TinyHF()
    configure(ds, {"name": "mixed", "data_dir": str(tmp_path), "train_split": "train",
                   "validation_split": None, "decode_threads": 4})
    src, _ = ds.train()
    for order in ([0, 1, 2, 3], [1, 0, 3, 2], [5, 3, 1]):
        b = src.get_batch(np.array(order))
        assert b["image"].shape == (len(order), 6, 5, 3)
        for j, k in enumerate(order):
            ref = np.asarray(imgs[k].convert("RGB"))
            assert np.array_equal(b["image"][j], ref)
