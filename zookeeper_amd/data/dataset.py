"""Dataset components.

Parity with the reference's TF adapters (zookeeper/tf/dataset.py):

* ``Dataset`` ABC: ``train(decoders=None) -> (source, num_examples)`` is
  abstract, ``validation``/``test`` raise ``ValueError`` unless overridden
  (:11-46);
* ``base_splits``: composite split specs (``"train+validation"``) → base
  splits so example counts can be summed (:49-66); TFDS slice syntax
  (``"train[:10%]"``) is understood too;
* ``TFDSDataset`` → :class:`HFDataset` (TFDS/TF are not part of this stack;
  the HuggingFace ``datasets`` library plays the same role: a named dataset
  with splits, cached under ``data_dir``, optional download, automatic
  ``num_classes`` from the ``label`` / ``labels.feature`` / ``objects.label``
  features — :69-166);
* ``MultiTFDSDataset`` → :class:`MultiDataset` (:169-255), with the
  reference's empty-dict bug fixed (an empty validation mapping raises
  instead of returning ``(None, 0)``).

Instead of a ``tf.data.Dataset`` a split is a *map-style source*: ``len()``
plus ``get_batch(indices) -> {"image": uint8[B,H,W,C], "label": int64[B]}``.
Sources are consumed by :class:`zookeeper_amd.data.loader.DeviceLoader`,
which assembles batches in pinned host memory and streams them to the GPU.

New for the MI355X benchmarks: synthetic datasets of ImageNet / CIFAR-10 /
MNIST shape (random uint8 images, uniform labels, deterministic per index) —
there is no network access for real data on the GPU boxes.
"""

from __future__ import annotations

import abc
import os
import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from zookeeper_amd.core import utils
from zookeeper_amd.core.field import Field

Batch = Dict[str, np.ndarray]


# --------------------------------------------------------------------------- #
# Sources
# --------------------------------------------------------------------------- #


class Source(abc.ABC):
    """Map-style collection of examples (features dict per index)."""

    @abc.abstractmethod
    def __len__(self) -> int: ...

    @abc.abstractmethod
    def get_batch(self, indices: np.ndarray) -> Batch: ...

    @property
    def image_shape(self) -> Optional[Tuple[int, ...]]:
        return None

    def gather_plan(self, indices: np.ndarray) -> Optional[Tuple[np.ndarray, np.ndarray, np.ndarray]]:
        """``(rows, row_index, labels)`` when the batch's images are whole
        rows of one C-contiguous array: the loader then gathers them with the
        native multi-threaded row gather straight into a pinned slot
        (``zk_gather_rows``) instead of materialising ``get_batch``.  None
        (default) → ``get_batch``."""
        return None


class ArraySource(Source):
    """Examples held in (possibly memory-mapped) numpy arrays."""

    def __init__(self, images: np.ndarray, labels: np.ndarray):
        if len(images) != len(labels):
            raise ValueError("images and labels must have the same length")
        self.images, self.labels = images, labels

    def __len__(self) -> int:
        return len(self.labels)

    def get_batch(self, indices: np.ndarray) -> Batch:
        idx = np.asarray(indices)
        return {"image": self.images[idx], "label": self.labels[idx].astype(np.int64)}

    def gather_plan(self, indices: np.ndarray):
        if not (isinstance(self.images, np.ndarray) and self.images.flags.c_contiguous):
            return None
        idx = np.asarray(indices, dtype=np.int64)
        return self.images, idx, self.labels[idx].astype(np.int64)

    @property
    def image_shape(self):
        return tuple(self.images.shape[1:])


class ConcatSource(Source):
    """Concatenation of sources in order (``MultiDataset`` splits)."""

    def __init__(self, sources: Sequence[Source]):
        self.sources = list(sources)
        self.offsets = np.cumsum([0] + [len(s) for s in self.sources])

    def __len__(self) -> int:
        return int(self.offsets[-1])

    def get_batch(self, indices: np.ndarray) -> Batch:
        idx = np.asarray(indices)
        which = np.searchsorted(self.offsets, idx, side="right") - 1
        parts: List[Tuple[np.ndarray, Batch]] = []
        for s in np.unique(which):
            sel = np.nonzero(which == s)[0]
            parts.append((sel, self.sources[s].get_batch(idx[sel] - self.offsets[s])))
        out: Batch = {}
        for key in parts[0][1]:
            first = parts[0][1][key]
            buf = np.empty((len(idx),) + first.shape[1:], dtype=first.dtype)
            for sel, b in parts:
                buf[sel] = b[key]
            out[key] = buf
        return out

    @property
    def image_shape(self):
        return self.sources[0].image_shape if self.sources else None


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser (vectorised), used for per-index determinism."""
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    return x


class SyntheticSource(Source):
    """Random uint8 images + uniform labels, a deterministic function of
    ``(seed, index)`` so every rank / epoch sees the same example for an index.

    To keep host cost bounded for ImageNet-sized images, pixel data is drawn
    from a pool of ``pool`` pre-generated images (selected per index); labels
    are independent per index.
    """

    def __init__(self, num_examples: int, image_shape: Tuple[int, int, int],
                 num_classes: int, seed: int = 0, pool: int = 64):
        self.num_examples, self.num_classes, self.seed = num_examples, num_classes, seed
        self._shape = tuple(image_shape)
        rng = np.random.default_rng(seed)
        self.pool = rng.integers(0, 256, size=(min(pool, num_examples),) + self._shape,
                                 dtype=np.uint8)

    def __len__(self) -> int:
        return self.num_examples

    def labels_for(self, idx: np.ndarray) -> np.ndarray:
        with np.errstate(over="ignore"):
            salt = np.uint64(self.seed) * np.uint64(0x9E3779B97F4A7C15)
            h = _mix64(idx.astype(np.uint64) + salt)
        return (h % np.uint64(self.num_classes)).astype(np.int64)

    def get_batch(self, indices: np.ndarray) -> Batch:
        idx = np.asarray(indices, dtype=np.int64)
        if idx.size and (idx.min() < 0 or idx.max() >= self.num_examples):
            raise IndexError("synthetic index out of range")
        return {"image": self.pool[self._pick(idx)], "label": self.labels_for(idx)}

    def _pick(self, idx: np.ndarray) -> np.ndarray:
        h = _mix64(idx.astype(np.uint64) ^ np.uint64(0xA5A5A5A5)) % np.uint64(len(self.pool))
        return h.astype(np.int64)

    def gather_plan(self, indices: np.ndarray):
        idx = np.asarray(indices, dtype=np.int64)
        if idx.size and (idx.min() < 0 or idx.max() >= self.num_examples):
            raise IndexError("synthetic index out of range")
        return self.pool, self._pick(idx), self.labels_for(idx)

    @property
    def image_shape(self):
        return self._shape


# --------------------------------------------------------------------------- #
# Split helpers
# --------------------------------------------------------------------------- #

_SLICE = re.compile(r"^(?P<name>[\w-]+)(\[(?P<lo>-?\d*%?):(?P<hi>-?\d*%?)\])?$")


def base_splits(split: str) -> List[str]:
    """``"train+validation"`` → ``["train", "validation"]``."""
    if "+" in split:
        return [s for part in split.split("+") for s in base_splits(part)]
    return [split.strip()]


def _bound(token: str, n: int, default: int) -> int:
    if token == "":
        return default
    if token.endswith("%"):
        v = int(round(int(token[:-1]) * n / 100))
    else:
        v = int(token)
    if v < 0:
        v += n
    return max(0, min(n, v))


def slice_range(split: str, n: int) -> Tuple[str, int, int]:
    """Parse ``name[lo:hi]`` (absolute or percent bounds) against size ``n``."""
    m = _SLICE.match(split.strip())
    if not m:
        raise ValueError(f"Invalid split specification '{split}'.")
    if m.group("lo") is None:
        return m.group("name"), 0, n
    return m.group("name"), _bound(m.group("lo"), n, 0), _bound(m.group("hi"), n, n)


class _SubsetSource(Source):
    def __init__(self, inner: Source, lo: int, hi: int):
        self.inner, self.lo, self.hi = inner, lo, hi

    def __len__(self) -> int:
        return self.hi - self.lo

    def get_batch(self, indices: np.ndarray) -> Batch:
        return self.inner.get_batch(np.asarray(indices) + self.lo)

    def gather_plan(self, indices: np.ndarray):
        return self.inner.gather_plan(np.asarray(indices, dtype=np.int64) + self.lo)

    @property
    def image_shape(self):
        return self.inner.image_shape


# --------------------------------------------------------------------------- #
# Dataset components
# --------------------------------------------------------------------------- #


class Dataset(abc.ABC):
    """A dataset with a mandatory training split and optional validation /
    test splits.  Subclass, add ``Field``s and decorate with ``@component``."""

    @abc.abstractmethod
    def train(self, decoders=None) -> Tuple[Source, int]:
        """Return ``(source, num_examples)`` of the training split."""
        raise NotImplementedError

    def validation(self, decoders=None) -> Tuple[Source, int]:
        raise ValueError(
            f"Dataset '{self.__class__.__name__}' is not configured with validation data."
        )

    def test(self, decoders=None) -> Tuple[Source, int]:
        raise ValueError(f"Dataset '{self.__class__.__name__}' is not configured with test data.")


class SplitDataset(Dataset):
    """Shared logic for datasets addressed by split strings."""

    train_split: str = Field()
    validation_split: Optional[str] = Field(None)
    test_split: Optional[str] = Field(None)

    def load(self, split: str, decoders=None, shuffle: bool = False) -> Source:
        parts = []
        for base in base_splits(split):
            name, lo, hi = slice_range(base, self.split_size(slice_range(base, 1)[0]))
            src = self.load_base_split(name, decoders)
            parts.append(src if (lo, hi) == (0, len(src)) else _SubsetSource(src, lo, hi))
        return parts[0] if len(parts) == 1 else ConcatSource(parts)

    def num_examples(self, split: str) -> int:
        total = 0
        for base in base_splits(split):
            name = slice_range(base, 1)[0]
            _, lo, hi = slice_range(base, self.split_size(name))
            total += hi - lo
        return total

    def split_size(self, name: str) -> int:
        return len(self.load_base_split(name, None))

    def load_base_split(self, name: str, decoders) -> Source:
        raise NotImplementedError

    def _split(self, split: Optional[str], what: str, decoders, shuffle: bool):
        if split is None:
            raise ValueError(
                f"Dataset {self.__class__.__name__} is not configured with a {what} split."
            )
        return self.load(split, decoders=decoders, shuffle=shuffle), self.num_examples(split)

    def train(self, decoders=None):
        return self._split(self.train_split, "train", decoders, True)

    def validation(self, decoders=None):
        return self._split(self.validation_split, "validation", decoders, False)

    def test(self, decoders=None):
        return self._split(self.test_split, "test", decoders, False)


class SyntheticDataset(SplitDataset):
    """Random images of a fixed shape (no download, no disk).  Splits are
    ``train`` / ``validation`` / ``test`` with the configured sizes."""

    image_shape: Tuple[int, int, int] = Field()
    num_classes: int = Field()
    num_train_examples: int = Field()
    num_validation_examples: int = Field(0)
    num_test_examples: int = Field(0)
    seed: int = Field(0)
    train_split: str = Field("train")
    validation_split: Optional[str] = Field("validation")
    test_split: Optional[str] = Field(None)

    def split_size(self, name: str) -> int:
        sizes = {
            "train": self.num_train_examples,
            "validation": self.num_validation_examples,
            "test": self.num_test_examples,
        }
        if name not in sizes:
            raise ValueError(f"Unknown synthetic split '{name}'.")
        return sizes[name]

    def load_base_split(self, name: str, decoders) -> Source:
        n = self.split_size(name)
        salt = {"train": 0, "validation": 1, "test": 2}[name]
        return SyntheticSource(n, self.image_shape, self.num_classes, seed=self.seed * 3 + salt)


class HFDataset(SplitDataset):
    """A HuggingFace ``datasets`` dataset (the TFDS role of the reference).

    ``name`` is a hub name or a local path; with ``data_dir`` pointing at a
    ``save_to_disk`` directory the data is read fully offline.  ``download``
    mirrors TFDS' flag: when False, a missing dataset raises with a hint.
    """

    name: str = Field()
    data_dir: Optional[str] = Field(None)
    download: bool = Field(False)
    image_key: str = Field("image")
    label_key: str = Field("label")
    # threads decoding a batch's images (encoded bytes decoded on a pool)
    decode_threads: int = Field(8)

    def _load_hf(self, split: Optional[str] = None):
        """The whole dataset (``split=None``) or one split.  ``download=False``
        loads strictly offline (a ``save_to_disk`` directory under
        ``data_dir`` or an already-prepared cache): a missing dataset raises
        instead of being fetched, like TFDS' ``download=False``
        (zookeeper/tf/dataset.py:119-138)."""
        import datasets as hf

        if "_hf" in self.__dict__:
            ds = self.__dict__["_hf"]
            return ds[split] if split is not None else ds
        try:
            if self.data_dir is not None and os.path.isdir(os.path.join(self.data_dir, self.name)):
                ds = hf.load_from_disk(os.path.join(self.data_dir, self.name))
                self.__dict__["_hf"] = ds
                return ds[split] if split is not None else ds
            if self.download:
                return hf.load_dataset(self.name, split=split, cache_dir=self.data_dir)
            old_env = os.environ.get("HF_DATASETS_OFFLINE")
            old_cfg = getattr(hf.config, "HF_DATASETS_OFFLINE", None)
            os.environ["HF_DATASETS_OFFLINE"] = "1"
            hf.config.HF_DATASETS_OFFLINE = True
            try:
                return hf.load_dataset(self.name, split=split, cache_dir=self.data_dir,
                                       download_mode="reuse_cache_if_exists")
            finally:
                if old_env is None:
                    os.environ.pop("HF_DATASETS_OFFLINE", None)
                else:
                    os.environ["HF_DATASETS_OFFLINE"] = old_env
                hf.config.HF_DATASETS_OFFLINE = old_cfg
        except Exception:
            if not self.download:
                utils.warn(
                    f"Field 'download' of component {self.__class__.__name__} is False. "
                    "If the dataset is not available locally, set 'download' to True to "
                    "download and prepare it automatically."
                )
            raise

    @property
    def info(self):
        if "_info" not in self.__dict__:
            self.__dict__["_info"] = self._load_hf()
        return self.__dict__["_info"]

    @property
    def num_classes(self) -> int:
        try:
            ds = self.info
            features = ds[next(iter(ds))].features if hasattr(ds, "keys") else ds.features
            if "label" in features and hasattr(features["label"], "num_classes"):
                return features["label"].num_classes
            if "labels" in features and hasattr(features["labels"], "feature"):
                return features["labels"].feature.num_classes
            if "objects" in features and "label" in features["objects"]:
                obj = features["objects"]
                inner = obj.feature if hasattr(obj, "feature") else obj
                return inner["label"].num_classes
        except Exception:
            pass
        raise ValueError("Unable to determine the number of classes automatically.")

    def split_size(self, name: str) -> int:
        return len(self._load_hf(name))

    def load_base_split(self, name: str, decoders) -> Source:
        return _HFSource(self._load_hf(name), self.image_key, self.label_key, decoders,
                         threads=self.decode_threads)


# ---------------------------------------------------------------------------
# Parallel image decode.  The reference decodes inside tf.data's C++ runtime
# (map(preprocessing) on TF's thread pool, examples/larq_experiment.py:126-139);
# here a batch's images are decoded by a pool of Python threads -- PIL's
# decoders and resizers release the GIL, so the threads run concurrently --
# straight into the batch array (no per-image list + np.stack copy).  The
# loader's producer thread calls get_batch one batch ahead of the step
# (data/loader.py), so decode overlaps the GPU work.
# ---------------------------------------------------------------------------
_POOLS: Dict[int, Any] = {}


def decode_pool(threads: int):
    """A process-wide thread pool of ``threads`` workers (created once)."""
    from concurrent.futures import ThreadPoolExecutor

    pool = _POOLS.get(threads)
    if pool is None:
        pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix="zk-decode")
        _POOLS[threads] = pool
    return pool


def decode_into(out: np.ndarray, items: Sequence[Any], fn, threads: int) -> np.ndarray:
    """``out[k] = fn(items[k])`` for every k, on ``threads`` threads (in
    contiguous chunks, one per thread)."""
    n = len(items)
    shape = out.shape[1:]

    def one(k):
        a = fn(items[k])
        if a.shape != shape:  # no silent broadcast of a 1-channel image into 3
            raise ValueError(f"decoded example {k} of the batch has shape {a.shape}, the batch "
                             f"{shape} (mixed image sizes or channel counts)")
        out[k] = a

    if threads <= 1 or n <= 1:
        for k in range(n):
            one(k)
        return out

    def work(lo, hi):
        for k in range(lo, hi):
            one(k)

    step = -(-n // threads)
    futs = [decode_pool(threads).submit(work, lo, min(n, lo + step)) for lo in range(0, n, step)]
    for f in futs:
        f.result()  # re-raises a decode error
    return out


class _HFSource(Source):
    def __init__(self, ds, image_key: str, label_key: str, decoders=None, threads: int = 8):
        self.ds, self.image_key, self.label_key = ds, image_key, label_key
        self.decoders = decoders or {}
        self.threads = threads
        # read encoded images (bytes) and decode them on the pool instead of
        # letting datasets decode every row in this thread
        self._encoded = False
        if threads > 1 and image_key not in self.decoders:
            try:
                import datasets as hf

                feat = ds.features.get(image_key) if hasattr(ds, "features") else None
                if isinstance(feat, hf.Image) and feat.decode:
                    self.ds = ds.cast_column(image_key, hf.Image(decode=False))
                    self._encoded = True
            except Exception:  # older datasets / non-image column: decode row by row
                pass
        # one channel layout for the whole dataset, fixed by its first image:
        # grayscale stays 1-channel only if the dataset starts grayscale; every
        # other image is converted to it (never per batch, never by order)
        self._mode = "RGB"
        if self._encoded and len(self.ds):
            self._mode = "L" if _encoded_mode(self.ds[0][image_key]) == "L" else "RGB"

    def __len__(self) -> int:
        return len(self.ds)

    def get_batch(self, indices: np.ndarray) -> Batch:
        rows = self.ds[np.asarray(indices).tolist()]
        items = rows[self.image_key]
        mode = self._mode
        decode = ((lambda it: _decode_encoded(it, mode)) if self._encoded
                  else self.decoders.get(self.image_key, _to_uint8_hwc))
        first = decode(items[0])
        out = np.empty((len(items),) + first.shape, dtype=np.uint8)
        out[0] = first
        decode_into(out[1:], items[1:], decode, self.threads)
        return {"image": out, "label": np.asarray(rows[self.label_key], dtype=np.int64)}


def _to_uint8_hwc(im: Any) -> np.ndarray:
    a = np.asarray(im, dtype=np.uint8)
    return a[..., None] if a.ndim == 2 else a


def _open_encoded(item: Any):
    import io

    from PIL import Image

    data = item.get("bytes") if isinstance(item, dict) else None
    return Image.open(io.BytesIO(data) if data is not None else item["path"])


def _encoded_mode(item: Any) -> str:
    with _open_encoded(item) as im:
        return im.mode


def _decode_encoded(item: Any, mode: str = "RGB") -> np.ndarray:
    """A datasets ``Image(decode=False)`` cell ({"bytes", "path"}) -> uint8 HWC
    in ``mode`` ("RGB": H x W x 3, "L": H x W x 1)."""
    with _open_encoded(item) as im:
        return _to_uint8_hwc(im if im.mode == mode else im.convert(mode))


class ImageFolderDataset(SplitDataset):
    """``root/<split>/<class_name>/<image files>`` decoded with PIL and resized
    to ``image_size`` (H, W)."""

    root: str = Field()
    image_size: Tuple[int, int] = Field((224, 224))
    train_split: str = Field("train")
    validation_split: Optional[str] = Field("val")
    # threads decoding a batch (PIL releases the GIL while decoding/resizing)
    decode_threads: int = Field(8)

    def _classes(self) -> List[str]:
        d = os.path.join(self.root, self.train_split.split("[")[0].split("+")[0])
        return sorted(e for e in os.listdir(d) if os.path.isdir(os.path.join(d, e)))

    @property
    def num_classes(self) -> int:
        return len(self._classes())

    def load_base_split(self, name: str, decoders) -> Source:
        classes = {c: i for i, c in enumerate(self._classes())}
        files, labels = [], []
        base = os.path.join(self.root, name)
        for c in sorted(os.listdir(base)):
            for f in sorted(os.listdir(os.path.join(base, c))):
                files.append(os.path.join(base, c, f))
                labels.append(classes[c])
        return _FileSource(files, np.asarray(labels, dtype=np.int64), tuple(self.image_size),
                           threads=self.decode_threads)


class _FileSource(Source):
    def __init__(self, files: List[str], labels: np.ndarray, size: Tuple[int, int],
                 threads: int = 8):
        self.files, self.labels, self.size, self.threads = files, labels, size, threads

    def __len__(self) -> int:
        return len(self.files)

    def _decode(self, path: str) -> np.ndarray:
        from PIL import Image

        with Image.open(path) as im:
            # JPEG: let libjpeg decode at the smallest DCT scale (1/2, 1/4,
            # 1/8) still >= the target size -- most of a large photo's
            # decode cost -- before the resize (measured on this host's CPU,
            # 500x375 -> 224x224: ~2-3x with 8 threads, where full-size
            # decodes did not scale with threads at all)
            im.draft("RGB", (self.size[1], self.size[0]))
            im = im.convert("RGB").resize((self.size[1], self.size[0]))
            return np.asarray(im, dtype=np.uint8)

    def get_batch(self, indices: np.ndarray) -> Batch:
        idx = np.asarray(indices)
        out = np.empty((len(idx), self.size[0], self.size[1], 3), dtype=np.uint8)
        decode_into(out, [self.files[i] for i in idx], self._decode, self.threads)
        return {"image": out, "label": self.labels[idx]}

    @property
    def image_shape(self):
        return (self.size[0], self.size[1], 3)


class NumpyDataset(SplitDataset):
    """Splits stored as ``<root>/<split>.npz`` with ``image`` (uint8 NHWC) and
    ``label`` arrays (loaded memory-mapped via ``np.load(mmap_mode='r')``)."""

    root: str = Field()

    def load_base_split(self, name: str, decoders) -> Source:
        path = os.path.join(self.root, f"{name}.npz")
        with np.load(path) as z:
            images, labels = z["image"], z["label"]
        return ArraySource(images, labels)

    @property
    def num_classes(self) -> int:
        src = self.load_base_split(base_splits(self.train_split)[0].split("[")[0], None)
        return int(np.max(src.labels)) + 1


class MultiDataset(Dataset):
    """Concatenation of several named datasets per split (parity with
    ``MultiTFDSDataset``, zookeeper/tf/dataset.py:169-255).  The split fields
    map dataset *component names* to split strings; ``datasets`` supplies the
    named member datasets."""

    datasets: Dict[str, Any] = Field()
    train_split: Dict[str, str] = Field()
    validation_split: Dict[str, str] = Field(lambda: {})
    test_split: Dict[str, str] = Field(lambda: {})

    def num_examples(self, splits: Dict[str, str]) -> int:
        return sum(self.datasets[n].num_examples(s) for n, s in splits.items())

    def load(self, splits: Dict[str, str], decoders=None, shuffle: bool = False) -> Source:
        return ConcatSource([self.datasets[n].load(s, decoders, shuffle) for n, s in splits.items()])

    def _split(self, splits, what, decoders, shuffle):
        if not splits:
            raise ValueError(
                f"Dataset {self.__class__.__name__} is not configured with a {what} split."
            )
        return self.load(splits, decoders, shuffle), self.num_examples(splits)

    def train(self, decoders=None):
        return self._split(self.train_split, "train", decoders, True)

    def validation(self, decoders=None):
        return self._split(self.validation_split, "validation", decoders, False)

    def test(self, decoders=None):
        return self._split(self.test_split, "test", decoders, False)
