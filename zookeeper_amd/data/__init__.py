"""Datasets, preprocessing and the device input pipeline.

Concrete synthetic datasets are provided as ready-to-use ``@component``s:
``SyntheticImageNet`` (224×224×3, 1000 classes, 1,281,167 / 50,000 examples),
``SyntheticCIFAR10`` (32×32×3, 10 classes, 50,000 / 10,000) and
``SyntheticMNIST`` (28×28×1, 10 classes, 60,000 / 10,000).
"""

from typing import Optional, Tuple

from zookeeper_amd.core import Field, component
from zookeeper_amd.data.dataset import (
    ArraySource,
    ConcatSource,
    Dataset,
    HFDataset,
    ImageFolderDataset,
    MultiDataset,
    NumpyDataset,
    Source,
    SplitDataset,
    SyntheticDataset,
    SyntheticSource,
    base_splits,
)
from zookeeper_amd.data.loader import DeviceLoader, IndexSampler, make_device_pool_batches
from zookeeper_amd.data.preprocessing import (
    ImageNetPreprocessing,
    PadCropAndFlip,
    Preprocessing,
    nhwc_to_model,
)


@component
class SyntheticImageNet(SyntheticDataset):
    image_shape: Tuple[int, int, int] = Field((224, 224, 3))
    num_classes: int = Field(1000)
    num_train_examples: int = Field(1281167)
    num_validation_examples: int = Field(50000)


@component
class SyntheticCIFAR10(SyntheticDataset):
    image_shape: Tuple[int, int, int] = Field((32, 32, 3))
    num_classes: int = Field(10)
    num_train_examples: int = Field(50000)
    num_validation_examples: int = Field(10000)


@component
class SyntheticMNIST(SyntheticDataset):
    image_shape: Tuple[int, int, int] = Field((28, 28, 1))
    num_classes: int = Field(10)
    num_train_examples: int = Field(60000)
    num_validation_examples: int = Field(10000)
    test_split: Optional[str] = Field(None)


__all__ = [
    "ArraySource",
    "base_splits",
    "ConcatSource",
    "Dataset",
    "DeviceLoader",
    "HFDataset",
    "ImageFolderDataset",
    "ImageNetPreprocessing",
    "IndexSampler",
    "make_device_pool_batches",
    "MultiDataset",
    "nhwc_to_model",
    "NumpyDataset",
    "PadCropAndFlip",
    "Preprocessing",
    "Source",
    "SplitDataset",
    "SyntheticCIFAR10",
    "SyntheticDataset",
    "SyntheticImageNet",
    "SyntheticMNIST",
    "SyntheticSource",
]
