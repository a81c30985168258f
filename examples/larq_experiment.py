"""BinaryNet on MNIST-shaped data — the reference example
(examples/larq_experiment.py) expressed with zookeeper_amd.

    python examples/larq_experiment.py BinaryNetMnist epochs=0
    python examples/larq_experiment.py BinaryNetMnist epochs=1 steps_per_epoch=20 batch_size=64
    python examples/larq_experiment.py BinaryNetCifar10 epochs=1 steps_per_epoch=20

``BinaryNetCifar10`` is BASELINE.json config 4 (CIFAR-10 BinaryNet ``@task``
running end to end on the CPU at world_size 1).

TFDS MNIST is not available offline, so the dataset is the synthetic
MNIST-shaped component (swap in ``HFDataset`` / ``NumpyDataset`` for real data).
"""

from typing import Sequence, Tuple

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from zookeeper_amd import ComponentField, Field, cli, task
from zookeeper_amd.data import PadCropAndFlip, SyntheticCIFAR10, SyntheticMNIST
from zookeeper_amd.models import BinaryNet
from zookeeper_amd.train import Adam, TrainingExperiment


@task
class BinaryNetMnist(TrainingExperiment):
    dataset = ComponentField(SyntheticMNIST)
    input_shape: Tuple[int, int, int] = Field((28, 28, 1))
    preprocessing = ComponentField(PadCropAndFlip, pad_size=32)
    model = ComponentField(BinaryNet)

    epochs = Field(100)
    batch_size = Field(128)
    learning_rate: float = Field(5e-3)
    optimizer = ComponentField(Adam)

    loss = Field("sparse_categorical_crossentropy")
    metrics: Sequence[str] = Field(lambda: ["accuracy"])


@task
class BinaryNetCifar10(BinaryNetMnist):
    """The same experiment on CIFAR-10-shaped data (32x32x3, 10 classes);
    every other field is inherited from ``BinaryNetMnist``."""

    dataset = ComponentField(SyntheticCIFAR10)
    input_shape: Tuple[int, int, int] = Field((32, 32, 3))
    preprocessing = ComponentField(PadCropAndFlip, pad_size=40)


if __name__ == "__main__":
    cli()
