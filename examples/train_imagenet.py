"""ImageNet-shape training of the model zoo (synthetic data by default).

    python examples/train_imagenet.py TrainImageNet model=BinaryResNetE18 batch_size=256
    python examples/train_imagenet.py TrainImageNet --nproc 8 model=QuickNetLarge
    python examples/train_imagenet.py TrainImageNet --grid learning_rate=[1e-3,2e-3] \
        --grid optimizer.weight_decay=[0.0,1e-5] --gpus-per-run 2
"""

from typing import Tuple

import torch.nn as nn

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from zookeeper_amd import ComponentField, Field, cli, task
from zookeeper_amd.data import ImageNetPreprocessing, SyntheticImageNet
from zookeeper_amd.models import BinaryResNetE18
from zookeeper_amd.train import Adam, TrainingExperiment


@task
class TrainImageNet(TrainingExperiment):
    dataset = ComponentField(SyntheticImageNet)
    input_shape: Tuple[int, int, int] = Field((224, 224, 3))
    preprocessing = ComponentField(ImageNetPreprocessing)
    model: nn.Module = ComponentField(BinaryResNetE18)
    optimizer = ComponentField(Adam)

    epochs = Field(1)
    batch_size = Field(256)
    learning_rate: float = Field(2e-3)


if __name__ == "__main__":
    cli()
