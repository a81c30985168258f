"""Model zoo: every model is a ``@factory`` whose ``build()`` returns an
``nn.Module`` mapping NHWC (channels_last) images to logits."""

from zookeeper_amd.models.base import ModelFactory, count_parameters, summary
from zookeeper_amd.models.binary_resnet import BinaryResBlock, BinaryResNetE, BinaryResNetE18
from zookeeper_amd.models.binarynet import BinaryNet, BinaryNetModule
from zookeeper_amd.models.quicknet import QuickNet, QuickNetLarge, QuickNetModule, QuickNetXL
from zookeeper_amd.models.resnet import ResNet50, ResNetModule

__all__ = [
    "BinaryNet",
    "BinaryNetModule",
    "BinaryResBlock",
    "BinaryResNetE",
    "BinaryResNetE18",
    "count_parameters",
    "ModelFactory",
    "QuickNet",
    "QuickNetLarge",
    "QuickNetModule",
    "QuickNetXL",
    "ResNet50",
    "ResNetModule",
    "summary",
]
