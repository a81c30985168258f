"""Model zoo on the pure-PyTorch oracle path (CPU): factories build through
the component system, shapes, parameter counts and a backward pass."""

from typing import Tuple

import pytest
import torch
import torch.nn as nn

from zookeeper_amd import ComponentField, Field, component, configure
from zookeeper_amd.data import Dataset, SyntheticCIFAR10, SyntheticImageNet, SyntheticMNIST
from zookeeper_amd.models import (BinaryNet, BinaryResNetE18, QuickNet, QuickNetLarge, ResNet50,
                                  count_parameters)


def build(model_cls, dataset_cls, shape, conf=None):
    @component
    class Holder:
        dataset: Dataset = ComponentField(dataset_cls)
        input_shape: Tuple[int, int, int] = Field(shape)
        model: nn.Module = ComponentField(model_cls)

    h = Holder()
    configure(h, dict(conf or {}, **{"model.backend": "torch"}) if model_cls is not BinaryNet
              else dict(conf or {}))
    return h.model


def test_binarynet_matches_reference_parameter_count():
    m = build(BinaryNet, SyntheticMNIST, (28, 28, 1))
    # 10.35 M latent weights (+ BN betas / statistics)
    n_kernels = sum(p.numel() for n, p in m.named_parameters() if n.endswith("weight"))
    assert n_kernels == 10_349_696  # sum of the SURVEY §2.4 table
    x = torch.randn(4, 1, 28, 28).contiguous(memory_format=torch.channels_last)
    out = m(x)
    assert out.shape == (4, 10)
    out.sum().backward()


@pytest.mark.parametrize("model_cls,shape,n_out", [
    (BinaryResNetE18, (64, 64, 3), 1000),
    (QuickNet, (64, 64, 3), 1000),
    (ResNet50, (64, 64, 3), 1000),
])
def test_imagenet_models_forward_backward(model_cls, shape, n_out):
    m = build(model_cls, SyntheticImageNet, shape)
    x = torch.randn(2, 3, shape[0], shape[1]).contiguous(memory_format=torch.channels_last)
    out = m(x)
    assert out.shape == (2, n_out)
    out.float().mean().backward()
    assert all(p.grad is not None for p in m.parameters() if p.requires_grad)


def test_e18_parameter_count():
    m = build(BinaryResNetE18, SyntheticImageNet, (224, 224, 3))
    # 16 binary 3x3 convs + stem + 3 shortcut 1x1 convs + fc ≈ 11.7 M
    assert 11_000_000 < count_parameters(m) < 12_500_000


def test_quicknet_large_deeper_than_quicknet():
    a = build(QuickNet, SyntheticImageNet, (64, 64, 3))
    b = build(QuickNetLarge, SyntheticImageNet, (64, 64, 3))
    assert count_parameters(b) > count_parameters(a)


def test_small_input_e18_uses_3x3_stem():
    m = build(BinaryResNetE18, SyntheticCIFAR10, (32, 32, 3))
    assert m.stem[0].kernel_size == (3, 3)
    out = m(torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last))
    assert out.shape == (2, 10)


def test_num_classes_inherited_from_sibling_dataset():
    m = build(BinaryNet, SyntheticCIFAR10, (32, 32, 3))
    assert m.num_classes == 10
