"""Reduction-length limit of the binary forward kernels: they store the exact
+-1 dot product as int16, so K = kh*kw*Cin must stay <= 32767 (an
all-agreeing sum of 32768 terms would wrap to -32768).  Longer reductions
must take the library path and still be exact."""

import pytest
import torch

from zookeeper_amd.nn.layers import QuantDense
from zookeeper_amd.ops import bconv

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


def test_dense_supported_boundary():
    w_ok = torch.zeros(64, 32704, device="cuda")
    x_ok = torch.zeros(4, 32704, device="cuda", dtype=torch.bfloat16)
    assert bconv.dense_supported(x_ok, w_ok)
    w_big = torch.zeros(64, 32768, device="cuda")
    x_big = torch.zeros(4, 32768, device="cuda", dtype=torch.bfloat16)
    assert not bconv.dense_supported(x_big, w_big)
    # a host weight is refused (a host pointer would fault the GPU)
    assert not bconv.dense_supported(x_ok, w_ok.cpu())


def test_conv_supported_boundary():
    x = torch.zeros(1, 2048, 4, 4, device="cuda", dtype=torch.bfloat16)
    w_big = torch.zeros(64, 2048, 4, 4, device="cuda")  # K = 32768
    assert not bconv.conv_supported(x, w_big, (1, 1), "same", 1)
    x2 = torch.zeros(1, 1984, 4, 4, device="cuda", dtype=torch.bfloat16)
    w_ok = torch.zeros(64, 1984, 4, 4, device="cuda")  # K = 31744
    assert bconv.conv_supported(x2, w_ok, (1, 1), "same", 1)


def test_dense_k32768_all_agreeing_is_exact():
    layer = QuantDense(32768, 64, "ste_sign", "ste_sign").cuda()
    with torch.no_grad():
        layer.weight.fill_(0.5)
    x = torch.ones(2, 32768, device="cuda", dtype=torch.bfloat16)
    y = layer(x)
    assert torch.all(y.float() == 32768.0), y.float().unique()
