"""zk_bn_bwd_reduce_coef (BN-backward reduction whose last-arriving block
computes the coefficients and gamma/beta gradients in the same launch) vs
the two-launch form zk_bn_bwd_reduce + zk_bn_bwd_coef and an fp64 oracle.
Run several times on the same persistent buffers: the last block must leave
the stripes and its arrival counter at zero."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


@pytest.mark.parametrize("P,C", [(4096, 64), (50000, 128), (3000, 512), (7, 32)])
def test_reduce_coef_tail_matches_two_launches(P, C):
    from zookeeper_amd.ops._native import lib, stream_ptr

    L = lib()
    dev = torch.device("cuda")
    st = stream_ptr(dev)
    torch.manual_seed(P + C)
    g = torch.randn(P, C, device=dev).to(torch.bfloat16)
    y = torch.randint(-300, 300, (P, C), device=dev, dtype=torch.int16)
    mean = torch.randn(C, device=dev) * 10
    rstd = torch.rand(C, device=dev) * 0.1 + 0.01
    gamma = torch.rand(C, device=dev) + 0.5
    stripes = 32
    sums_a = torch.zeros(stripes, 2, C, device=dev)
    sums_b = torch.zeros(stripes, 2, C, device=dev)
    counter = torch.zeros(1, dtype=torch.int32, device=dev)
    # fp64 oracle
    gd = g.double()
    yhat = (y.double() - mean.double()) * rstd.double()
    sg, sgy = gd.sum(0), (gd * yhat).sum(0)
    k1 = gamma.double() * rstd.double()
    k3 = k1 * rstd.double() * sgy / P
    ref = torch.stack([k1, k3 * mean.double() - k1 * sg / P, k3])
    dg_a, db_a = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dg_b, db_b = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    for rep in range(3):
        coef_a = torch.empty(3, C, device=dev)
        coef_b = torch.empty(3, C, device=dev)
        assert L.zk_bn_bwd_reduce_coef(g.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                       rstd.data_ptr(), sums_a.data_ptr(), P, C, stripes,
                                       counter.data_ptr(), gamma.data_ptr(), coef_a.data_ptr(),
                                       dg_a.data_ptr(), db_a.data_ptr(), st) == 0
        assert L.zk_bn_bwd_reduce(g.data_ptr(), y.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                  sums_b.data_ptr(), P, C, stripes, st) == 0
        assert L.zk_bn_bwd_coef(sums_b.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                gamma.data_ptr(), float(P), C, stripes, coef_b.data_ptr(),
                                dg_b.data_ptr(), db_b.data_ptr(), st) == 0
        torch.cuda.synchronize()
        torch.testing.assert_close(coef_a, coef_b, rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(coef_a.double(), ref, rtol=1e-3, atol=1e-5)
        assert int(counter.item()) == 0
        assert bool((sums_a == 0).all())
    torch.testing.assert_close(dg_a, dg_b, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db_a, db_b, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(db_a.double(), 3 * sg, rtol=1e-3, atol=1e-2)
