"""Backward building blocks on the GPU (csrc/backward_ops.hip) against float64 torch.

* wgrad (dW = A^T B over pixel rows): ragged tiles (N not a multiple of 128), short and long
  reductions, strided row views, accumulate, the single-slab direct path; bit-identical
  across repeated runs (fixed slabs, fixed-order reduction);
* colsum: ragged N, accumulate.
"""
import pytest
import torch

from count_pipnet_amd import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,n1,n2", [(86528, 768, 3072), (4096, 192, 96), (37, 12, 20), (1000, 132, 260),
                                     (32, 128, 128), (5, 4, 8)])
def test_wgrad(gpu, m, n1, n2):
    g = torch.Generator().manual_seed(m + n1 + n2)
    a = torch.randn(m, n1, generator=g).to(gpu)
    b = torch.randn(m, n2, generator=g).to(gpu)
    out = K.wgrad(a, b)
    ref = (a.double().t() @ b.double())
    tol = 2e-5 * (m ** 0.5)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=tol)
    again = K.wgrad(a, b)
    assert torch.equal(out, again)


def test_wgrad_strided_and_accumulate(gpu):
    g = torch.Generator().manual_seed(1)
    big = torch.randn(3000, 520, generator=g).to(gpu)
    a, b = big[:, 8:264], big[:, 264:520]          # row stride 520
    c0 = torch.randn(256, 256, generator=g).to(gpu)
    c = c0.clone()
    K.wgrad(a, b, out=c, accumulate=True)
    torch.testing.assert_close(c.double(), c0.double() + a.double().t() @ b.double(), rtol=1e-5, atol=2e-3)


@pytest.mark.parametrize("m,n", [(86528, 768), (17, 300), (1, 4)])
def test_colsum(gpu, m, n):
    g = torch.Generator().manual_seed(m * 7 + n)
    a = torch.randn(m, n, generator=g).to(gpu)
    torch.testing.assert_close(K.colsum(a).double(), a.double().sum(0), rtol=1e-5, atol=2e-5 * m ** 0.5)
    o = torch.ones(n, device=gpu)
    K.colsum(a, out=o, accumulate=True)
    torch.testing.assert_close(o.double(), 1.0 + a.double().sum(0), rtol=1e-5, atol=2e-5 * m ** 0.5)
