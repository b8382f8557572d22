"""Digest of the fp32 GEMM outputs on the ConvNeXt MLP shapes (A/B builds must match bitwise).

    python tools/ab_digest.py
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/
from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402
from gemm_bench import shapes  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
h = hashlib.sha256()
for name, m, n, k, epi, _ in shapes(64):
    A = torch.randn(m, k, device=dev, generator=g)
    W = torch.randn(n, k, device=dev, generator=g) * 0.05
    b = torch.randn(n, device=dev, generator=g)
    R = torch.randn(m, n, device=dev, generator=g) if epi == _lib.EPI_RESID else None
    out = K.linear(A, W, b, epi, r=R)
    h.update(out.cpu().numpy().tobytes())
print("digest", h.hexdigest()[:32])
