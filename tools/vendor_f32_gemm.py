"""The library's exact-fp32 MFMA GEMMs (with their fused epilogues) against the vendor fp32 GEMM
(torch.matmul -> hipBLASLt / rocBLAS, no epilogue: the vendor gets the easier problem) on the
ConvNeXt-tiny CNBlock Linear shapes of C2 (batch 64, 224^2), interleaved rounds, median.

    python tools/vendor_f32_gemm.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

PEAK = 157.3


def shapes(batch=64):
    out = []
    for d, hw in [(96, 56), (192, 28), (384, 27), (768, 26)]:
        m = batch * hw * hw
        out.append((f"s{d}_fc1", m, 4 * d, d, _lib.EPI_BIAS_GELU))
        out.append((f"s{d}_fc2", m, d, 4 * d, _lib.EPI_RESID))
    return out


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    for name, m, n, k, epi in shapes():
        A = torch.randn(m, k, device=dev, generator=g)
        W = torch.randn(n, k, device=dev, generator=g) * 0.05
        b = torch.randn(n, device=dev, generator=g)
        R = torch.randn(m, n, device=dev, generator=g) if epi == _lib.EPI_RESID else None
        C = torch.empty(m, n, device=dev)
        ours, vend = [], []
        for _ in range(3):
            ours.append(timeit(lambda: K.linear(A, W, b, epi, r=R)))
            vend.append(timeit(lambda: torch.matmul(A, W.t(), out=C)))
        fl = 2.0 * m * n * k
        o, v = sorted(ours)[1], sorted(vend)[1]
        print(json.dumps({"shape": name, "M": m, "N": n, "K": k, "ours_us": round(o, 1), "vendor_us": round(v, 1),
                          "ours_frac": round(fl / o / 1e6 / PEAK, 3), "vendor_frac": round(fl / v / 1e6 / PEAK, 3),
                          "ours_epilogue": "bias+GELU" if epi == _lib.EPI_BIAS_GELU else "bias+residual",
                          "vendor_epilogue": "none"}), flush=True)


if __name__ == "__main__":
    main()
