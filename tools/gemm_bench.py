"""Time every MFMA GEMM shape of the ConvNeXt-tiny-26 bs=64 forward through the C-ABI.

    python tools/gemm_bench.py [--batch 64] [--iters 20]

Prints per-shape TFLOP/s and the fraction of the 157.3 TF fp32 peak (HIP events).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib, build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402


def shapes(batch):
    out = []
    for d, hw, n in [(96, 56, 3), (192, 28, 3), (384, 27, 9), (768, 26, 3)]:
        m = batch * hw * hw
        out.append((f"s{d}_fc1_gelu", m, 4 * d, d, _lib.EPI_BIAS_GELU, n))
        out.append((f"s{d}_fc2_resid", m, d, 4 * d, _lib.EPI_RESID, n))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = []
    tot_t, tot_f = 0.0, 0.0
    for name, m, n, k, epi, reps in shapes(a.batch):
        A = torch.randn(m, k, device=dev, generator=g)
        W = torch.randn(n, k, device=dev, generator=g) * 0.05
        b = torch.randn(n, device=dev, generator=g)
        s = torch.randn(n, device=dev, generator=g)
        R = torch.randn(m, n, device=dev, generator=g) if epi == _lib.EPI_RESID else None
        out = torch.empty(m, n, device=dev)
        for _ in range(3):
            K.linear(A, W, b, epi, scale=s, r=R, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.iters):
            K.linear(A, W, b, epi, scale=s, r=R, out=out)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / a.iters * 1e-3
        f = 2.0 * m * n * k
        tot_t += t * reps
        tot_f += f * reps
        res.append(dict(name=name, M=m, N=n, K=k, us=t * 1e6, tflops=f / t / 1e12, frac=f / t / 1e12 / 157.3))
        print(f"{name:16s} M={m:7d} N={n:5d} K={k:5d}  {t * 1e6:8.1f} us  {f / t / 1e12:6.1f} TF  "
              f"{100 * f / t / 1e12 / 157.3:5.1f}%", flush=True)
        del A, W, R, out
    print(f"network MLP GEMMs: {tot_t * 1e3:.2f} ms/step  {tot_f / tot_t / 1e12:.1f} TF "
          f"({100 * tot_f / tot_t / 1e12 / 157.3:.1f}% of peak)")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
