"""Feasibility probe for a 3-term bf16 split GEMM ("bf16x3") on the ConvNeXt MLP shapes.

x = hi(x) + lo(x) with hi = bf16_rne(x), lo = bf16_rne(x - hi); x.w is then
hi.hi + lo.hi + hi.lo (lo.lo dropped, ~2^-16 relative), i.e. a plain bf16 GEMM over
K' = 3K with A' = [hi | lo | hi] and B' = [hi | hi | lo].  Times the existing bf16
implicit-GEMM conv (1x1) at K' = 3K and measures the error against fp64 next to the fp32
MFMA GEMM's.

    python tools/split3_probe.py [--batch 64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from count_pipnet_amd import _lib, build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

# (name, grid, K, N, count in the C2 network)
SHAPES = [("s1.fc1", 56, 96, 384, 3), ("s1.fc2", 56, 384, 96, 3),
          ("s2.fc1", 28, 192, 768, 3), ("s2.fc2", 28, 768, 192, 3),
          ("s3.fc1", 27, 384, 1536, 9), ("s3.fc2", 27, 1536, 384, 9),
          ("s4.fc1", 26, 768, 3072, 3), ("s4.fc2", 26, 3072, 768, 3)]


def split3(x: torch.Tensor, order: str) -> torch.Tensor:
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    parts = [hi, lo, hi] if order == "a" else [hi, hi, lo]
    return torch.cat(parts, dim=-1).contiguous()


def timed(fn, reps):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    t32 = t3 = 0.0
    for name, g, k, n, cnt in SHAPES:
        m = a.batch * g * g
        x = torch.randn(m, k, device=dev)
        w = torch.randn(n, k, device=dev) * k ** -0.5
        b = torch.zeros(n, device=dev)
        xs = split3(x, "a").view(a.batch, g, g, 3 * k)
        ws = K.pack_conv_weight_bf16(split3(w, "b").view(n, 1, 1, 3 * k))
        ms32 = timed(lambda: K.linear(x, w, b, _lib.EPI_BIAS), a.reps)
        ms3 = timed(lambda: K.conv2d_nhwc_bf16(xs, ws, 1, 1, b, 1, 0, _lib.EPI_BIAS, None), a.reps)
        fl = 2.0 * m * n * k
        # accuracy on the first 2048 rows vs fp64
        rows = slice(0, 2048)
        ref = x[rows].double() @ w.double().t()
        y32 = K.linear(x[rows].contiguous(), w, b, _lib.EPI_BIAS).double()
        xh, xl = x[rows].to(torch.bfloat16).float(), None
        xl = (x[rows] - xh).to(torch.bfloat16).float()
        wh = w.to(torch.bfloat16).float()
        wl = (w - wh).to(torch.bfloat16).float()
        y3 = (xh.double() @ wh.double().t() + xl.double() @ wh.double().t() + xh.double() @ wl.double().t())
        scale = ref.abs().max().item()
        e32 = (y32 - ref).abs().max().item() / scale
        e3 = (y3 - ref).abs().max().item() / scale
        t32 += ms32 * cnt
        t3 += ms3 * cnt
        print(f"{name:7s} M={m:6d} N={n:5d} K={k:5d}  f32 {fl / ms32 / 1e9:6.1f} TF ({ms32 * 1e3:6.0f} us)   "
              f"bf16x3 {fl / ms3 / 1e9:6.1f} eff TF ({ms3 * 1e3:6.0f} us, {3 * fl / ms3 / 1e9:6.1f} bf16 TF)   "
              f"max err/max|y|: f32 {e32:.2e} split3(fp64 acc) {e3:.2e}", flush=True)
    print(f"network MLP GEMM time: f32 {t32:.2f} ms  bf16x3 {t3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
