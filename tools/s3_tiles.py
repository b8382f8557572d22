"""Per-shape throughput of the split-bf16 GEMM/conv (pipnet_conv2d_nhwc_s3) on the C2
network's shapes (ConvNeXt-tiny-26, bs=64, 224x224) for every tile it can run on.

    python tools/s3_tiles.py [--batch 64] [--reps 10]
TF/s are fp32-equivalent (2*M*N*K of the fp32 product; the kernel executes 3x that in bf16).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib, build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

# (name, grid in, Cin, Cout, k, stride, epilogue, count in the network)
SHAPES = [("s1.fc1", 56, 96, 384, 1, 1, _lib.EPI_S3_GELU, 3), ("s1.fc2", 56, 384, 96, 1, 1, _lib.EPI_F32_RESID, 3),
          ("ds1", 56, 96, 192, 2, 2, _lib.EPI_F32_BIAS, 1),
          ("s2.fc1", 28, 192, 768, 1, 1, _lib.EPI_S3_GELU, 3), ("s2.fc2", 28, 768, 192, 1, 1, _lib.EPI_F32_RESID, 3),
          ("ds2", 28, 192, 384, 2, 1, _lib.EPI_F32_BIAS, 1),
          ("s3.fc1", 27, 384, 1536, 1, 1, _lib.EPI_S3_GELU, 9), ("s3.fc2", 27, 1536, 384, 1, 1, _lib.EPI_F32_RESID, 9),
          ("ds3", 27, 384, 768, 2, 1, _lib.EPI_F32_BIAS, 1),
          ("s4.fc1", 26, 768, 3072, 1, 1, _lib.EPI_S3_GELU, 3), ("s4.fc2", 26, 3072, 768, 1, 1, _lib.EPI_F32_RESID, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="-1,4,5,7")
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    tiles = [int(t) for t in a.tiles.split(",")]
    total = {t: 0.0 for t in tiles}
    best_total = 0.0
    for name, g, cin, cout, k, s, epi, cnt in SHAPES:
        x3 = K.split_planes(torch.randn(a.batch, g, g, cin, device=dev))
        wp = K.split_planes_weight(torch.randn(cout, k, k, cin, device=dev) * (k * k * cin) ** -0.5)
        b = torch.randn(cout, device=dev) * 0.1
        oh = (g - k) // s + 1
        sc = torch.rand(cout, device=dev)
        r = torch.randn(a.batch, oh, oh, cout, device=dev) if epi == _lib.EPI_F32_RESID else None
        fl = 2.0 * a.batch * oh * oh * cout * k * k * cin
        line = f"{name:7s} M={a.batch * oh * oh:6d} N={cout:5d} K={k * k * cin:5d}"
        best = float("inf")
        for t in tiles:
            def run():
                K.conv_s3(x3, wp, k, k, cout, b, s, 0, epi, scale=sc if r is not None else None, r=r,
                          out=r, tile=t)
            try:
                run()
                run()
            except RuntimeError:
                line += f"  t{t}:   n/a"
                total[t] += float("nan")
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            total[t] += ms * cnt
            best = min(best, ms)
            line += f"  t{t}: {fl / ms / 1e9:6.1f} TF ({ms * 1e3:5.0f} us)"
        best_total += best * cnt
        print(line, flush=True)
    print("network split-GEMM time (ms):", " ".join(f"t{t}={v:.2f}" for t, v in total.items()),
          f"best-per-shape={best_total:.2f}", flush=True)


if __name__ == "__main__":
    main()
