"""Where the bf16 1x1 tiles lose to the vendor GEMM: per-CU efficiency vs tile quantisation.

Times the persistent ping-pong tile (9), the ping-pong tile (5) and hipBLASLt (torch linear,
no epilogue) on dense bf16 GEMMs: the C3 layer shapes at 64 images (M = 50,176: 196 row
tiles of 256, so N = 256 / 512 / 1024 give 0.77 / 1.53 / 3.06 waves of 256x256 tiles on 256
CUs) beside the same N, K at M = 65,536 (whole waves), and square GEMMs.  Interleaved rounds
in one process, median of 5 (cdna_hip_programming.md rule 24).
    python tools/c3_diag.py [--reps 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

SHAPES = [  # (name, M, N, K)
    ("l3.c1", 50176, 256, 1024), ("l3.c1/w", 65536, 256, 1024),
    ("l4.c1", 50176, 512, 2048), ("l4.c1/w", 65536, 512, 2048),
    ("l3.c3", 50176, 1024, 256), ("l3.c3/w", 65536, 1024, 256),
    ("l4.ds", 50176, 2048, 1024), ("l4.ds/w", 65536, 2048, 1024),
    ("l4.c3", 50176, 2048, 512),
    ("sq4k", 4096, 4096, 4096), ("sq8k", 8192, 8192, 8192),
]


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tiles", default="9,5")
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    tiles = [int(t) for t in a.tiles.split(",")]
    for name, m, n, k in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        x = torch.randn(1, 1, m, k, device=dev, generator=g).to(torch.bfloat16)
        w = torch.randn(n, k, device=dev, generator=g).mul_(0.05)
        wp = K.pack_conv_weight_bf16(w.view(n, 1, 1, k))
        wb = w.to(torch.bfloat16)
        b = torch.randn(n, device=dev, generator=g)
        x2 = x.view(m, k)
        def conv(t):
            return K.conv2d_nhwc_bf16(x, wp, 1, 1, b, 1, 0, _lib.EPI_BIAS_RELU, None, tile=t)
        fns = {}
        for t in tiles:
            fns[f"t{t}"] = (lambda t=t: conv(t))
        fns["lib"] = lambda: torch.nn.functional.linear(x2, wb)
        for f in fns.values():
            f(), f()
        torch.cuda.synchronize()
        res = {key: [] for key in fns}
        for _ in range(5):
            for key, f in fns.items():
                res[key].append(timed(f, a.reps))
        flops = 2.0 * m * n * k
        tiles256 = -(-m // 256) * -(-n // 256)
        line = f"{name:8s} M={m:6d} N={n:5d} K={k:5d} tiles256={tiles256:5d} waves={tiles256 / 256:5.2f}"
        for key, v in res.items():
            ms = sorted(v)[len(v) // 2]
            line += f"  {key}: {flops / ms / 1e9:7.1f} TF ({ms * 1e3:7.1f} us)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
