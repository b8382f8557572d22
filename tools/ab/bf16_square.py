"""Main-loop ceiling check of the bf16 GEMM tiles on large square GEMMs (1x1 conv, dense A),
against the vendor library (torch bf16 matmul = hipBLASLt) on the same random data.

    python tools/bf16_square.py [--sizes 4096,8192] [--reps 10] [--tiles -1,5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from count_pipnet_amd import _lib, build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
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
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="-1")
    ap.add_argument("--epi", type=int, default=_lib.EPI_NONE)
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    for n in [int(s) for s in a.sizes.split(",")]:
        # M = n pixels as [n/64, 8, 8] images, Cin = Cout = n
        x = (torch.rand(n // 64, 8, 8, n, device=dev) * 2 - 1).to(torch.bfloat16)
        wf = torch.rand(n, 1, 1, n, device=dev) * 2 - 1
        w = K.pack_conv_weight_bf16(wf)
        b = torch.zeros(n, device=dev)
        flops = 2.0 * n * n * n
        line = f"{n}^3"
        for t in [int(v) for v in a.tiles.split(",")]:
            ms = timeit(lambda: K.conv2d_nhwc_bf16(x, w, 1, 1, b, 1, 0, a.epi, None, tile=t), a.reps)
            line += f"  t{t}: {flops / ms / 1e9:7.1f} TF"
        a2 = x.reshape(n, n)
        wt = wf.reshape(n, n).to(torch.bfloat16)
        ms = timeit(lambda: torch.nn.functional.linear(a2, wt), a.reps)
        line += f"  hipBLASLt: {flops / ms / 1e9:7.1f} TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
