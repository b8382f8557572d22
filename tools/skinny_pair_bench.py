"""Time C5's bilinear pair GEMM (M = 64 images, N = 2 x 6144, K = 2048 prototypes, fp32) through the
C ABI at several split-K factors, beside a plain 100 MB weight read and torch.matmul, to see how far
the weight stream is from HBM speed.

    python tools/skinny_pair_bench.py [--m 64] [--nh 6144] [--k 2048]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3        # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--nh", type=int, default=6144)
    ap.add_argument("--k", type=int, default=2048)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    m, nh, k = a.m, a.nh, a.k
    x = torch.randint(0, 4, (m, k), device=dev, generator=g).float()
    w = torch.randn(2 * nh, k, device=dev, generator=g) * 0.02
    wbytes = w.numel() * 4
    out = torch.empty(m, nh, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    res = {"shape": [m, 2 * nh, k], "weight_MB": wbytes / 1e6, "product_splits": K.splitk_factor(m, 2 * nh, k)}
    ref = K.linear_pair_mul(x, w)
    for splits in (1, 2, 4, 6, 8, 12, 16, 32, 64):
        if splits > k // 32:
            continue
        ws = torch.empty(splits, m, 2 * nh, device=dev)

        def run():
            _lib.call("pipnet_linear_pair_mul_f32", x.data_ptr(), x.stride(0), w.data_ptr(), out.data_ptr(),
                      out.stride(0), m, nh, k, splits, ws.data_ptr(), s)
        us = timed(run)
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        res[f"splits{splits}_us"] = round(us, 1)
        res[f"splits{splits}_TBs"] = round(wbytes / us / 1e6, 2)
        res[f"splits{splits}_relerr"] = err
    res["read_sum_us"] = round(timed(lambda: w.sum()), 1)
    res["read_sum_TBs"] = round(wbytes / res["read_sum_us"] / 1e6, 2)
    res["torch_matmul_us"] = round(timed(lambda: torch.matmul(x, w.t())), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
