"""C5's BilinearIntermediate GEMMs at M = 64 (batch): embed 2048 -> 6144, W and V 6144 x 6144,
weight-read bound.  Times kernels.linear (split-K path) per shape with HIP events and reports
weight TB/s and fp32 TF/s.

    python tools/skinny_bench.py [--iters 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

SHAPES = [("embed", 64, 6144, 2048, _lib.EPI_BIAS), ("W", 64, 6144, 6144, _lib.EPI_NONE),
          ("V_mul", 64, 6144, 6144, _lib.EPI_MUL)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=48)
    ap.add_argument("--rotate", type=int, default=3,
                    help="weight copies cycled per call (3 x 151 MB > the 256 MB Infinity Cache: HBM-cold "
                         "weights, as in the network where W and V stream once per forward)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = []
    tot = 0.0
    for name, m, n, k, epi in SHAPES:
        A = torch.randn(m, k, device=dev, generator=g)
        Ws = [torch.randn(n, k, device=dev, generator=g) * 0.02 for _ in range(a.rotate)]
        W = Ws[0]
        b = torch.randn(n, device=dev, generator=g)
        R = torch.randn(m, n, device=dev, generator=g) if epi == _lib.EPI_MUL else None
        out = torch.empty(m, n, device=dev)
        for _ in range(5):
            K.linear(A, W, b if epi == _lib.EPI_BIAS else None, epi, r=R, out=out)
        ref = (A.double() @ W.double().t() + (b.double() if epi == _lib.EPI_BIAS else 0))
        if R is not None:
            ref = ref * R.double()
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for i in range(a.iters):
            K.linear(A, Ws[i % a.rotate], b if epi == _lib.EPI_BIAS else None, epi, r=R, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / a.iters * 1e3
        tot += us
        rec = dict(shape=name, M=m, N=n, K=k, splits=K.splitk_factor(m, n, k), us=us,
                   weight_tbps=n * k * 4 / us / 1e6, tflops=2.0 * m * n * k / us / 1e6, rel_err=err)
        res.append(rec)
        del Ws, W
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": tot, "splitk_wg_per_cu": K.SPLITK_WG_PER_CU}), flush=True)


if __name__ == "__main__":
    main()
