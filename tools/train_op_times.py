"""Per-op GPU time of one ResNet-50 PIP-Net joint iteration on the HIP path: every
``kernels`` entry point the train-mode backbone calls is wrapped with HIP events (synchronised
per call, so the numbers are isolated op times, not overlapped ones) and reported with its
shapes and achieved TF/s (GEMM-shaped ops).

    python tools/train_op_times.py [--batch 64]
"""
from __future__ import annotations

import argparse
import collections
import functools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from bench_train_resnet import build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402
from count_pipnet_amd import train as T  # noqa: E402

RECS = []


def _flops(name, args, kw, out):
    try:
        if name == "conv2d_nhwc":
            x, w = args[0], args[1]
            o = out
            return 2.0 * o.numel() * w.shape[1] * w.shape[2] * w.shape[3]
        if name == "linear":
            x, w = args[0], args[1]
            return 2.0 * x.shape[0] * x.shape[1] * w.shape[0]
        if name == "wgrad":
            dy, x = args[0], args[1]
            return 2.0 * dy.shape[0] * dy.shape[1] * x.shape[1]
        if name == "wgrad_conv":
            dy, x, kh, kw_ = args[0], args[1], args[2], args[3]
            return 2.0 * dy.shape[0] * dy.shape[1] * dy.shape[2] * dy.shape[3] * x.shape[3] * kh * kw_
    except Exception:  # noqa: BLE001
        return 0.0
    return 0.0


def _shape(a):
    return tuple(a.shape) if torch.is_tensor(a) else a


def wrap(name):
    fn = getattr(K, name)

    @functools.wraps(fn)
    def inner(*args, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        out = fn(*args, **kw)
        e1.record()
        torch.cuda.synchronize()
        first = out[0] if isinstance(out, tuple) else out
        RECS.append((name, tuple(_shape(a) for a in args[:4] if torch.is_tensor(a) or isinstance(a, int)),
                     e0.elapsed_time(e1), _flops(name, args, kw, first)))
        return out
    setattr(K, name, inner)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    xs1 = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev)
    xs2 = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev)
    ys = torch.randint(0, 200, (a.batch,), generator=g).to(dev)
    net, opt, opt_net = build(dev, True)
    step = lambda: T.hip_train_step(net, xs1, xs2, ys, opt_net, opt, False, 1, 1, True)  # noqa: E731
    step()
    torch.cuda.synchronize()
    for n in ("conv2d_nhwc", "linear", "wgrad", "wgrad_conv", "bn_stats", "bn_apply", "bn_backward",
              "stride_scatter", "maxpool2d_nhwc"):
        wrap(n)
    RECS.clear()
    step()
    torch.cuda.synchronize()
    tot = collections.defaultdict(float)
    for name, shp, ms, fl in RECS:
        tot[name] += ms
        tf = f"{fl / ms / 1e9:7.1f} TF/s" if fl else ""
        print(f"{name:15s} {ms:8.3f} ms {tf:>12s}  {shp}")
    print("totals (ms):", {k: round(v, 2) for k, v in sorted(tot.items(), key=lambda t: -t[1])},
          "sum", round(sum(tot.values()), 2))


if __name__ == "__main__":
    main()
