"""Per-layer throughput of the bf16 implicit-GEMM conv on the ResNet50 (layer3/4 stride 1)
shapes of BASELINE C3 (bs=128, 224x224), for every workgroup tile and the automatic choice.

    python tools/conv_bf16_bench.py [--batch 128] [--reps 10]
Prints one line per layer shape: TFLOP/s per tile (0 = 64x128, 1 = 128x128, 2 = 256x256).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib, build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

# (name, H_in, Cin, Cout, k, stride, pad, epilogue, count in the network)
LAYERS = [
    ("stem7x7", 224, 8, 64, 7, 2, 3, _lib.EPI_BIAS_RELU, 1),
    ("l1.c1", 56, 256, 64, 1, 1, 0, _lib.EPI_BIAS_RELU, 2),
    ("l1.c2", 56, 64, 64, 3, 1, 1, _lib.EPI_BIAS_RELU, 3),
    ("l1.c3", 56, 64, 256, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 3),
    ("l2.c1", 56, 512, 128, 1, 1, 0, _lib.EPI_BIAS_RELU, 1),
    ("l2.c2s2", 56, 128, 128, 3, 2, 1, _lib.EPI_BIAS_RELU, 1),
    ("l2.ds", 56, 256, 512, 1, 2, 0, _lib.EPI_BIAS, 1),
    ("l2.c2", 28, 128, 128, 3, 1, 1, _lib.EPI_BIAS_RELU, 3),
    ("l2.c3", 28, 128, 512, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 4),
    ("l3.c1", 28, 1024, 256, 1, 1, 0, _lib.EPI_BIAS_RELU, 5),
    ("l3.c2", 28, 256, 256, 3, 1, 1, _lib.EPI_BIAS_RELU, 6),
    ("l3.c3", 28, 256, 1024, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 6),
    ("l4.c1", 28, 2048, 512, 1, 1, 0, _lib.EPI_BIAS_RELU, 2),
    ("l4.c2", 28, 512, 512, 3, 1, 1, _lib.EPI_BIAS_RELU, 3),
    ("l4.c3", 28, 512, 2048, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 3),
    ("l4.ds", 28, 1024, 2048, 1, 1, 0, _lib.EPI_BIAS, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default=None, help="comma-separated layer names")
    ap.add_argument("--tiles", default="-1,0,1,2,3,4,5")
    ap.add_argument("--rotate", type=int, default=1,
                    help="cycle through this many input / identity / output buffer sets, so a layer's "
                         "working set exceeds the 256 MB Infinity Cache as it does in the network")
    ap.add_argument("--lib", action="store_true",
                    help="also time the vendor library on the same shape (torch bf16: hipBLASLt GEMM for 1x1 "
                         "convs, MIOpen channels_last conv otherwise) as a reference ceiling")
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    tiles = [int(t) for t in a.tiles.split(',')]
    total = {t: 0.0 for t in tiles}
    for name, h, cin, cout, k, s, pad, epi, cnt in LAYERS:
        if a.only and name not in a.only.split(","):
            continue
        xs = [torch.randn(a.batch, h, h, cin, device=dev).to(torch.bfloat16) for _ in range(a.rotate)]
        w = K.pack_conv_weight_bf16(torch.randn(cout, k, k, cin, device=dev) * 0.05)
        b = torch.randn(cout, device=dev)
        oh = (h + 2 * pad - k) // s + 1
        rs = [torch.randn(a.batch, oh, oh, cout, device=dev).to(torch.bfloat16) if epi == _lib.EPI_BIAS_RESID_RELU
              else None for _ in range(a.rotate)]
        x, r = xs[0], rs[0]
        flops = 2.0 * a.batch * oh * oh * cout * k * k * cin
        auto = K.bf16_conv_plan(a.batch, h, h, cin, cout, k, k, s, pad, epi)
        line = f"{name:8s} M={a.batch * oh * oh:6d} N={cout:4d} K={k * k * cin:5d} auto={auto}"
        for t in tiles:
            ti = t
            try:
                for _ in range(2):
                    K.conv2d_nhwc_bf16(x, w, k, k, b, s, pad, epi, r, tile=ti)
            except RuntimeError:          # tile not applicable to this layer (e.g. 5 on the Cin=8 stem)
                line += f"  t{t}:    n/a"
                total[t] += float("nan")
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(a.reps):
                K.conv2d_nhwc_bf16(xs[i % a.rotate], w, k, k, b, s, pad, epi, rs[i % a.rotate], tile=ti)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            total[t] += ms * cnt
            line += f"  t{t}: {flops / ms / 1e9:6.1f} TF ({ms * 1e3:6.0f} us)"
        if a.lib:
            ms = _time_lib(x, w.shape, cout, k, s, pad, a.reps, dev)
            total.setdefault("lib", 0.0)
            total["lib"] += ms * cnt
            line += f"  lib: {flops / ms / 1e9:6.1f} TF ({ms * 1e3:6.0f} us)"
        print(line, flush=True)
    print("network conv time (ms, sum over layers x count):",
          " ".join(f"t{t}={v:.2f}" for t, v in total.items()), flush=True)


def _time_lib(x, wshape, cout, k, s, pad, reps, dev):
    """Vendor-library time of the same conv (no fused epilogue): hipBLASLt for 1x1 stride-1,
    MIOpen (torch conv2d, channels_last bf16) otherwise."""
    b, h, _, cin = x.shape
    if k == 1 and s == 1:
        a2 = x.reshape(-1, cin)
        wt = torch.randn(cout, cin, device=dev).to(torch.bfloat16)
        fn = lambda: torch.nn.functional.linear(a2, wt)      # noqa: E731
    else:
        xc = x.permute(0, 3, 1, 2)                             # NCHW view of NHWC storage = channels_last
        wt = torch.randn(cout, cin, k, k, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        fn = lambda: torch.nn.functional.conv2d(xc, wt, stride=s, padding=pad)    # noqa: E731
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


if __name__ == "__main__":
    main()
