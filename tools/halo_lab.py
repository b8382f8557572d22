"""Time breakdown of the 3x3 LDS-halo ping-pong conv (conv3x3_bf16_halo_kernel, C3's dominant kernel) by
ablation (tools/bf16_lab.hip lab_halo; ABL bits 1 = no B DMA, 2 = no epilogue, 4 = no barriers, 8 = no A
fragment reads, 16 = no halo DMA; 1000 + bits = the one-32-MFMA-segment-per-K-tile schedule, SEG = 1), on the
layer3 / layer4 conv2 shapes at the two-stream half batch and the full batch.  Variants 0 / 1000 are full
kernels (checked bitwise against the library's tile 8).

    python tools/halo_lab.py            (HALO_VARIANTS=0,1,2,... HALO_ROUNDS=3)
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

import bf16_lab  # noqa: E402

SHAPES = [("l3.c2", 64, 28, 256, 256), ("l4.c2", 64, 28, 512, 512), ("l3.c2", 128, 28, 256, 256),
          ("l4.c2", 128, 28, 512, 512)]


def main():
    lib = bf16_lab.build()
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.lab_halo.argtypes = [I, P, I, I, I, I, P, I, P, P]
    variants = [int(v) for v in os.environ.get("HALO_VARIANTS", "0,1000,3000,2,1002,3002,19,1019,3019").split(",")]
    rounds = int(os.environ.get("HALO_ROUNDS", "3"))
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    stream = torch.cuda.current_stream().cuda_stream
    for name, b, hw, cin, n in SHAPES:
        x = (torch.rand(b, hw, hw, cin, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = K.pack_conv_weight_bf16(torch.randn(n, 3, 3, cin, device=dev, generator=g) * 0.05)
        y = torch.empty(b, hw, hw, n, device=dev, dtype=torch.bfloat16)
        ref = K.conv2d_nhwc_bf16(x, w, 3, 3, None, 1, 1, _lib.EPI_NONE, tile=8)
        same = {}
        for v in [v for v in variants if v in (0, 1000, 3000)]:   # full (non-ablated) forms: bitwise the library's tile 8
            y.zero_()
            assert lib.lab_halo(v, x.data_ptr(), b, hw, hw, cin, w.data_ptr(), n, y.data_ptr(), stream) == 0
            torch.cuda.synchronize()
            same[v] = torch.equal(y, ref)
        flops = 2.0 * b * hw * hw * n * 9 * cin
        times = {v: [] for v in variants}
        for _ in range(rounds):
            for v in variants:
                def run():
                    assert lib.lab_halo(v, x.data_ptr(), b, hw, hw, cin, w.data_ptr(), n, y.data_ptr(), stream) == 0
                for _ in range(2):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 10 * 1e3)
        rec = {"layer": name, "batch": b, "bitwise_tile8": same}
        for v in variants:
            us = sorted(times[v])[len(times[v]) // 2]
            rec[f"abl{v}"] = {"us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
