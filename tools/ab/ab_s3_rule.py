"""A/B two tile rules for the split-bf16 GEMMs inside the full C2 forward (one process, one
GPU, alternating runs so clock / thermal drift cancels).

    python tools/ab_s3_rule.py [--rounds 4] [--steps 20]
Rule "auto": the library's choice.  Rule "pp": the ping-pong 256-wide tile for every N >= 192,
the 128x128 tile (or 64x128 at small M) below.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
from count_pipnet_amd import build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402
from count_pipnet_amd.synthetic import synth_images  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    net, _ = bench.make_net(dev, precision="bf16x3")
    xs = synth_images(64, 224, seed=100).to(dev)
    orig = K.conv_s3

    def pp_rule(x2, w, kh, kw, cout, *args, tile=-1, **kw_):
        if tile == -1:
            b, h, wd, _ = x2.shape
            m = b * ((h - kh) // args[1] + 1) * ((wd - kw) // args[1] + 1)
            tile = 5 if cout >= 192 else (4 if -(-m // 128) * -(-cout // 128) >= 512 else 0)
        return orig(x2, w, kh, kw, cout, *args, tile=tile, **kw_)

    rules = {"auto": orig, "pp": pp_rule}
    res = {k: [] for k in rules}
    with torch.no_grad():
        for _ in range(a.rounds):
            for name, fn in rules.items():
                K.conv_s3 = fn
                for _ in range(3):
                    net(xs, inference=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    net(xs, inference=True)
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) / a.steps * 1e3)
    K.conv_s3 = orig
    for name, v in res.items():
        print(f"{name:5s} ms/step: min {min(v):.3f}  all " + " ".join(f"{x:.3f}" for x in v), flush=True)


if __name__ == "__main__":
    main()
