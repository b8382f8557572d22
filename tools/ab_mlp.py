"""A/B of the fused narrow-stage CNBlock MLP (csrc/mlp_f32.hip) against the unfused Linear1+GELU /
Linear2+residual GEMMs on the C2 (ConvNeXt-26, 64 x 224^2) and C5 (mid-layer, 64 x 128^2, 2048
prototypes) forwards, interleaved rounds in one process; also times the stage-1/2 MLPs alone.

    python tools/ab_mlp.py [--rounds 5] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib, build, convnext_features  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_configs import CONFIGS, make  # noqa: E402


def timed(fn, steps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    # the MLPs alone at the C2 stage-1 / stage-2 and C5 sizes
    g = torch.Generator(device=dev).manual_seed(0)
    for c, m in [(96, 64 * 56 * 56), (192, 64 * 28 * 28), (96, 64 * 32 * 32), (192, 64 * 16 * 16)]:
        t = torch.randn(m, c, device=dev, generator=g)
        x = torch.randn(m, c, device=dev, generator=g)
        w1 = torch.randn(4 * c, c, device=dev, generator=g) * 0.1
        b1 = torch.randn(4 * c, device=dev, generator=g) * 0.1
        w2 = torch.randn(c, 4 * c, device=dev, generator=g) * 0.05
        b2 = torch.randn(c, device=dev, generator=g)
        gm = torch.randn(c, device=dev, generator=g)
        fl = 2.0 * 2 * m * 4 * c * c

        def fused():
            K.cnblock_mlp(t, w1, b1, w2, b2, gm, x)

        def unfused():
            u = K.linear(t, w1, b1, _lib.EPI_BIAS_GELU)
            K.linear(u, w2, b2, _lib.EPI_RESID, scale=gm, r=x, out=x)
        res = {"fused": [], "unfused": []}
        for _ in range(a.rounds):
            res["fused"].append(timed(fused, a.steps))
            res["unfused"].append(timed(unfused, a.steps))
        rec = {"mlp": f"C={c} M={m}"}
        for k, v in res.items():
            ms = sorted(v)[len(v) // 2]
            rec[k + "_us"] = ms * 1e3
            rec[k + "_tflops"] = fl / (ms * 1e-3) / 1e12
        print(json.dumps(rec), flush=True)
    # whole forwards
    for name, batch in (("c2", 64), ("c5", 64)):
        if name == "c2":
            cfg = dict(model="pipnet", batch=64, size=224, classes=200,
                       args=dict(net="convnext_tiny_26", num_features=0, bias=False))
        else:
            cfg = CONFIGS["c5"]
        net = make(cfg, dev)
        xs = torch.randn(cfg["batch"], 3, cfg["size"], cfg["size"], device=dev)
        res = {True: [], False: []}
        for _ in range(a.rounds):
            for fusedv in (True, False):
                convnext_features.FUSED_MLP = fusedv
                with torch.no_grad():
                    res[fusedv].append(timed(lambda: net(xs, inference=True), a.steps))
        convnext_features.FUSED_MLP = True
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        print(json.dumps({"forward": name, "batch": cfg["batch"], "fused_ms": med[True], "unfused_ms": med[False],
                          "fused_img_s": cfg["batch"] / med[True] * 1e3,
                          "unfused_img_s": cfg["batch"] / med[False] * 1e3}), flush=True)
        del net


if __name__ == "__main__":
    main()
