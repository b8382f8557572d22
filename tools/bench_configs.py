"""Throughput of the non-headline BASELINE configs on one GPU (bench.py measures configs[1]).

  C1  CountPIPNet identity.yaml, 64x64, bs=16          (the reference's CPU case; here on HIP)
  C2  PIP-Net ConvNeXt-tiny-26 224x224, bs=64, fp32     (bench.py's headline, for stream-split A/B)
  C3  PIP-Net ResNet50 224x224, bs=128, bf16 (BASELINE C3) and fp32 (exact reference arithmetic)
  C5  CountPIPNet bilinear 2048 prototypes, 128x128, 64 images per GPU (bs=256 over 4 GPUs)
  C2' PIP-Net ConvNeXt-tiny-13 224x224, bs=64          (the 13x13 variant)
  *_bf16x3: the same ConvNeXt configs with split-bf16 GEMMs (set_hip_dtype "bf16x3")

    python tools/bench_configs.py [--steps 10] [--only c5] [--stream-split 2]
Prints one JSON line per config (images/sec, ms/step, model TFLOP/s where defined).
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import build  # noqa: E402
from count_pipnet_amd.count_pipnet import get_count_network  # noqa: E402
from count_pipnet_amd.pipnet import get_pipnet, set_stream_split  # noqa: E402
from count_pipnet_amd.pipnet import stream_split as _stream_split  # noqa: E402


def split_of(net, xs):
    return _stream_split(net, xs) if hasattr(net, "_hip_logits") else 1
from count_pipnet_amd.synthetic import fill_module_, synth_images  # noqa: E402

CONFIGS = {
    "c1": dict(model="count", batch=16, size=64, classes=9,
               args=dict(net="convnext_tiny_26", use_mid_layers=True, num_stages=3, num_features=16,
                         activation="gumbel_softmax", intermediate_layer="identity", max_count=3, use_ste=True,
                         bias=False), gflop=0.2495),
    "c2": dict(model="pipnet", batch=64, size=224, classes=200,
               args=dict(net="convnext_tiny_26", num_features=0, bias=False), gflop=40.094),
    "c3": dict(model="pipnet", batch=128, size=224, classes=200, args=dict(net="resnet50", num_features=0, bias=False,
                                                                           hip_dtype="bf16"), gflop=38.16),
    "c3_fp32": dict(model="pipnet", batch=128, size=224, classes=200,
                    args=dict(net="resnet50", num_features=0, bias=False), gflop=38.16),
    "c5": dict(model="count", batch=64, size=128, classes=9,
               args=dict(net="convnext_tiny_26", use_mid_layers=True, num_stages=3, num_features=2048,
                         activation="gumbel_softmax", intermediate_layer="bilinear", max_count=3, use_ste=True,
                         bias=False), gflop=1.248),   # executed: the bilinear embedding is folded into W / V (1.374 reference)
    "c2_13": dict(model="pipnet", batch=64, size=224, classes=200,
                  args=dict(net="convnext_tiny_13", num_features=0, bias=False), gflop=12.617),
}
# the split-bf16 build of every ConvNeXt config (fp32 in / out, three bf16 products per fp32 product)
for _k in ("c1", "c2", "c5", "c2_13"):
    CONFIGS[_k + "_bf16x3"] = dict(CONFIGS[_k], args=dict(CONFIGS[_k]["args"], hip_dtype="bf16x3"))


def make(cfg, dev):
    a = argparse.Namespace(disable_pretrained=True, backward_clamp_strategy="Gated", **cfg["args"])
    with contextlib.redirect_stdout(io.StringIO()):
        if cfg["model"] == "pipnet":
            net, _ = get_pipnet(cfg["classes"], a)
        else:
            net, _ = get_count_network(cfg["classes"], a, max_count=a.max_count, use_ste=a.use_ste)
    fill_module_(net, 7, "trained")
    return net.eval().to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", default=None)
    ap.add_argument("--graph", action="store_true", help="also time HIP-graph replay (count_pipnet_amd.graph)")
    ap.add_argument("--stream-split", type=int, default=0,
                    help="force pipnet.set_stream_split(net, n) on every config (0 = the model's default)")
    a = ap.parse_args()
    build.build()
    dev = torch.device("cuda:0")
    for name, cfg in CONFIGS.items():
        if a.only and name not in a.only.split(","):
            continue
        net = make(cfg, dev)
        if a.stream_split:
            set_stream_split(net, a.stream_split)
        xs = synth_images(cfg["batch"], cfg["size"], seed=5).to(dev)
        with torch.no_grad():
            for _ in range(a.warmup):
                net(xs, inference=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                net(xs, inference=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        ips = cfg["batch"] * a.steps / el
        dt = cfg["args"].get("hip_dtype", "f32")
        # bf16x3 runs three bf16 products per fp32 product: its fp32-equivalent ceiling is
        # the bf16 dense peak / 3 (833 TF/s), not the fp32 MFMA peak
        peak = {"bf16": 2500.0, "bf16x3": 2500.0 / 3.0}.get(dt, 157.3)
        rec = dict(config=name, images_per_sec=ips, ms_per_step=el / a.steps * 1e3, batch=cfg["batch"],
                   image_size=cfg["size"], dtype=dt, model_tflops=ips * cfg["gflop"] / 1e3,
                   model_frac_of_peak=ips * cfg["gflop"] / 1e3 / peak, peak_tflops=peak,
                   stream_split=split_of(net, xs))
        if a.graph:
            from count_pipnet_amd.graph import GraphedForward
            g = GraphedForward(net)
            for _ in range(a.warmup):
                g(xs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                g(xs)
            torch.cuda.synchronize()
            elg = time.perf_counter() - t0
            rec["graph_images_per_sec"] = cfg["batch"] * a.steps / elg
            rec["graph_ms_per_step"] = elg / a.steps * 1e3
            del g
        print(json.dumps(rec), flush=True)
        del net, xs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
