"""ResNet-50 PIP-Net training throughput on one GPU (C3 shapes: 224x224, 200 classes, batch B
per view, so one iteration forwards 2B images, train.py:84).  Synthetic trained-like weights.

* joint phase ("train + freeze params", main.py:377-390 with the util/args.py:280-290 ResNet
  groups: layer3 + layer4 + classifier train; every BatchNorm in train mode):
  HIP = count_pipnet_amd.train.hip_train_step (train-mode BN kernels, Bottleneck backward,
  AdamW for every trainable tensor); torch = autograd through the same modules on ROCm
  (MIOpen / rocBLAS) with torch.optim.AdamW -- what the reference's loop costs on this GPU;
* finetune phase (classifier only; the backbone still runs train-mode BN):
  HIP = hip_finetune_step; torch = the same module's torch path.

Prints one JSON line per phase: images/s and ms per iteration for both.

    python tools/bench_train_resnet.py [--batch 64] [--steps 5]
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from bench_train import timed, torch_joint_step, torch_step  # noqa: E402
from count_pipnet_amd import train as T  # noqa: E402
from count_pipnet_amd.pipnet import get_pipnet  # noqa: E402
from count_pipnet_amd.synthetic import fill_module_  # noqa: E402


def build(dev, joint: bool, num_classes=200):
    args = argparse.Namespace(net="resnet50", disable_pretrained=True, num_features=0, bias=False)
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_pipnet(num_classes, args)
    fill_module_(net, 31, "trained")
    net = net.to(dev).train()
    for p in net.parameters():
        p.requires_grad = False
    net._classification.weight.requires_grad = True
    opt = torch.optim.AdamW([{"params": [net._classification.weight], "lr": 0.05, "weight_decay": 0.0}], lr=0.05)
    if not joint:
        return net, opt, None
    suffix = [p for n, p in net._net.named_parameters() if n.startswith(("layer3", "layer4"))]
    for p in suffix:
        p.requires_grad = True
    opt_net = torch.optim.AdamW([{"params": suffix, "lr": 5e-4, "weight_decay": 0.0}], lr=5e-4)
    return net, opt, opt_net


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64, help="images per view (iteration = 2x)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--torch-steps", type=int, default=3)
    ap.add_argument("--phases", default="joint,finetune")
    ap.add_argument("--hip-only", action="store_true", help="skip the torch-path timing (profiling runs)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    xs1 = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev)
    xs2 = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev)
    ys = torch.randint(0, 200, (a.batch,), generator=g).to(dev)
    imgs = 2 * a.batch
    out = {}
    for phase in a.phases.split(","):
        net, opt, opt_net = build(dev, phase == "joint")
        if phase == "joint":
            hip_s = timed(lambda: T.hip_train_step(net, xs1, xs2, ys, opt_net, opt, False, 1, 1, True), a.steps,
                          a.warmup)
        else:
            hip_s = timed(lambda: T.hip_finetune_step(net, xs1, xs2, ys, opt, True), a.steps, a.warmup)
        del net, opt, opt_net
        torch.cuda.empty_cache()
        if a.hip_only:
            print(json.dumps({"phase": phase, "hip_ms_per_iter": hip_s * 1e3}), flush=True)
            continue
        net, opt, opt_net = build(dev, phase == "joint")
        if phase == "joint":
            torch_s = timed(lambda: torch_joint_step(net, opt, opt_net, xs1, xs2, ys), a.torch_steps, 1)
        else:
            torch_s = timed(lambda: torch_step(net, opt, xs1, xs2, ys), a.torch_steps, 1)
        del net, opt, opt_net
        torch.cuda.empty_cache()
        out[phase] = {
            "metric": f"{phase}-phase iteration images/sec (ResNet-50 PIP-Net, 224x224, "
                      + ("layer3-4 + classifier" if phase == "joint" else "classifier-only, train-mode BN") + ")",
            "images_per_iteration": imgs, "hip_images_per_sec": imgs / hip_s, "hip_ms_per_iter": hip_s * 1e3,
            "torch_images_per_sec": imgs / torch_s, "torch_ms_per_iter": torch_s * 1e3,
            "speedup_vs_torch_path": torch_s / hip_s}
        print(json.dumps(out[phase]), flush=True)


if __name__ == "__main__":
    main()
