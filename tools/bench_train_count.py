"""CountPIPNet training throughput on one GPU (CountPIPNet slices).

C5 shapes per GPU: CountPIPNet bilinear.yaml with a 2048-prototype head (mid-layer
ConvNeXt-tiny, num_stages=3, 128x128, max_count 3, STE), 64 images per view, so one
iteration forwards 128 images (cat([xs1, xs2]), train.py:84).  Synthetic trained-like
weights, fresh Philox Gumbel noise per forward.

* finetune (main.py:333-343): classifier + bilinear intermediate train (train_intermediate);
  HIP = count_pipnet_amd.train.hip_count_finetune_step;
* joint ("train + freeze params", main.py:360-390): backbone stages 2-3 + add-on + classifier
  + intermediate train; HIP = hip_count_train_step (count head / STE / intermediate backward
  kernels, suffix backward, device AdamW);
* torch: the same modules on their torch path in train mode (ROCm ATen / MIOpen / rocBLAS,
  autograd, torch.optim.AdamW) -- what the reference's loop costs on this GPU.  The loss is
  written inline here (same math, not the reference's code).

Prints one JSON line per phase: images/s and ms per iteration for both.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from count_pipnet_amd import train as T  # noqa: E402
from count_pipnet_amd.backend import torch_backend  # noqa: E402
from count_pipnet_amd.count_pipnet import get_count_network  # noqa: E402
from count_pipnet_amd.synthetic import fill_module_  # noqa: E402

NUM_CLASSES = 9


def build(dev, joint: bool):
    args = argparse.Namespace(net="convnext_tiny_26", disable_pretrained=True, use_mid_layers=True, num_stages=3,
                              num_features=2048, activation="gumbel_softmax", intermediate_layer="bilinear",
                              max_count=3, use_ste=True, bias=False, backward_clamp_strategy="Gated")
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_count_network(NUM_CLASSES, args, max_count=3, use_ste=True)
    fill_module_(net, 15, "trained")
    net = net.to(dev).train()
    for p in net.parameters():
        p.requires_grad = False
    cls = net._classification
    cls.weight.requires_grad = True
    inter = list(net._intermediate.parameters())
    for p in inter:
        p.requires_grad = True
    opt_cls = torch.optim.AdamW([{"params": [cls.weight], "lr": 0.05, "weight_decay": 0.01},
                                 {"params": inter, "lr": 0.05, "weight_decay": 0.01}], lr=0.05)
    if not joint:
        return net, opt_cls, None
    suffix = [p for n, p in net._net.named_parameters() if n.split(".")[1] in ("2", "3")]
    for p in suffix + list(net._add_on.parameters()):
        p.requires_grad = True
    opt_net = torch.optim.AdamW([{"params": suffix, "lr": 5e-4, "weight_decay": 0.0},
                                 {"params": list(net._add_on.parameters()), "lr": 5e-3, "weight_decay": 0.0}],
                                lr=5e-4)
    return net, opt_cls, opt_net


def torch_step(net, opt_cls, opt_net, xs1, xs2, ys, joint: bool):
    """One iteration on the torch path; finetune: 2 * class; joint: 5 align + 2 tanh + 2 class."""
    opt_cls.zero_grad(set_to_none=True)
    if opt_net is not None:
        opt_net.zero_grad(set_to_none=True)
    with torch_backend():
        proto, counts, out = net(torch.cat([xs1, xs2]))
    cls = net._classification
    cls_loss = F.cross_entropy(torch.log1p(out ** cls.normalization_multiplier), torch.cat([ys, ys]))
    if joint:
        n = counts.shape[0] // 2
        e1 = proto[:n].flatten(2).transpose(1, 2).reshape(-1, proto.shape[1])
        e2 = proto[n:].flatten(2).transpose(1, 2).reshape(-1, proto.shape[1])
        align = 0.5 * (-torch.log((e1 * e2.detach()).sum(1) + 1e-12).mean()
                       - torch.log((e2 * e1.detach()).sum(1) + 1e-12).mean())
        tanh = -0.5 * sum(torch.log(torch.tanh(h.sum(0)) + 1e-8).mean() for h in counts.chunk(2))
        loss = 5.0 * align + 2.0 * tanh + 2.0 * cls_loss
    else:
        loss = 2.0 * cls_loss
    loss.backward()
    opt_cls.step()
    if opt_net is not None:
        opt_net.step()
    with torch.no_grad():
        cls.weight.copy_(torch.clamp(cls.weight - 1e-3, min=0.0))
        cls.normalization_multiplier.clamp_(min=1.0)
    return loss.detach()


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64, help="images per view (iteration = 2x)")
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--torch-steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    xs1 = torch.randn(a.batch, 3, a.size, a.size, generator=g).to(dev)
    xs2 = torch.randn(a.batch, 3, a.size, a.size, generator=g).to(dev)
    ys = torch.randint(0, NUM_CLASSES, (a.batch,), generator=g).to(dev)
    imgs = 2 * a.batch
    sdg = torch.Generator().manual_seed(1)
    for joint in (False, True):
        net, opt_cls, opt_net = build(dev, joint)
        if joint:
            assert T.hip_count_train_supported(net)
            hip = timed(lambda: T.hip_count_train_step(net, xs1, xs2, ys, opt_net, opt_cls, False, 1, 1, True, 1.0,
                                                       generator=sdg), a.steps, a.warmup)
        else:
            assert T.hip_count_finetune_supported(net)
            hip = timed(lambda: T.hip_count_finetune_step(net, xs1, xs2, ys, opt_cls, True, 1.0, generator=sdg),
                        a.steps, a.warmup)
        del net, opt_cls, opt_net
        torch.cuda.empty_cache()
        net, opt_cls, opt_net = build(dev, joint)
        tt = timed(lambda: torch_step(net, opt_cls, opt_net, xs1, xs2, ys, joint), a.torch_steps, 1)
        del net, opt_cls, opt_net
        torch.cuda.empty_cache()
        phase = ("joint-phase (stages 2-3 + add-on + classifier + bilinear intermediate)" if joint
                 else "finetune (classifier + bilinear intermediate)")
        print(json.dumps({
            "metric": f"CountPIPNet {phase} iteration images/sec (C5: bilinear, P=2048, {a.size}x{a.size})",
            "images_per_iteration": imgs, "hip_images_per_sec": imgs / hip, "hip_ms_per_iter": hip * 1e3,
            "torch_images_per_sec": imgs / tt, "torch_ms_per_iter": tt * 1e3, "speedup_vs_torch_path": tt / hip}),
            flush=True)


if __name__ == "__main__":
    main()
