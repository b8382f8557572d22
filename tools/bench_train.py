"""Finetune-phase training throughput on one GPU.

C2 shapes: PIP-Net ConvNeXt-tiny-26, 224x224, 200 classes, batch 64 per view, so one
iteration forwards 128 images (cat([xs1, xs2]), train.py:84).  Synthetic trained-like
weights, classifier-only training (the finetune freeze of main.py:333-345).

* hip:   count_pipnet_amd.train.hip_finetune_step (HIP forward with stochastic depth, loss /
         d_out kernel, NonNegLinear backward, AdamW + clamps), host-drawn SD masks;
* torch: the same module on its torch path in train mode (torchvision-equivalent ops on
         ROCm ATen/MIOpen/rocBLAS, autograd for the classifier, torch.optim.AdamW) -- what
         the reference's loop costs on this GPU.  The loss is written inline here (same
         math, not the reference's code).

Also the joint phase ("train + freeze params", main.py:377-390: features.6 and features.7 +
classifier train, the rest frozen): HIP = count_pipnet_amd.train.hip_train_step (forward
keeping the suffix activations, head / CNBlock / downsample backward kernels, AdamW for every
trainable tensor); torch = autograd through the same modules.

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
from count_pipnet_amd.pipnet import get_pipnet  # noqa: E402
from count_pipnet_amd.synthetic import fill_module_  # noqa: E402


def build(dev, num_classes=200, joint=False):
    args = argparse.Namespace(net="convnext_tiny_26", disable_pretrained=True, num_features=0, bias=False)
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_pipnet(num_classes, args)
    fill_module_(net, 21, "trained")
    net = net.to(dev).train()
    for p in net.parameters():
        p.requires_grad = False
    net._classification.weight.requires_grad = True
    opt = torch.optim.AdamW([{"params": [net._classification.weight], "lr": 0.05, "weight_decay": 0.0}], lr=0.05)
    if not joint:
        return net, opt
    suffix = [p for n, p in net._net.named_parameters() if n.startswith(("features.6", "features.7"))]
    for p in suffix:
        p.requires_grad = True
    opt_net = torch.optim.AdamW([{"params": suffix, "lr": 5e-4, "weight_decay": 0.0}], lr=5e-4)
    return net, opt, opt_net


def torch_joint_step(net, opt, opt_net, xs1, xs2, ys):
    """Joint-phase iteration on the torch path: 5 align + 2 tanh + 2 class (inline loss)."""
    opt.zero_grad(set_to_none=True)
    opt_net.zero_grad(set_to_none=True)
    with torch_backend():
        proto, pooled, out = net(torch.cat([xs1, xs2]))
    cls = net._classification
    n = pooled.shape[0] // 2
    e1 = proto[:n].flatten(2).transpose(1, 2).reshape(-1, proto.shape[1])
    e2 = proto[n:].flatten(2).transpose(1, 2).reshape(-1, proto.shape[1])
    align = 0.5 * (-torch.log((e1 * e2.detach()).sum(1) + 1e-12).mean()
                   - torch.log((e2 * e1.detach()).sum(1) + 1e-12).mean())
    tanh = -0.5 * sum(torch.log(torch.tanh(h.sum(0)) + 1e-8).mean() for h in pooled.chunk(2))
    cls_loss = F.cross_entropy(torch.log1p(out ** cls.normalization_multiplier), torch.cat([ys, ys]))
    loss = 5.0 * align + 2.0 * tanh + 2.0 * cls_loss
    loss.backward()
    opt.step()
    opt_net.step()
    with torch.no_grad():
        cls.weight.copy_(torch.clamp(cls.weight - 1e-3, min=0.0))
        cls.normalization_multiplier.clamp_(min=1.0)
    return loss.detach()


def torch_step(net, opt, xs1, xs2, ys):
    """Classifier-only iteration on the torch path (inline loss: 2 * NLL of log1p(out^m))."""
    opt.zero_grad(set_to_none=True)
    with torch_backend():
        proto, pooled, out = net(torch.cat([xs1, xs2]))
    cls = net._classification
    n = pooled.shape[0] // 2
    e1 = proto[:n].flatten(2).transpose(1, 2).reshape(-1, proto.shape[1])
    e2 = proto[n:].flatten(2).transpose(1, 2).reshape(-1, proto.shape[1])
    with torch.no_grad():                       # logged terms (not in the finetune gradient)
        align = -torch.log((e1 * e2).sum(1) + 1e-12).mean()
        tanh = -0.5 * sum(torch.log(torch.tanh(h.sum(0)) + 1e-8).mean() for h in pooled.chunk(2))
    x = torch.log1p(out ** cls.normalization_multiplier)
    loss = 2.0 * F.cross_entropy(x, torch.cat([ys, ys]))
    loss.backward()
    opt.step()
    with torch.no_grad():
        cls.weight.copy_(torch.clamp(cls.weight - 1e-3, min=0.0))
        cls.normalization_multiplier.clamp_(min=1.0)
    return torch.stack([align, tanh, loss.detach()])


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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--torch-steps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    xs1 = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev)
    xs2 = torch.randn(a.batch, 3, 224, 224, generator=g).to(dev)
    ys = torch.randint(0, 200, (a.batch,), generator=g).to(dev)
    net, opt = build(dev)
    sdg = torch.Generator().manual_seed(1)
    hip_s = timed(lambda: T.hip_finetune_step(net, xs1, xs2, ys, opt, True, generator=sdg), a.steps, a.warmup)
    xs = torch.cat([xs1, xs2])
    fwd_s = timed(lambda: T.train_forward_hip(net, xs, T.stochastic_depth_masks(net._net.features, xs.shape[0], sdg)),
                  a.steps, a.warmup)
    net_t, opt_t = build(dev)
    torch_s = timed(lambda: torch_step(net_t, opt_t, xs1, xs2, ys), a.torch_steps, 1)
    imgs = 2 * a.batch
    del net_t, opt_t
    net_j, opt_j, opt_jn = build(dev, joint=True)
    joint_s = timed(lambda: T.hip_train_step(net_j, xs1, xs2, ys, opt_jn, opt_j, False, 1, 1, True, generator=sdg),
                    a.steps, a.warmup)
    del net_j, opt_j, opt_jn
    torch.cuda.empty_cache()
    net_jt, opt_jt, opt_jtn = build(dev, joint=True)
    joint_t = timed(lambda: torch_joint_step(net_jt, opt_jt, opt_jtn, xs1, xs2, ys), a.torch_steps, 1)
    print(json.dumps({
        "metric": "joint-phase iteration images/sec (ConvNeXt-tiny-26 PIP-Net, 224x224, features.6-7 + classifier)",
        "images_per_iteration": imgs, "hip_images_per_sec": imgs / joint_s, "hip_ms_per_iter": joint_s * 1e3,
        "torch_images_per_sec": imgs / joint_t, "torch_ms_per_iter": joint_t * 1e3,
        "speedup_vs_torch_path": joint_t / joint_s}), flush=True)
    print(json.dumps({
        "metric": "finetune iteration images/sec (ConvNeXt-tiny-26 PIP-Net, 224x224, classifier-only)",
        "images_per_iteration": imgs, "hip_images_per_sec": imgs / hip_s, "hip_ms_per_iter": hip_s * 1e3,
        "hip_forward_ms": fwd_s * 1e3, "hip_loss_backward_optimizer_ms": (hip_s - fwd_s) * 1e3,
        "torch_images_per_sec": imgs / torch_s, "torch_ms_per_iter": torch_s * 1e3,
        "speedup_vs_torch_path": torch_s / hip_s}), flush=True)


if __name__ == "__main__":
    main()
