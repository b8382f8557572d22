"""Conditioning probe for ResNet-50 backbone gradients in fp32 (ResNet-50 training).

Train-mode forward of the ResNet-50 PIP-Net fixture's backbone (tests/golden
pipnet_resnet50_small, layer3-4 trainable) on the HIP kernels, backward of a fixed random
d-features, and the same through torch's own fp32 and fp64 autograd; prints the forward error
and the median / max over parameters of max|g - g64| / max|g64| for HIP and torch fp32.

    SIZE=64 NB=4 [PROFILE=init] python tools/resnet_grad_conditioning.py
"""
import sys, copy
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
from golden_util import load_train_golden, train_loader_batches
from model_util import build_model
from count_pipnet_amd import resnet_train as R
from count_pipnet_amd.backend import torch_backend
gpu = torch.device("cuda:0")
meta, rec, fwd_meta = load_train_golden("train_joint_resnet50")
net = build_model(fwd_meta).to(gpu).train()
c = fwd_meta["case"]
xs1, xs2, ys = train_loader_batches(c["size"], c["num_classes"], 1, meta["batch_per_view"], meta["seed"])[0]
import os
size = int(os.environ.get("SIZE", "64")); nb = int(os.environ.get("NB", "4"))
if os.environ.get("PROFILE"):
    from count_pipnet_amd.synthetic import fill_module_
    fill_module_(net, 32, os.environ["PROFILE"])
xs = torch.randn(nb, 3, size, size, generator=torch.Generator().manual_seed(5)).to(gpu)
for p in net.parameters():
    p.requires_grad = False
for n, p in net._net.named_parameters():
    if "layer3" in n or "layer4" in n:
        p.requires_grad = True
bb = net._net
start = R.trainable_start(bb)
feats, saved = R.train_forward(bb, xs, start)
g = torch.Generator().manual_seed(0)
dfeat = torch.randn(feats.shape, generator=g).to(gpu)
R.backward(bb, saved, dfeat)
hip = {n: p.grad.clone() for n, p in bb.named_parameters() if p.grad is not None}
outs = {}
for tag, dt in (("t32", torch.float32), ("t64", torch.float64)):
    m = copy.deepcopy(bb).to(dt)
    for p in m.parameters():
        p.grad = None
    with torch_backend():
        f = m(xs.to(dt))
    f.backward(dfeat.permute(0, 3, 1, 2).to(dt))
    outs[tag] = (f.detach().permute(0, 2, 3, 1), {n: p.grad for n, p in m.named_parameters() if p.grad is not None})
f64 = outs["t64"][0]
sc = f64.abs().max().item()
print("features: hip", (feats.double() - f64).abs().max().item() / sc, "t32", (outs["t32"][0].double() - f64).abs().max().item() / sc)
errs_h, errs_t = [], []
for n in hip:
    c64 = outs["t64"][1][n]
    s = c64.abs().max().item() + 1e-30
    errs_h.append((hip[n].double() - c64).abs().max().item() / s)
    errs_t.append((outs['t32'][1][n].double() - c64).abs().max().item() / s)
import statistics
print("SIZE", size, "NB", nb, "PROFILE", os.environ.get("PROFILE"), "median hip", statistics.median(errs_h), "max hip", max(errs_h),
      "median t32", statistics.median(errs_t), "max t32", max(errs_t))
raise SystemExit(0)
for n in hip:
    c64 = outs["t64"][1][n]
    s = c64.abs().max().item() + 1e-30
    print(f"{n:40s} hip {(hip[n].double() - c64).abs().max().item() / s:.3g}  t32 {(outs['t32'][1][n].double() - c64).abs().max().item() / s:.3g}")
