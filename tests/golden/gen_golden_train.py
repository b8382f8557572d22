"""Golden fixtures for the finetune-phase training iteration, recorded
by running the REFERENCE's own ``pipnet/train.py:train_pipnet`` (unchanged) on CPU with
``finetune=True`` for a few iterations.

Setup mirrors main.py: the net of a forward golden case (gen_golden.CASES, same synthetic
weights) in ``nn.DataParallel`` (CPU: calls the module directly), optimizers from the
reference's ``util/args.py:get_optimizer_nn`` (AdamW; lr 0.05, weight decay 0.01 on the
classifier weight), the finetune freeze of main.py:333-345 (only ``_classification``
trains), ``CosineAnnealingWarmRestarts(T_0=10, eta_min=0.001)`` as main.py:314,
``NLLLoss``, ``enforce_weight_sparsity=True``.

Stochastic depth: ``torch.Tensor.bernoulli_`` is patched to emit ``synth_bernoulli``
masks (recorded).  They are drawn with keep probability min(1 - p, 0.75) so that drops
actually occur in a few-iteration fixture; the branch scale is still the module's own
1/(1 - p), so the masks are simply an input of the step.

Recorded per iteration i: labels, the SD masks (one per CNBlock with p > 0, in forward
order), the forward's ``pooled`` / ``out`` (forward hook), the proto map (small cases),
the classifier weight / bias / multiplier the forward saw, the loss components and
accuracy ``calculate_loss`` returned; at the end: classifier weight / bias / multiplier,
AdamW state and ``train_info``.

Usage:  python tests/golden/gen_golden_train.py
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys

sys.dont_write_bytecode = True            # /root/reference is read-only
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

import gen_golden as G  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from golden_util import train_loader_batches  # noqa: E402
from count_pipnet_amd.synthetic import synth_bernoulli  # noqa: E402

# name -> (forward golden case, iterations, batch per view, seed, record proto map, phase)
# phase: "finetune" (main.py:333-345), "joint" (the "train + freeze params" epochs,
# main.py:377-390) or "pretrain" (main.py:238-256)
TRAIN_CASES = {
    "train_finetune_mid_addon": ("pipnet_mid_addon", 3, 3, 301, True, "finetune"),
    "train_finetune_c2": ("c2_pipnet_convnext26", 2, 2, 302, False, "finetune"),
    "train_joint_mid_addon": ("pipnet_mid_addon", 3, 3, 303, True, "joint"),
    "train_pretrain_mid_addon": ("pipnet_mid_addon", 2, 3, 304, True, "pretrain"),
    "train_joint_c2": ("c2_pipnet_convnext26", 2, 2, 305, False, "joint"),
    # CountPIPNet finetune (main.py:333-343: classifier + intermediate train; train_intermediate
    # puts the intermediate into the classifier optimizer, util/args.py:318-321); soft Gumbel
    # noise injected as in gen_golden (synth_exponential, seeds noise_seed + k per forward)
    "train_count_finetune_onehot": ("count_onehot", 3, 3, 306, True, "count_finetune"),
    "train_count_finetune_bilinear": ("count_bilinear_small", 3, 2, 307, True, "count_finetune"),
    # CountPIPNet pretrain / joint (main.py:238-256, 360-390): the mid-layer suffix + add-on
    # (+ classifier + intermediate in the joint phase) train; backward through the soft Gumbel
    # head, STE round / ClampSTE and the intermediate layer (ModifiedSTE for one-hot)
    "train_count_pretrain_onehot": ("count_onehot", 2, 3, 308, True, "count_pretrain"),
    "train_count_joint_onehot": ("count_onehot", 3, 3, 309, True, "count_joint"),
    "train_count_joint_identity": ("c1_count_identity", 2, 3, 310, True, "count_joint"),
    "train_count_joint_linear_full": ("count_linear_full", 2, 3, 311, True, "count_joint"),
    "train_count_joint_bilinear": ("count_bilinear_small", 2, 2, 312, True, "count_joint"),
    # LinearIntermediate (Linear(1, max_count) per count): finetune and joint phases
    "train_count_finetune_linear": ("count_linear", 3, 3, 316, True, "count_finetune"),
    "train_count_joint_linear": ("count_linear", 2, 3, 317, True, "count_joint"),
    # "train everything" epochs (main.py:362-373, epoch > freeze_epochs): the whole backbone,
    # stem included, + add-on + classifier (+ intermediate) train
    "train_full_mid_addon": ("pipnet_mid_addon", 2, 3, 313, True, "full"),
    "train_full_c2": ("c2_pipnet_convnext26", 2, 2, 314, False, "full"),
    "train_count_full_onehot": ("count_onehot", 2, 3, 315, True, "count_full"),
    # ResNet-50 (util/args.py:280-290 groups; every BatchNorm2d in train mode, running
    # statistics recorded): finetune, pretrain, "train + freeze params" (layer3 / layer4) and
    # "train everything" (layer2 too; the stem and layer1 never train)
    "train_finetune_resnet50": ("pipnet_resnet50_small", 2, 2, 320, False, "finetune"),
    "train_pretrain_resnet50": ("pipnet_resnet50_small", 2, 2, 321, False, "pretrain"),
    "train_joint_resnet50": ("pipnet_resnet50_small", 2, 2, 322, False, "joint"),
    "train_full_resnet50": ("pipnet_resnet50_small", 2, 2, 323, False, "full"),
}
LR, WD = 0.05, 0.01


@contextlib.contextmanager
def injected_bernoulli(seed: int):
    orig = torch.Tensor.bernoulli_
    drawn = []

    def fake(self, p=0.5, *, generator=None):
        mask = synth_bernoulli(tuple(self.shape), min(float(p), 0.75), seed + len(drawn))
        drawn.append(mask.flatten().clone())
        with torch.no_grad():
            self.copy_(mask)
        return self

    torch.Tensor.bernoulli_ = fake
    try:
        yield drawn
    finally:
        torch.Tensor.bernoulli_ = orig


def run(name):
    fwd_case, nb, bs, seed, keep_proto, phase = TRAIN_CASES[name]
    net, case = G.build_reference(fwd_case)
    sys.path.insert(0, G.REF)
    import pipnet.train as ref_train
    from util.args import get_optimizer_nn
    dp = nn.DataParallel(net)
    count = phase.startswith("count_")
    base = phase[len("count_"):] if count else phase            # finetune / joint / pretrain
    args = argparse.Namespace(net=case["net"], use_mid_layers=case.get("use_mid_layers", False),
                              num_stages=case.get("num_stages", 2), bias=case["bias"], lr=LR, lr_net=5e-4,
                              lr_block=5e-4, weight_decay=WD, optimizer="Adam", seed=1, train_intermediate=count)
    with contextlib.redirect_stdout(io.StringIO()):
        opt_net, opt_cls, to_freeze, to_train, backbone = get_optimizer_nn(dp, args)
    for p in net.parameters():                       # main.py:335-339 (finetune)
        p.requires_grad = False
    for p in net._classification.parameters():
        p.requires_grad = base != "pretrain"
    if count and getattr(net, "_intermediate", None) is not None:     # main.py:341-343, 251-253, 386-388
        for p in net._intermediate.parameters():
            p.requires_grad = base != "pretrain"
    if base != "finetune":                           # main.py:240-249 / 377-385
        for group in (to_train, to_freeze, list(net._add_on.parameters())):
            for p in group:
                p.requires_grad = True
    if base == "full":                               # main.py:362-373
        for p in backbone:
            p.requires_grad = True
    net._classification.normalization_multiplier.requires_grad = False
    sched_net = torch.optim.lr_scheduler.CosineAnnealingLR(opt_net, T_max=10, eta_min=5e-6)
    sched_cls = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(opt_cls, T_0=10, eta_min=0.001, T_mult=1)
    criterion = nn.NLLLoss(reduction="mean")
    batches = train_loader_batches(case["size"], case["num_classes"], nb, bs, seed)

    seen, comps = [], []

    def hook(mod, inp, outp):
        cls = mod._classification
        seen.append(dict(pooled=outp[1].detach().clone(), out=outp[2].detach().clone(),
                         proto=outp[0].detach().clone() if keep_proto else None,
                         w=cls.weight.detach().clone(),
                         b=None if cls.bias is None else cls.bias.detach().clone(),
                         mult=cls.normalization_multiplier.detach().clone()))

    orig_loss = ref_train.calculate_loss

    def rec_loss(*a, **kw):
        loss, acc, comp = orig_loss(*a, **kw)
        comps.append(dict(comp, acc=acc, loss=float(loss.item())))
        return loss, acc, comp

    ref_train.calculate_loss = rec_loss
    # every iteration's gradients as the optimizers see them (first 256 values per tensor;
    # 2048 of the classifier weight): the tests derive per-element AdamW step tolerances
    # from them (an element whose gradient is decisive in every step must follow the
    # reference's trajectory closely, one whose gradient is near zero may flip its sign-like
    # step)
    grads = {"net": [], "cls": []}

    def recording(opt, key, limit):
        orig = opt.step

        def step(*a, **kw):
            mine = {id(q) for g in opt.param_groups for q in g["params"]}
            grads[key].append({n: p.grad.detach().flatten()[:limit].clone() for n, p in net.named_parameters()
                               if p.grad is not None and p.requires_grad and id(p) in mine})
            return orig(*a, **kw)
        opt.step = step
        return orig

    orig_net_step = recording(opt_net, "net", 256)
    orig_cls_step = recording(opt_cls, "cls", 2048)
    h = net.register_forward_hook(hook)
    try:
        with injected_bernoulli(seed=5000 + seed) as drawn, G.injected_exponential(seed=7000 + seed) as noise, \
                contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            info = ref_train.train_pipnet(dp, batches, opt_net, opt_cls,
                                          sched_net, None if base == "pretrain" else sched_cls, criterion,
                                          1, 2 if base == "pretrain" else 1, torch.device("cpu"),
                                          is_count_pipnet=count, pretrain=base == "pretrain",
                                          finetune=base == "finetune",
                                          enforce_weight_sparsity=True)
    finally:
        h.remove()
        ref_train.calculate_loss = orig_loss
        opt_net.step, opt_cls.step = orig_net_step, orig_cls_step
    nmask = len(drawn) // nb
    rec = {}

    def put(key, t):
        """Full tensors for small cases; for the C2-sized head: first 8 rows + row sums."""
        a = t.detach().numpy()
        if keep_proto or a.ndim < 2:
            rec[key] = a
        else:
            rec[key + "_rows8"] = a[:8]
            rec[key + "_rowsum"] = a.astype(np.float64).sum(axis=1)
    for i, ((xs1, xs2, ys), s) in enumerate(zip(batches, seen)):
        rec[f"s{i}_ys"] = ys.numpy()
        rec[f"s{i}_masks"] = (torch.stack(drawn[i * nmask:(i + 1) * nmask]).numpy() if nmask
                              else np.zeros((0, 2 * bs), dtype=np.float32))
        for k in ("pooled", "out", "b", "mult", "proto"):
            if s[k] is not None:
                rec[f"s{i}_{k}"] = s[k].numpy()
        if keep_proto:
            rec[f"s{i}_w"] = s["w"].numpy()
    if count:                    # the trained intermediate tensors, in full (small cases)
        for pname, prm in net._intermediate.named_parameters():
            rec[f"inter/{pname}"] = prm.detach().numpy()
    if base != "finetune":       # every trainable backbone / add-on tensor
        for pname, prm in net.named_parameters():
            if prm.requires_grad and not pname.startswith("_classification"):
                a = prm.detach().double()
                rec[f"param/{pname}/sum"] = np.array(float(a.sum()))
                rec[f"param/{pname}/abs"] = np.array(float(a.abs().sum()))
                rec[f"param/{pname}/head"] = prm.detach().flatten()[:256].numpy()
                st_p = opt_net.state.get(prm, {})
                if "exp_avg_sq" in st_p:
                    rec[f"param/{pname}/v_head"] = st_p["exp_avg_sq"].flatten()[:256].numpy()
    for key in ("net", "cls"):
        for i, gd in enumerate(grads[key]):
            for pname, g in gd.items():
                rec[f"grad{i}/{pname}"] = g.numpy()
    for bname, buf in net.named_buffers():          # BatchNorm running statistics (ResNet)
        if bname.endswith(("running_mean", "running_var")):
            a = buf.detach().double()
            rec[f"buffer/{bname}/sum"] = np.array(float(a.sum()))
            rec[f"buffer/{bname}/abs"] = np.array(float(a.abs().sum()))
            rec[f"buffer/{bname}/head"] = buf.detach().flatten()[:64].numpy()
        elif bname.endswith("num_batches_tracked"):
            rec[f"buffer/{bname}"] = buf.detach().numpy()
    cls = net._classification
    put("final_w", cls.weight)
    rec["final_mult"] = cls.normalization_multiplier.detach().numpy()
    st = opt_cls.state.get(cls.weight, {"exp_avg": torch.zeros_like(cls.weight),
                                         "exp_avg_sq": torch.zeros_like(cls.weight), "step": 0.0})
    put("final_w_exp_avg", st["exp_avg"])
    put("final_w_exp_avg_sq", st["exp_avg_sq"])
    if cls.bias is not None and cls.bias in opt_cls.state:
        rec["final_b"] = cls.bias.detach().numpy()
        rec["final_b_exp_avg"] = opt_cls.state[cls.bias]["exp_avg"].numpy()
        rec["final_b_exp_avg_sq"] = opt_cls.state[cls.bias]["exp_avg_sq"].numpy()
    meta = dict(name=name, forward_case=fwd_case, phase=phase, iterations=nb, batch_per_view=bs, seed=seed,
                lr_net=5e-4, lr_block=5e-4,
                mask_seed=5000 + seed, masks_per_step=nmask, lr=LR, weight_decay=WD,
                noise_seed=7000 + seed, noise_draws=len(noise),
                steps=float(st["step"]), components=comps,
                info={k: (v if isinstance(v, list) else float(v)) for k, v in info.items()},
                torch=torch.__version__)
    rec["meta"] = np.array(json.dumps(meta))
    return rec


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    only = sys.argv[1:]
    for name in TRAIN_CASES:
        if only and name not in only:
            continue
        rec = run(name)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **rec)
        meta = json.loads(str(rec["meta"]))
        print(f"wrote {path} ({os.path.getsize(path) / 1e3:.1f} kB)", meta["components"], flush=True)


if __name__ == "__main__":
    main()
