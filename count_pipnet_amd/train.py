"""Finetune-phase PIP-Net training iteration on the MI355X kernels (SURVEY.md 8f rank 4,
first slice).

The reference trains with ``pipnet/train.py:train_pipnet`` (train.py:8-150).  In its
finetune phase (main.py:333-345) only the classification layer trains, so one iteration is:
forward of cat([xs1, xs2]) in train mode -> ``calculate_loss`` (train.py:154-250, loss =
2 * class loss; the align / tanh terms are computed for logging) -> backward into the
NonNegLinear weight / bias -> ``optimizer_classifier.step()`` (AdamW, util/args.py:327)
-> scheduler -> the sparsity clamps (train.py:134-140).  Here that iteration is:

  * forward: the same HIP backbone / head as inference, plus torchvision's row stochastic
    depth -- a dropped sample skips the block's branch outright
    (``convnext_features._cnblock_hip``); pooled is not thresholded (inference=False);
  * ``kernels.train_loss`` (csrc/train_ops.hip): align / tanh / class terms, correct count
    and d loss / d out in two launches (the align term reads the proto map once);
  * ``kernels.nonneg_linear_backward`` and ``kernels.adamw_step_`` (AdamW fused with the
    clamps), updating the torch optimizer's own ``state`` tensors (``step``, ``exp_avg``,
    ``exp_avg_sq``) so optimizer, scheduler and their ``state_dict``s stay interchangeable
    with the reference's.

No host synchronisation inside the loop (the reference reads five ``.item()`` per
iteration): loss terms and accuracy accumulate on the device and are read once per epoch.
Stochastic-depth masks come from a host ``torch.Generator`` (the reference draws them with
the device RNG: same distribution, different stream -- RNG parity unpinned; the tests
inject the masks recorded from the reference).

Other phases (pretrain, joint training) need backbone gradients: this package's modules
run them on the torch autograd path under the reference's own ``train_pipnet`` (forward
dispatches to torch whenever grad is enabled); HIP backward kernels for the trainable
ConvNeXt stages are the next slice.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from . import kernels as K
from .convnext_features import CNBlock, ConvNeXt, MidLayerConvNeXt, convnext_features_hip

# (align, tanh, class) loss weights of the non-pretrain phases (train.py:56-61)
FINETUNE_LOSS_WEIGHTS = (5.0, 2.0, 2.0)
SPARSITY_DELTA = 1e-3          # train.py:135: W <- max(W - 1e-3, 0) after every step


def _inner(net: nn.Module) -> nn.Module:
    return getattr(net, "module", net)


def stochastic_depth_masks(features: nn.Sequential, batch: int,
                           generator: Optional[torch.Generator] = None) -> Dict[int, Tensor]:
    """Host keep masks (bool [batch]) for every CNBlock with p > 0, keyed by block id in
    module order: StochasticDepth("row") keeps a sample's branch with probability 1 - p."""
    masks: Dict[int, Tensor] = {}
    blocks = [b for mod in features if isinstance(mod, nn.Sequential) for b in mod if isinstance(b, CNBlock)]
    for bid, blk in enumerate(blocks):
        if blk.stochastic_depth.p > 0.0:
            masks[bid] = torch.rand(batch, generator=generator) >= blk.stochastic_depth.p
    return masks


def hip_finetune_supported(net: nn.Module) -> bool:
    """True when the finetune iteration runs on the HIP kernels: a PIP-Net (not Count)
    with a ConvNeXt backbone, fp32 on a ROCm device, only classifier parameters trainable."""
    m = _inner(net)
    if hasattr(m, "_max_count") or not hasattr(m, "_classification"):
        return False
    if not isinstance(m._net, (ConvNeXt, MidLayerConvNeXt)):
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 for p in m.parameters()):
        return False
    cls = m._classification
    allowed = {id(cls.weight)} | ({id(cls.bias)} if cls.bias is not None else set())
    return {id(p) for p in m.parameters() if p.requires_grad} <= allowed


def train_forward_hip(net: nn.Module, xs: Tensor, sd_keep: Optional[Dict[int, Tensor]]):
    """PIPNet.forward(xs, inference=False) with train-mode stochastic depth on the HIP
    kernels: (proto NHWC [B,h,w,P], pooled [B,P], out [B,K])."""
    from .pipnet import add_on_logits_hip
    m = _inner(net)
    with torch.no_grad():
        feats = convnext_features_hip(m._net.features, xs, m._net._hip_pack, sd_keep)
        proto, pooled = K.softmax_pool(add_on_logits_hip(m._add_on, feats), pool_mode=0)
        _, out = K.nonneg_linear(pooled, m._classification.weight, m._classification.bias, None)
    return proto, pooled, out


def _group_of(optimizer: torch.optim.Optimizer, param: Tensor) -> Optional[dict]:
    for g in optimizer.param_groups:
        if any(p is param for p in g["params"]):
            return g
    return None


def hip_adamw_step(optimizer: torch.optim.Optimizer, param: Tensor, grad: Tensor,
                   post: Optional[Tuple[float, float]] = None) -> bool:
    """``optimizer.step()`` restricted to ``param`` with torch.optim.AdamW's math, on the
    device; state tensors are created exactly as AdamW's ``_init_group`` does (CPU float32
    ``step``).  Returns False when ``param`` is not in any group (nothing to do)."""
    if not isinstance(optimizer, torch.optim.AdamW):
        raise RuntimeError(f"HIP finetune step implements torch.optim.AdamW, got {type(optimizer).__name__}")
    g = _group_of(optimizer, param)
    if g is None:
        return False
    if g.get("amsgrad", False) or g.get("maximize", False) or g.get("capturable", False):
        raise RuntimeError("HIP AdamW step: amsgrad / maximize / capturable groups are not supported")
    st = optimizer.state[param]
    if not st:
        st["step"] = torch.tensor(0.0, dtype=torch.float32)
        st["exp_avg"] = torch.zeros_like(param, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(param, memory_format=torch.preserve_format)
    st["step"] += 1
    beta1, beta2 = g["betas"]
    K.adamw_step_(param.data, grad, st["exp_avg"], st["exp_avg_sq"], float(g["lr"]), beta1, beta2,
                  float(g["eps"]), float(g["weight_decay"]), int(st["step"].item()), post)
    return True


def hip_finetune_step(net: nn.Module, xs1: Tensor, xs2: Tensor, ys: Tensor,
                      optimizer_classifier: torch.optim.Optimizer, enforce_weight_sparsity: bool = True,
                      sd_keep: Optional[Dict[int, Tensor]] = None,
                      generator: Optional[torch.Generator] = None) -> Tensor:
    """One finetune iteration on the device (no host sync).  Returns ``kernels.train_loss``'s
    stats: [align, tanh, class, loss, correct, w_align, w_tanh, w_class]."""
    m = _inner(net)
    cls = m._classification
    xs = torch.cat([xs1, xs2])
    if sd_keep is None:
        sd_keep = stochastic_depth_masks(m._net.features, xs.shape[0], generator)
    proto, pooled, out = train_forward_hip(m, xs, sd_keep)
    w_align, w_tanh, w_class = FINETUNE_LOSS_WEIGHTS
    with torch.no_grad():
        stats, d_out = K.train_loss(proto, pooled, out, ys, cls.normalization_multiplier, enforce_weight_sparsity,
                                    1.0, w_align, w_tanh, w_class, "finetune")
        train_b = cls.bias is not None and cls.bias.requires_grad
        dw, db = K.nonneg_linear_backward(d_out, pooled, cls.weight, train_b)
        clamp_w = (SPARSITY_DELTA, 0.0) if enforce_weight_sparsity else None
        clamp_b = (0.0, 0.0) if enforce_weight_sparsity else None
        stepped_w = stepped_b = False
        if cls.weight.requires_grad:
            cls.weight.grad = dw
            stepped_w = hip_adamw_step(optimizer_classifier, cls.weight, dw, clamp_w)
        if train_b:
            cls.bias.grad = db
            stepped_b = hip_adamw_step(optimizer_classifier, cls.bias, db, clamp_b)
        if enforce_weight_sparsity:          # the clamps of parameters the optimizer did not touch
            if not stepped_w:
                K.weight_sparsify_(cls.weight.data, SPARSITY_DELTA)
            if cls.bias is not None and not stepped_b:
                K.clamp_min_(cls.bias.data, 0.0)
            K.clamp_min_(cls.normalization_multiplier.data, 1.0)
    return stats


class FinetuneEpoch:
    """Runs finetune iterations back to back with all bookkeeping on the device.

    Per batch (view-1 images, view-2 images, labels): ``hip_finetune_step``, then the
    classifier LR schedule is advanced to the fractional epoch position of the next batch
    (CosineAnnealingWarmRestarts is stepped with a float epoch in the reference,
    train.py:120).  The five running sums (align, tanh, class, loss, accuracy) live in one
    device vector; ``summary()`` is the single host read."""

    TERMS = ("align", "tanh", "class")

    def __init__(self, net: nn.Module, optimizer: torch.optim.Optimizer, enforce_weight_sparsity: bool = True,
                 generator: Optional[torch.Generator] = None):
        self.net, self.optimizer = net, optimizer
        self.enforce = enforce_weight_sparsity
        self.generator = generator
        self.sums: Optional[Tensor] = None
        self.count = 0
        self.lrs: list = []

    def add(self, stats: Tensor, labels: int) -> None:
        acc = stats[4:5] / float(2 * labels)
        row = torch.cat([stats[:4], acc]).double()
        self.sums = row if self.sums is None else self.sums.add_(row)
        self.count += 1

    def run(self, batches, scheduler, epoch: int, device, extra_optimizers=()) -> None:
        n_batches = len(batches)
        for pos, batch in enumerate(batches):
            a, b, labels = (t.to(device, non_blocking=True) for t in batch)
            for opt in (self.optimizer, *extra_optimizers):
                opt.zero_grad(set_to_none=True)
            self.add(hip_finetune_step(self.net, a, b, labels, self.optimizer, self.enforce,
                                       generator=self.generator), labels.shape[0])
            scheduler.step((epoch - 1) + pos / n_batches)
            self.lrs.append(scheduler.get_last_lr()[0])

    def summary(self) -> dict:
        vals = self.sums.cpu().tolist() if self.sums is not None else [0.0] * 5
        n = float(max(self.count, 1))
        info = {}
        for j, term in enumerate(self.TERMS):
            info[f"{term}_loss_raw"] = vals[j] / n
            info[f"{term}_loss_weighted"] = vals[j] / n * FINETUNE_LOSS_WEIGHTS[j]
        info.update(train_accuracy=vals[4] / n, loss=vals[3] / n, lrs_net=[0.0] * self.count,
                    lrs_class=list(self.lrs))
        return info


def train_pipnet(net, train_loader, optimizer_net, optimizer_classifier, scheduler_net, scheduler_classifier,
                 criterion, epoch, nr_epochs, device, is_count_pipnet=False, pretrain=False, finetune=False,
                 progress_prefix: str = "Train Epoch", enforce_weight_sparsity=True, tanh_loss_coeff=1.0,
                 generator: Optional[torch.Generator] = None, verbose: bool = False) -> dict:
    """Drop-in for train.py:8-150 in the finetune phase (same arguments, same ``train_info``
    keys; progress output reduced to one optional line).  Other phases raise: run the
    reference's own loop on this package's modules (torch autograd path)."""
    if pretrain or not finetune or is_count_pipnet or not hip_finetune_supported(net):
        raise NotImplementedError(
            "count_pipnet_amd.train_pipnet runs the finetune phase of a ConvNeXt PIP-Net on the HIP kernels; "
            "for other phases use the reference train_pipnet with these modules (torch autograd path)")
    net.train()
    _inner(net)._classification.requires_grad = True
    runner = FinetuneEpoch(net, optimizer_classifier, enforce_weight_sparsity, generator)
    extra = (optimizer_net,) if optimizer_net is not None and optimizer_net is not optimizer_classifier else ()
    runner.run(train_loader, scheduler_classifier, epoch, device, extra)
    info = runner.summary()
    if verbose:
        terms = ", ".join(f"{t}={info[t + '_loss_raw']:.4f}" for t in FinetuneEpoch.TERMS)
        print(f"[{progress_prefix} {epoch}] finetune on HIP: {runner.count} iterations, {terms}", flush=True)
    return info
