"""PIP-Net / CountPIPNet training iterations on the MI355X kernels.

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

The pretrain / joint / "train everything" phases backpropagate into a trainable backbone
suffix on the same kernels: ConvNeXt CNBlocks / downsamples / stem (``_forward_saving``,
``_block_backward``) and the ResNet-50 Bottlenecks with train-mode BatchNorm
(``resnet_train``; every BN of the backbone, frozen ones included, normalises with batch
statistics and updates its running statistics, as under the reference's ``net.train()``).
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


def _is_resnet(m: nn.Module) -> bool:
    from .resnet_features import ResNet_features
    return isinstance(getattr(m, "_net", None), ResNet_features)


def _backbone_ok(m: nn.Module) -> bool:
    """A backbone with a HIP train-mode forward: ConvNeXt (full or mid-layer) or a Bottleneck
    ResNet with the stem frozen (resnet_train.supported)."""
    if isinstance(getattr(m, "_net", None), (ConvNeXt, MidLayerConvNeXt)):
        return True
    if _is_resnet(m):
        from . import resnet_train
        return resnet_train.supported(m._net)
    return False


def _sd_masks(m: nn.Module, batch: int, generator: Optional[torch.Generator]) -> Dict[int, Tensor]:
    """Stochastic-depth keep masks of the backbone (ResNets have none)."""
    if _is_resnet(m):
        return {}
    return stochastic_depth_masks(m._net.features, batch, generator)


def _backbone_train_forward(m: nn.Module, xs: Tensor, sd_keep: Dict[int, Tensor]) -> Tensor:
    """Train-mode backbone forward without kept activations -> NHWC features."""
    if _is_resnet(m):
        from . import resnet_train
        return resnet_train.train_forward(m._net, xs, None)[0]
    return convnext_features_hip(m._net.features, xs, m._net._hip_pack, sd_keep)


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
    if not _backbone_ok(m):
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 for p in m.parameters()):
        return False
    cls = m._classification
    allowed = {id(cls.weight)} | ({id(cls.bias)} if cls.bias is not None else set())
    return {id(p) for p in m.parameters() if p.requires_grad} <= allowed


def train_forward_hip(net: nn.Module, xs: Tensor, sd_keep: Optional[Dict[int, Tensor]],
                      update_bn_stats: bool = True):
    """PIPNet.forward(xs, inference=False) with train-mode stochastic depth on the HIP
    kernels: (proto NHWC [B,h,w,P], pooled [B,P], out [B,K]).  Like the module's own forward
    under ``net.train()``, a ResNet backbone's BatchNorms normalise with batch statistics and
    take the running-statistics update; ``update_bn_stats=False`` restores every running
    statistic and counter afterwards (an observer forward that must not advance them)."""
    from .pipnet import add_on_logits_hip
    m = _inner(net)
    saved = None
    if not update_bn_stats:
        saved = [(b, b.clone()) for b in m._net.buffers()]
    with torch.no_grad():
        try:
            feats = _backbone_train_forward(m, xs, sd_keep)
        finally:
            for b, v in saved or ():
                b.copy_(v)
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
    K.adamw_step_(param.detach(), grad, st["exp_avg"], st["exp_avg_sq"], float(g["lr"]), beta1, beta2,
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
        sd_keep = _sd_masks(m, xs.shape[0], generator)
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
                K.weight_sparsify_(cls.weight.detach(), SPARSITY_DELTA)
            if cls.bias is not None and not stepped_b:
                K.clamp_min_(cls.bias.detach(), 0.0)
            K.clamp_min_(cls.normalization_multiplier.detach(), 1.0)
    return stats


# ------------------------------------------------------------------------------------------
# CountPIPNet finetune phase (main.py:333-343): classifier + intermediate layer train
# ------------------------------------------------------------------------------------------
def hip_count_finetune_supported(net: nn.Module) -> bool:
    """A ConvNeXt CountPIPNet (fp32, ROCm) whose trainable parameters are within the
    classifier and an intermediate layer with a HIP backward (identity, one-hot, linear_full,
    bilinear)."""
    from .count_pipnet_utils import (BilinearIntermediate, IdentityIntermediate, LinearFull, LinearIntermediate,
                                     OneHotEncoder)
    m = _inner(net)
    if not hasattr(m, "_max_count") or not _backbone_ok(m):
        return False
    if not isinstance(m._intermediate, (IdentityIntermediate, OneHotEncoder, LinearFull, LinearIntermediate,
                                       BilinearIntermediate)):
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 for p in m.parameters()):
        return False
    allowed = {id(p) for p in m._classification.parameters()} | {id(p) for p in m._intermediate.parameters()}
    return {id(p) for p in m.parameters() if p.requires_grad} <= allowed


def _count_train_forward(m: nn.Module, xs: Tensor, sd_keep: Dict[int, Tensor], j: Optional[int] = None):
    """CountPIPNet.forward(xs) in train mode (count_pipnet.py:70-110) on the HIP kernels, keeping
    what the backward needs: (proto NHWC, raw counts, clamped counts, intermediate activations
    dict, classifier input, out).  With ``j`` the backbone suffix features[j:] runs with its
    activations kept (``_forward_saving``); they and the features are added to the dict
    (``feats``, ``suffix``) together with the head's temperature (``tau``)."""
    from . import _lib
    from .count_pipnet_utils import BilinearIntermediate, GumbelSoftmax
    from .pipnet import add_on_logits_hip
    saved = {}
    if j is None:
        feats = _backbone_train_forward(m, xs, sd_keep)
    else:
        feats, saved["suffix"] = _backbone_forward_saving(m, xs, j, sd_keep)
        saved["feats"] = feats
    act = list(m._add_on)[-1] if isinstance(m._add_on, nn.Sequential) else m._add_on
    if isinstance(act, GumbelSoftmax):
        logits = add_on_logits_hip(m._add_on, feats, activation=GumbelSoftmax)
        noise = act.exp_noise
        if noise is not None:
            proto, sums = K.count_gumbel_soft(logits, act.tau, noise.to(device=logits.device,
                                                                        dtype=torch.float32).contiguous(), 0)
        else:
            seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())   # fresh noise per call
            proto, sums = K.count_gumbel_soft(logits, act.tau, None, seed)
        saved["tau"] = float(act.tau)
    else:
        logits = add_on_logits_hip(m._add_on, feats, activation=nn.Softmax)
        proto, sums = K.softmax_pool(logits, pool_mode=1)
        saved["tau"] = 1.0
    del logits
    # train mode: STE round in the forward only with use_ste (count_pipnet.py:90-97)
    counts, clamped = K.count_finish(None, sums, m._max_count, bool(m._use_ste))
    layer = m._intermediate
    if isinstance(layer, BilinearIntermediate):
        e = K.linear(clamped, layer.embed.weight)
        u = K.linear(e, layer.W.weight)
        v = K.linear(e, layer.V.weight)
        inter = torch.empty_like(u)
        K.linear(e, layer.V.weight, epilogue=_lib.EPI_MUL, r=u, out=inter)
        saved.update(e=e, u=u, v=v)
    else:
        from .count_pipnet import intermediate_hip
        inter = intermediate_hip(layer, clamped)
    _, out = K.nonneg_linear(inter, m._classification.weight, m._classification.bias, None)
    return proto, counts, clamped, saved, inter, out


def _intermediate_backward(layer: nn.Module, x: Tensor, saved: dict, d_inter: Tensor,
                           need_dx: bool = False) -> Optional[Tensor]:
    """Parameter gradients of the intermediate layer (count_pipnet_utils.py:323-539) and, with
    ``need_dx``, the gradient w.r.t. its input x (the clamped counts) -- None where no gradient
    flows (a OneHotEncoder without STE: create_modified_encoding is not differentiable)."""
    from . import _lib
    from .count_pipnet_utils import (BilinearIntermediate, IdentityIntermediate, LinearFull, LinearIntermediate,
                                     OneHotEncoder)
    if isinstance(layer, IdentityIntermediate):
        return d_inter if need_dx else None
    if isinstance(layer, OneHotEncoder):
        if not (need_dx and layer.use_ste):
            return None
        return K.onehot_ste_backward(x, d_inter, layer.positive_grad_strategy, layer.respect_active_grad)
    if isinstance(layer, LinearFull):
        w = layer.linear.weight
        if w.requires_grad:
            _set_grad(w, K.wgrad(d_inter, x))
        if layer.linear.bias is not None and layer.linear.bias.requires_grad:
            _set_grad(layer.linear.bias, K.colsum(d_inter))
        return K.linear(d_inter, w.detach().t().contiguous(), None, _lib.EPI_NONE) if need_dx else None
    if isinstance(layer, LinearIntermediate):
        w = layer.linear.weight
        if not (w.requires_grad or need_dx):
            return None
        dx, dw = K.linear_intermediate_backward(x, d_inter, w, want_dx=need_dx)
        if w.requires_grad:
            _set_grad(w, dw.view_as(w))
        return dx
    if isinstance(layer, BilinearIntermediate):
        e, u, v = saved["e"], saved["u"], saved["v"]
        du, dv = K.bilinear_bwd_prep(d_inter, u, v)
        if layer.W.weight.requires_grad:
            _set_grad(layer.W.weight, K.wgrad(du, e))
        if layer.V.weight.requires_grad:
            _set_grad(layer.V.weight, K.wgrad(dv, e))
        if not (layer.embed.weight.requires_grad or need_dx):
            return None
        de = K.linear(du, layer.W.weight.detach().t().contiguous())
        ones = torch.ones(de.shape[1], device=de.device)
        K.linear(dv, layer.V.weight.detach().t().contiguous(), None, _lib.EPI_RESID, scale=ones, r=de, out=de)
        if layer.embed.weight.requires_grad:
            _set_grad(layer.embed.weight, K.wgrad(de, x))
        return K.linear(de, layer.embed.weight.detach().t().contiguous(), None, _lib.EPI_NONE) if need_dx else None
    raise NotImplementedError(f"HIP count training: no backward for {type(layer).__name__}")


def hip_count_finetune_step(net: nn.Module, xs1: Tensor, xs2: Tensor, ys: Tensor,
                            optimizer_classifier: torch.optim.Optimizer, enforce_weight_sparsity: bool = True,
                            tanh_loss_coeff: float = 1.0, sd_keep: Optional[Dict[int, Tensor]] = None,
                            generator: Optional[torch.Generator] = None) -> Tensor:
    """One CountPIPNet finetune iteration (train.py:75-140 with finetune=True,
    is_count_pipnet=True): train-mode forward (soft Gumbel head, stochastic depth), the loss
    kernel (loss = 2 * class; align / tanh over C * raw counts for logging), backward into the
    classifier and the intermediate layer, AdamW for every parameter the classifier optimizer
    holds (intermediate included when ``train_intermediate`` put it there), the sparsity clamps.
    Returns the loss-kernel stats without synchronising."""
    m = _inner(net)
    cls = m._classification
    xs = torch.cat([xs1, xs2])
    if sd_keep is None:
        sd_keep = _sd_masks(m, xs.shape[0], generator)
    w_align, w_tanh, w_class = FINETUNE_LOSS_WEIGHTS
    with torch.no_grad():
        proto, counts, clamped, saved, inter, out = _count_train_forward(m, xs, sd_keep)
        stats, d_out = K.train_loss(proto, counts, out, ys, cls.normalization_multiplier, enforce_weight_sparsity,
                                    tanh_loss_coeff, w_align, w_tanh, w_class, "finetune")
        train_b = cls.bias is not None and cls.bias.requires_grad
        dw, db = K.nonneg_linear_backward(d_out, inter, cls.weight, train_b)
        if cls.weight.requires_grad:
            cls.weight.grad = dw
        if train_b:
            cls.bias.grad = db
        layer = m._intermediate
        if any(p.requires_grad for p in layer.parameters()):
            _intermediate_backward(layer, clamped, saved, K.nonneg_linear_dx(d_out, cls.weight.detach()))
        stepped = set()
        for g in optimizer_classifier.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                post = None
                if enforce_weight_sparsity:
                    post = (SPARSITY_DELTA, 0.0) if p is cls.weight else (0.0, 0.0) if p is cls.bias else None
                if hip_adamw_step(optimizer_classifier, p, p.grad, post):
                    stepped.add(id(p))
        if enforce_weight_sparsity:          # the clamps of parameters the optimizer did not touch
            if id(cls.weight) not in stepped:
                K.weight_sparsify_(cls.weight.detach(), SPARSITY_DELTA)
            if cls.bias is not None and id(cls.bias) not in stepped:
                K.clamp_min_(cls.bias.detach(), 0.0)
            K.clamp_min_(cls.normalization_multiplier.detach(), 1.0)
    return stats


# ------------------------------------------------------------------------------------------
# Pretrain / joint phases: a trainable backbone suffix + add-on (+ classifier) on the HIP
# kernels (main.py:238-256 pretrain, :377-390 "train + freeze params")
# ------------------------------------------------------------------------------------------
def _cnblocks(seq) -> list:
    return [b for mod in seq if isinstance(mod, nn.Sequential) for b in mod if isinstance(b, CNBlock)]


def trainable_suffix_start(net: nn.Module) -> int:
    """Index j of the first ``features`` entry (ConvNeXt) or residual block (ResNet) holding a
    trainable parameter (their count when the backbone is frozen).  Gradients flow through
    every entry from j on."""
    m = _inner(net)
    if _is_resnet(m):
        from . import resnet_train
        return resnet_train.trainable_start(m._net)
    for j, mod in enumerate(m._net.features):
        if any(p.requires_grad for p in mod.parameters()):
            return j
    return len(m._net.features)


def _backbone_units(m: nn.Module) -> int:
    if _is_resnet(m):
        from . import resnet_train
        return len(resnet_train._blocks(m._net))
    return len(m._net.features)


def _backbone_forward_saving(m: nn.Module, xs: Tensor, j: int, sd_keep: Dict[int, Tensor]):
    """Train-mode backbone forward keeping the activations of the trainable suffix from j."""
    if _is_resnet(m):
        from . import resnet_train
        feats, saved = resnet_train.train_forward(m._net, xs, j)
        return feats, [("resnet", None, None, saved)]
    return _forward_saving(m, xs, j, sd_keep)


def hip_train_supported(net: nn.Module) -> bool:
    """A ConvNeXt PIP-Net (fp32, ROCm) whose trainable backbone part is a suffix features[j:]
    (the reference's pretrain / "train + freeze params" phases; j = 0, the stem included: the
    "train everything" epochs after freeze_epochs, main.py:362-373)."""
    m = _inner(net)
    if hasattr(m, "_max_count") or not _backbone_ok(m):
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 for p in m.parameters()):
        return False
    return trainable_suffix_start(m) < _backbone_units(m)


def _forward_saving(m: nn.Module, xs: Tensor, j: int, sd_keep: Dict[int, Tensor]):
    """Train-mode forward; features[:j] on the inference executor, features[j:] with plain
    (unfused) kernels whose intermediates are kept: per CNBlock the input x, the depthwise
    output z, the LayerNorm output t, the Linear1 pre-activation h1, GELU output g and the
    Linear2 output y2; per downsample its input and LayerNorm output."""
    from . import _lib
    from .convnext_features import LayerNorm2d, packed, stochastic_depth_row_scales
    feats, cache = m._net.features, m._net._hip_pack
    saved = []
    if j == 0:       # trainable stem (the "train everything" epochs): conv k4 s4 and LN unfused
        conv, ln = feats[0][0], feats[0][1]
        if conv.kernel_size != (4, 4) or conv.stride != (4, 4) or conv.in_channels != 3 or conv.padding != (0, 0):
            raise RuntimeError(f"HIP training step: unsupported ConvNeXt stem {conv}")
        xp = K.nchw_to_nhwc(xs.contiguous(), 4)                     # channels zero-padded 3 -> 4
        wp = packed(cache, "0.conv.train", conv.weight,
                    lambda w: torch.nn.functional.pad(w.permute(0, 2, 3, 1), (0, 1)))
        z = K.conv2d_nhwc(xp, wp, conv.bias, 4, 0, _lib.EPI_BIAS)
        h = K.layernorm(z, ln.weight, ln.bias)
        saved.append(("stem", feats[0], "0", dict(x=xp, z=z)))
        start = 1
    else:
        h = convnext_features_hip(feats[:j], xs, cache, sd_keep)
        start = j
    scales = stochastic_depth_row_scales(feats, sd_keep, xs.shape[0], xs.device)
    bid = len(_cnblocks(feats[:start]))
    for idx in range(start, len(feats)):
        mod = feats[idx]
        if len(mod) > 0 and isinstance(mod[0], CNBlock):
            for jb, blk in enumerate(mod):
                dw, ln, l1, l2 = blk.block[0], blk.block[2], blk.block[3], blk.block[5]
                b, hh, ww, c = h.shape
                key = f"{idx}.{jb}"
                wdw = packed(cache, key + ".dw", dw.weight, lambda w: w.reshape(c, 49).t())
                z = K.dwconv7_plain(h, wdw, dw.bias)
                t = K.layernorm(z, ln.weight, ln.bias)
                h1 = K.linear(t.view(-1, c), l1.weight, l1.bias, _lib.EPI_BIAS)
                g = K.gelu_fwd(h1)
                y2 = K.linear(g, l2.weight, l2.bias, _lib.EPI_BIAS)
                rs = scales.get(bid) if blk.stochastic_depth.p > 0.0 else None
                out = K.resid_scale(h.view(-1, c), y2, blk.layer_scale.view(-1), rs, hh * ww).view(b, hh, ww, c)
                saved.append(("block", blk, key, dict(x=h, z=z, t=t, h1=h1, g=g, y2=y2, rs=rs)))
                h = out
                bid += 1
        elif len(mod) == 2 and isinstance(mod[0], LayerNorm2d) and isinstance(mod[1], nn.Conv2d):
            ln, conv = mod[0], mod[1]
            t = K.layernorm(h, ln.weight, ln.bias)
            wp = packed(cache, f"{idx}.conv", conv.weight, lambda w: w.permute(0, 2, 3, 1))
            out = K.conv2x2(t, wp, conv.bias, conv.stride[0])
            saved.append(("down", mod, f"{idx}.conv", dict(x=h, t=t)))
            h = out
        else:
            raise RuntimeError(f"HIP training step: unsupported ConvNeXt features entry {idx}")
    return h, saved


def _set_grad(p: Tensor, g: Tensor) -> None:
    if p.requires_grad:
        p.grad = g.reshape(p.shape).contiguous()


def _block_backward(blk: CNBlock, sv: dict, dy: Tensor) -> Tensor:
    """Gradients of one CNBlock (written to the parameters' .grad); returns d input [B,H,W,C]."""
    from . import _lib
    dw, ln, l1, l2 = blk.block[0], blk.block[2], blk.block[3], blk.block[5]
    x = sv["x"]
    b, hh, ww, c = x.shape
    dev = x.device
    d_ls, d_b2 = torch.empty(c, device=dev), torch.empty(c, device=dev)
    dyv = dy.reshape(-1, c)
    dy2 = K.ls_backward(dyv, sv["y2"], blk.layer_scale.view(-1), sv["rs"], hh * ww, d_ls, d_b2)
    _set_grad(blk.layer_scale, d_ls)
    _set_grad(l2.bias, d_b2)
    if l2.weight.requires_grad:
        _set_grad(l2.weight, K.wgrad(dy2, sv["g"]))
    dh1 = K.linear(dy2, l2.weight.t().contiguous(), None, _lib.EPI_GELU_BWD, r=sv["h1"])
    if l1.weight.requires_grad:
        _set_grad(l1.weight, K.wgrad(dh1, sv["t"].view(-1, c)))
    if l1.bias.requires_grad:
        _set_grad(l1.bias, K.colsum(dh1))
    dt = K.linear(dh1, l1.weight.t().contiguous(), None, _lib.EPI_NONE)
    d_lnw, d_lnb = torch.empty(c, device=dev), torch.empty(c, device=dev)
    dz = K.ln_backward(sv["z"].view(-1, c), dt, ln.weight, d_lnw, d_lnb, want_dz=True).view(b, hh, ww, c)
    _set_grad(ln.weight, d_lnw)
    _set_grad(ln.bias, d_lnb)
    dwp, d_dwb = torch.empty(49, c, device=dev), torch.empty(c, device=dev)
    K.dwconv7_wgrad(dz, x, dwp, d_dwb)
    _set_grad(dw.weight, dwp.t())
    _set_grad(dw.bias, d_dwb)
    wflip = dw.weight.detach().flip(2, 3).reshape(c, 49).t().contiguous()
    dx = dy.reshape(b, hh, ww, c)                    # residual path; the branch's input grad adds in place
    K.dwconv7_plain(dz, wflip, None, out=dx, accumulate=True)
    return dx


def _stem_backward(mod: nn.Sequential, sv: dict, dy: Tensor) -> None:
    """Stem backward (Conv2d(3, 96, 4, 4) + LayerNorm2d): LN gradients, then the conv's
    weight (stride-4 patch gather, MFMA) and bias gradients; the input images need none."""
    conv, ln = mod[0], mod[1]
    z = sv["z"]
    b, h, w, c = z.shape
    dev = z.device
    d_lnw, d_lnb = torch.empty(c, device=dev), torch.empty(c, device=dev)
    need_dz = conv.weight.requires_grad or (conv.bias is not None and conv.bias.requires_grad)
    dz = K.ln_backward(z.view(-1, c), dy.reshape(-1, c), ln.weight, d_lnw, d_lnb, want_dz=need_dz)
    _set_grad(ln.weight, d_lnw)
    _set_grad(ln.bias, d_lnb)
    if not need_dz:
        return
    if conv.weight.requires_grad:
        gp = torch.empty(c, 4 * 4 * 4, device=dev)
        K.wgrad_conv(dz.view(b, h, w, c), sv["x"], 4, 4, 4, gp)
        _set_grad(conv.weight, gp.view(c, 4, 4, 4)[..., :3].permute(0, 3, 1, 2))
    if conv.bias is not None and conv.bias.requires_grad:
        _set_grad(conv.bias, K.colsum(dz))


def _down_backward(mod: nn.Sequential, sv: dict, dy: Tensor, need_dx: bool) -> Optional[Tensor]:
    """LayerNorm2d + Conv2d(k2, stride 1|2) backward; returns d input when ``need_dx``."""
    from . import _lib
    ln, conv = mod[0], mod[1]
    x, t = sv["x"], sv["t"]
    b, h, w, cin = t.shape
    cout, stride = conv.out_channels, conv.stride[0]
    if conv.weight.requires_grad:
        gp = torch.empty(cout, 4 * cin, device=t.device)
        K.wgrad_conv2x2(dy, t, stride, gp)
        _set_grad(conv.weight, gp.view(cout, 2, 2, cin).permute(0, 3, 1, 2))
    if conv.bias is not None and conv.bias.requires_grad:
        _set_grad(conv.bias, K.colsum(dy.reshape(-1, cout)))
    if not (ln.weight.requires_grad or ln.bias.requires_grad or need_dx):
        return None
    wd = conv.weight.detach()
    if stride == 1:        # transposed conv = conv of dy (pad 1) with the flipped, transposed taps
        dt = K.conv2d_nhwc(dy.contiguous(), wd.permute(1, 2, 3, 0).flip(1, 2).contiguous(), None, 1, 1,
                           _lib.EPI_NONE)
    else:                  # stride 2: taps do not overlap -> one GEMM, then place the 2x2 blocks
        oh, ow = dy.shape[1], dy.shape[2]
        gm = K.linear(dy.reshape(-1, cout), wd.permute(2, 3, 1, 0).reshape(4 * cin, cout).contiguous(), None,
                      _lib.EPI_NONE)
        dt = torch.zeros(b, h, w, cin, device=t.device)
        dt[:, :2 * oh, :2 * ow] = gm.view(b, oh, ow, 2, 2, cin).permute(0, 1, 3, 2, 4, 5).reshape(b, 2 * oh, 2 * ow, cin)
    d_lnw, d_lnb = torch.empty(cin, device=t.device), torch.empty(cin, device=t.device)
    dx = K.ln_backward(x.reshape(-1, cin), dt.reshape(-1, cin), ln.weight, d_lnw, d_lnb, want_dz=need_dx)
    _set_grad(ln.weight, d_lnw)
    _set_grad(ln.bias, d_lnb)
    return None if dx is None else dx.view(b, h, w, cin)


def _addon_suffix_backward(m: nn.Module, feats: Tensor, saved: list, d_logits: Tensor) -> None:
    """Backward from d logits (before the prototype softmax) through the add-on (1x1 conv when
    present) and the saved backbone suffix; every parameter with requires_grad gets .grad."""
    from . import _lib
    mods = list(m._add_on) if isinstance(m._add_on, nn.Sequential) else [m._add_on]
    if len(mods) == 2:                           # 1x1 prototype conv before the softmax
        conv = mods[0]
        bsz, hh, ww, cf = feats.shape
        pn = conv.out_channels
        dl = d_logits.view(-1, pn)
        if conv.weight.requires_grad:
            _set_grad(conv.weight, K.wgrad(dl, feats.view(-1, cf)))
        if conv.bias is not None and conv.bias.requires_grad:
            _set_grad(conv.bias, K.colsum(dl))
        dy = K.linear(dl, conv.weight.detach().view(pn, cf).t().contiguous(), None, _lib.EPI_NONE)
        dy = dy.view(bsz, hh, ww, cf)
    else:
        dy = d_logits
    if saved and saved[0][0] == "resnet":
        from . import resnet_train
        resnet_train.backward(m._net, saved[0][3], dy)
        saved.clear()
        return
    for i in range(len(saved) - 1, -1, -1):
        kind, mod, _, sv = saved[i]
        if kind == "block":
            dy = _block_backward(mod, sv, dy)
        elif kind == "stem":
            _stem_backward(mod, sv, dy)
        else:
            dy = _down_backward(mod, sv, dy, need_dx=i > 0)
        saved[i] = None                          # free the activations as we go


def _step_train_optimizers(m: nn.Module, optimizer_net, optimizer_classifier, pretrain: bool,
                           enforce_weight_sparsity: bool) -> None:
    """optimizer_classifier (not in pretrain; train.py:117-120) and optimizer_net (train.py:122-124)
    as device AdamW steps, then the sparsity clamps (train.py:131-140)."""
    cls = m._classification
    if not pretrain:
        for g in optimizer_classifier.param_groups:
            for p in g["params"]:
                if p.grad is not None:
                    post = None
                    if enforce_weight_sparsity:
                        post = (SPARSITY_DELTA, 0.0) if p is cls.weight else (0.0, 0.0) if p is cls.bias else None
                    hip_adamw_step(optimizer_classifier, p, p.grad, post)
    for g in optimizer_net.param_groups:
        for p in g["params"]:
            if p.grad is not None:
                hip_adamw_step(optimizer_net, p, p.grad)
    if not pretrain and enforce_weight_sparsity:
        if not cls.weight.requires_grad:
            K.weight_sparsify_(cls.weight.detach(), SPARSITY_DELTA)
        if cls.bias is not None and not cls.bias.requires_grad:
            K.clamp_min_(cls.bias.detach(), 0.0)
        K.clamp_min_(cls.normalization_multiplier.detach(), 1.0)


def hip_train_step(net: nn.Module, xs1: Tensor, xs2: Tensor, ys: Tensor, optimizer_net, optimizer_classifier,
                   pretrain: bool, epoch: int, nr_epochs: int, enforce_weight_sparsity: bool = True,
                   sd_keep: Optional[Dict[int, Tensor]] = None, generator: Optional[torch.Generator] = None,
                   step_optimizers: bool = True) -> Tensor:
    """One pretrain (``pretrain=True``) or joint iteration (train.py:75-140 with
    finetune=False) for a trainable backbone suffix: train-mode forward keeping the
    suffix's activations, the loss kernel, backward through head, add-on and suffix (every
    parameter with requires_grad gets its .grad), then optimizer_classifier (joint only)
    and optimizer_net steps (AdamW on the device) and the sparsity clamps.  Returns the
    loss-kernel stats without synchronising."""
    from .pipnet import add_on_logits_hip
    m = _inner(net)
    j = trainable_suffix_start(m)
    if j >= _backbone_units(m):
        raise NotImplementedError("HIP training step: no trainable backbone parameter (use the finetune step)")
    xs = torch.cat([xs1, xs2])
    if sd_keep is None:
        sd_keep = _sd_masks(m, xs.shape[0], generator)
    cls = m._classification
    w_align, w_tanh, w_class = (epoch / nr_epochs, 5.0, 0.0) if pretrain else FINETUNE_LOSS_WEIGHTS
    with torch.no_grad():
        feats, saved = _backbone_forward_saving(m, xs, j, sd_keep)
        logits = add_on_logits_hip(m._add_on, feats)
        proto, pooled = K.softmax_pool(logits, pool_mode=0)
        _, out = K.nonneg_linear(pooled, cls.weight, cls.bias, None)
        stats, d_out = K.train_loss(proto, pooled, out, ys, cls.normalization_multiplier, enforce_weight_sparsity,
                                    1.0, w_align, w_tanh, w_class, "pretrain" if pretrain else "train")
        if d_out is not None and (cls.weight.requires_grad or (cls.bias is not None and cls.bias.requires_grad)):
            dw, db = K.nonneg_linear_backward(d_out, pooled, cls.weight, cls.bias is not None)
            _set_grad(cls.weight, dw)
            if cls.bias is not None:
                _set_grad(cls.bias, db)
        d_logits = K.head_backward(proto, pooled, d_out, cls.weight, w_align, w_tanh)
        _addon_suffix_backward(m, feats, saved, d_logits)
        if step_optimizers:
            _step_train_optimizers(m, optimizer_net, optimizer_classifier, pretrain, enforce_weight_sparsity)
    return stats


def hip_count_train_supported(net: nn.Module) -> bool:
    """A ConvNeXt CountPIPNet (fp32, ROCm) whose trainable backbone part is a suffix
    features[j:] (j = 0: the stem too), with an intermediate layer that has a HIP backward
    (the reference's pretrain, "train + freeze params" and "train everything" phases for
    CountPIPNet, main.py:238-256, 360-390)."""
    from .count_pipnet_utils import (BilinearIntermediate, IdentityIntermediate, LinearFull, LinearIntermediate,
                                     OneHotEncoder)
    m = _inner(net)
    if not hasattr(m, "_max_count") or not _backbone_ok(m):
        return False
    if not isinstance(m._intermediate, (IdentityIntermediate, OneHotEncoder, LinearFull, LinearIntermediate,
                                       BilinearIntermediate)):
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 for p in m.parameters()):
        return False
    return trainable_suffix_start(m) < _backbone_units(m)


def hip_count_train_step(net: nn.Module, xs1: Tensor, xs2: Tensor, ys: Tensor, optimizer_net, optimizer_classifier,
                         pretrain: bool, epoch: int, nr_epochs: int, enforce_weight_sparsity: bool = True,
                         tanh_loss_coeff: float = 1.0, sd_keep: Optional[Dict[int, Tensor]] = None,
                         generator: Optional[torch.Generator] = None, step_optimizers: bool = True) -> Tensor:
    """One CountPIPNet pretrain (``pretrain=True``) or joint iteration (train.py:75-140 with
    is_count_pipnet=True, finetune=False): train-mode forward keeping the backbone suffix's
    activations (soft Gumbel-softmax / softmax head, spatial sums = raw counts, STE round and
    clamp, intermediate layer, classifier), the loss kernel (tanh over C * raw counts), then
    the backward: classifier -> intermediate (parameter and input gradients; ModifiedSTE for
    a one-hot encoder) -> ClampSTE / STE_Round -> d counts (+ the tanh term) -> d proto
    (+ the align term) -> soft-max backward scaled by 1/tau -> add-on -> suffix; AdamW steps
    and the sparsity clamps as ``hip_train_step``.  Returns the loss-kernel stats."""
    m = _inner(net)
    j = trainable_suffix_start(m)
    if j >= _backbone_units(m):
        raise NotImplementedError("HIP count training step: no trainable backbone parameter (use the finetune step)")
    xs = torch.cat([xs1, xs2])
    if sd_keep is None:
        sd_keep = _sd_masks(m, xs.shape[0], generator)
    cls = m._classification
    w_align, w_tanh, w_class = (epoch / nr_epochs, 5.0, 0.0) if pretrain else FINETUNE_LOSS_WEIGHTS
    with torch.no_grad():
        proto, counts, clamped, saved, inter, out = _count_train_forward(m, xs, sd_keep, j)
        stats, d_out = K.train_loss(proto, counts, out, ys, cls.normalization_multiplier, enforce_weight_sparsity,
                                    tanh_loss_coeff, w_align, w_tanh, w_class, "pretrain" if pretrain else "train")
        d_counts = None
        if d_out is not None:
            if cls.weight.requires_grad or (cls.bias is not None and cls.bias.requires_grad):
                dw, db = K.nonneg_linear_backward(d_out, inter, cls.weight, cls.bias is not None)
                _set_grad(cls.weight, dw)
                if cls.bias is not None:
                    _set_grad(cls.bias, db)
            d_inter = K.nonneg_linear_dx(d_out, cls.weight.detach())
            d_clamped = _intermediate_backward(m._intermediate, clamped, saved, d_inter, need_dx=True)
            if d_clamped is not None:
                d_counts = K.count_ste_backward(counts, d_clamped, m._max_count, bool(m._use_ste),
                                                not m._is_clamp_backward_identity or not m._use_ste)
        d_logits = K.count_head_backward(proto, counts, d_counts, w_align, w_tanh, tanh_loss_coeff, saved["tau"])
        del proto
        _addon_suffix_backward(m, saved["feats"], saved["suffix"], d_logits)
        if step_optimizers:
            _step_train_optimizers(m, optimizer_net, optimizer_classifier, pretrain, enforce_weight_sparsity)
    return stats


# ------------------------------------------------------------------------------------------
# epoch loop (train.py:8-150 drop-in)
# ------------------------------------------------------------------------------------------
class HipEpoch:
    """Runs HIP training iterations back to back with all bookkeeping on the device.

    Per batch (view-1 images, view-2 images, labels): one device step, then the schedules
    advance as in the reference -- the classifier's CosineAnnealingWarmRestarts to the
    fractional epoch position (train.py:120, not in pretrain), the backbone's scheduler once
    per iteration (train.py:124-126, not in finetune).  The five running sums (align, tanh,
    class, loss, accuracy) live in one device vector; ``summary()`` is the single host read."""

    TERMS = ("align", "tanh", "class")

    def __init__(self, step, weights: Tuple[float, float, float], track_acc: bool):
        self.step, self.weights, self.track_acc = step, weights, track_acc
        self.sums: Optional[Tensor] = None
        self.count = 0
        self.lrs_class: list = []
        self.lrs_net: list = []

    def _add(self, stats: Tensor, labels: int) -> None:
        acc = stats[4:5] / float(2 * labels) if self.track_acc else torch.zeros_like(stats[4:5])
        row = torch.cat([stats[:4], acc]).double()
        self.sums = row if self.sums is None else self.sums.add_(row)
        self.count += 1

    def run(self, batches, optimizers, epoch: int, device, scheduler_classifier=None, scheduler_net=None) -> None:
        n_batches = len(batches)
        for pos, batch in enumerate(batches):
            a, b, labels = (t.to(device, non_blocking=True) for t in batch)
            for opt in optimizers:
                opt.zero_grad(set_to_none=True)
            self._add(self.step(a, b, labels), labels.shape[0])
            if scheduler_classifier is not None:
                scheduler_classifier.step((epoch - 1) + pos / n_batches)
                self.lrs_class.append(scheduler_classifier.get_last_lr()[0])
            if scheduler_net is not None:
                scheduler_net.step()
                self.lrs_net.append(scheduler_net.get_last_lr()[0])
            else:
                self.lrs_net.append(0.0)

    def summary(self) -> dict:
        vals = self.sums.cpu().tolist() if self.sums is not None else [0.0] * 5
        n = float(max(self.count, 1))
        info = {}
        for j, term in enumerate(self.TERMS):
            info[f"{term}_loss_raw"] = vals[j] / n
            info[f"{term}_loss_weighted"] = vals[j] / n * self.weights[j]
        info.update(train_accuracy=vals[4] / n, loss=vals[3] / n, lrs_net=list(self.lrs_net),
                    lrs_class=list(self.lrs_class))
        return info


def train_pipnet(net, train_loader, optimizer_net, optimizer_classifier, scheduler_net, scheduler_classifier,
                 criterion, epoch, nr_epochs, device, is_count_pipnet=False, pretrain=False, finetune=False,
                 progress_prefix: str = "Train Epoch", enforce_weight_sparsity=True, tanh_loss_coeff=1.0,
                 generator: Optional[torch.Generator] = None, verbose: bool = False) -> dict:
    """Drop-in for train.py:8-150 (same arguments, same ``train_info`` keys; progress output
    reduced to one optional line) for a ConvNeXt or ResNet-50 PIP-Net and a ConvNeXt
    CountPIPNet: the finetune phase (``hip_finetune_step`` / ``hip_count_finetune_step``) and
    the pretrain / joint / "train everything" phases with a trainable backbone suffix
    (``hip_train_step`` / ``hip_count_train_step``).  Anything else (a trainable ResNet stem,
    an intermediate layer without a HIP backward, non-fp32 parameters) raises -- run the
    reference's own loop on these modules (torch autograd path)."""
    if pretrain and finetune:
        raise NotImplementedError("count_pipnet_amd.train_pipnet: pretrain and finetune are exclusive")
    if is_count_pipnet and finetune:
        if not hip_count_finetune_supported(net):
            raise NotImplementedError("count_pipnet_amd.train_pipnet: this CountPIPNet finetune setup has no HIP "
                                      "step; run the reference train_pipnet with these modules")
        weights = FINETUNE_LOSS_WEIGHTS

        def step(a, b, labels):
            return hip_count_finetune_step(net, a, b, labels, optimizer_classifier, enforce_weight_sparsity,
                                           tanh_loss_coeff, generator=generator)
    elif is_count_pipnet:
        if not hip_count_train_supported(net):
            raise NotImplementedError("count_pipnet_amd.train_pipnet: this CountPIPNet training setup (ResNet "
                                      "backbone or non-fp32 parameters) runs on the torch path")
        weights = (epoch / nr_epochs, 5.0, 0.0) if pretrain else FINETUNE_LOSS_WEIGHTS

        def step(a, b, labels):
            return hip_count_train_step(net, a, b, labels, optimizer_net, optimizer_classifier, pretrain, epoch,
                                        nr_epochs, enforce_weight_sparsity, tanh_loss_coeff, generator=generator)
    elif finetune and hip_finetune_supported(net):
        weights = FINETUNE_LOSS_WEIGHTS

        def step(a, b, labels):
            return hip_finetune_step(net, a, b, labels, optimizer_classifier, enforce_weight_sparsity,
                                     generator=generator)
    elif not finetune and hip_train_supported(net):
        weights = (epoch / nr_epochs, 5.0, 0.0) if pretrain else FINETUNE_LOSS_WEIGHTS

        def step(a, b, labels):
            return hip_train_step(net, a, b, labels, optimizer_net, optimizer_classifier, pretrain, epoch,
                                  nr_epochs, enforce_weight_sparsity, generator=generator)
    else:
        raise NotImplementedError(
            "count_pipnet_amd.train_pipnet: this configuration (phase / trainable parameters / device) has no HIP "
            "step; use the reference train_pipnet with these modules (torch autograd path)")
    net.train()
    _inner(net)._classification.requires_grad = not pretrain
    runner = HipEpoch(step, weights, track_acc=not pretrain)
    opts = [o for o in (optimizer_classifier, optimizer_net) if o is not None]
    opts = [o for i, o in enumerate(opts) if all(o is not q for q in opts[:i])]
    runner.run(train_loader, opts, epoch, device, None if pretrain else scheduler_classifier,
               None if finetune else scheduler_net)
    info = runner.summary()
    if verbose:
        terms = ", ".join(f"{t}={info[t + '_loss_raw']:.4f}" for t in HipEpoch.TERMS)
        print(f"[{progress_prefix} {epoch}] HIP: {runner.count} iterations, {terms}", flush=True)
    return info
