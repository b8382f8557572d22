"""Train-mode ResNet backbone on the HIP kernels: the forward and backward of
``features/resnet_features.py`` (Bottleneck, resnet_features.py:77-119; stem, :137-140)
under ``net.train()`` (pipnet/train.py:14), for the reference's ResNet-50 training phases
(util/args.py:280-290 parameter groups: ``layer4.2`` "train", ``layer3`` / ``layer4``
"freeze" -- trainable in pretrain and in the "train + freeze params" epochs -- and
``layer2`` "backbone", trainable in the "train everything" epochs; the stem and ``layer1``
never train, main.py:238-256, 360-390).

Every BatchNorm2d runs in train mode, frozen layers included: batch mean / biased variance
normalise, the running statistics take the momentum update (``kernels.bn_stats``), exactly
what autograd's BatchNorm2d does under ``net.train()``.  The eval path folds BN into the
conv weights (``resnet_hip``); train mode cannot, so each conv runs raw (implicit-GEMM MFMA,
``kernels.conv2d_nhwc`` / ``kernels.linear`` for 1x1) followed by the statistics and the
normalise (+ residual) (+ ReLU) pass.

Backward, from d features (NHWC) down to the first block holding a trainable parameter:
  BN (+ReLU mask from the saved output)  -> ``kernels.bn_backward`` (d gamma / d beta, dx)
  1x1 conv        dW = dY^T X (``kernels.wgrad``), dX = dY W (``kernels.linear``; into the
                  identity-path gradient with the residual epilogue)
  3x3 conv        dW: ``kernels.wgrad_conv`` (zero padding 1), dX: the flipped, transposed
                  taps as a stride-1 conv of dY -- zero-inserted first when the forward
                  stride is 2 (``kernels.stride_scatter``)
  downsample      1x1 stride-s conv + BN on the identity path
Weights are repacked only when their version changes (every optimizer step).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from . import _lib
from . import kernels as K

Tensor = torch.Tensor


def _blocks(model) -> List[Tuple[str, nn.Module]]:
    out = []
    for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4)):
        for j, blk in enumerate(layer):
            out.append((f"layer{li + 1}.{j}", blk))
    return out


def supported(model) -> bool:
    """Bottleneck ResNets (the reference trains resnet50 only, util/args.py:280) with the
    stem frozen (it never trains in the reference)."""
    from .resnet_features import Bottleneck, ResNet_features
    if not isinstance(model, ResNet_features):
        return False
    if any(not isinstance(b, Bottleneck) for _, b in _blocks(model)):
        return False
    stem = list(model.conv1.parameters()) + list(model.bn1.parameters())
    return not any(p.requires_grad for p in stem)


def trainable_start(model) -> int:
    """Index (in ``_blocks`` order) of the first block with a trainable parameter; the block
    count when the backbone is frozen."""
    blocks = _blocks(model)
    for i, (_, blk) in enumerate(blocks):
        if any(p.requires_grad for p in blk.parameters()):
            return i
    return len(blocks)


def _packed(cache: Dict, key: str, w: Tensor, fn):
    stamp = (w.data_ptr(), w._version)
    ent = cache.get(key)
    if ent is None or ent[0] != stamp:
        with torch.no_grad():
            ent = (stamp, fn(w.detach()).contiguous())
        cache[key] = ent
    return ent[1]


def _conv(cache: Dict, key: str, conv: nn.Conv2d, x: Tensor, cpad: Optional[int] = None) -> Tensor:
    """Raw (bias-free) conv of NHWC x."""
    if conv.groups != 1 or conv.dilation != (1, 1) or conv.bias is not None or \
            conv.kernel_size[0] != conv.kernel_size[1]:
        raise RuntimeError(f"ResNet HIP training: unsupported conv {conv}")
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    b, h, w, cin = x.shape
    if k == 1 and s == 1 and p == 0:
        wt = _packed(cache, key + ".w11", conv.weight, lambda t: t.view(t.shape[0], t.shape[1]))
        return K.linear(x.view(-1, cin), wt).view(b, h, w, wt.shape[0])
    wp = _packed(cache, key + ".wohwi", conv.weight,
                 lambda t: torch.nn.functional.pad(t.permute(0, 2, 3, 1), (0, (cpad or t.shape[1]) - t.shape[1])))
    return K.conv2d_nhwc(x, wp, None, s, p, _lib.EPI_NONE)


def _bn(bn: nn.BatchNorm2d, c: Tensor, relu: bool, residual: Optional[Tensor] = None):
    """Train-mode BatchNorm2d (+ residual) (+ ReLU) of the raw conv output c; running stats
    updated as torch does (momentum None = cumulative average)."""
    if not bn.affine:
        raise RuntimeError("ResNet HIP training: BatchNorm2d without affine parameters")
    rm = rv = None
    mom = 0.0
    if bn.track_running_stats and bn.running_mean is not None:
        bn.num_batches_tracked.add_(1)
        mom = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked.item())
        rm, rv = bn.running_mean, bn.running_var
    mean, invstd = K.bn_stats(c, bn.eps, float(mom), rm, rv)
    y = K.bn_apply(c, mean, invstd, bn.weight.detach(), bn.bias.detach(), residual, relu)
    return y, (mean, invstd)


def _block_forward(cache: Dict, key: str, blk, x: Tensor, save: bool):
    c1 = _conv(cache, key + ".c1", blk.conv1, x)
    a1, s1 = _bn(blk.bn1, c1, True)
    c2 = _conv(cache, key + ".c2", blk.conv2, a1)
    a2, s2 = _bn(blk.bn2, c2, True)
    c3 = _conv(cache, key + ".c3", blk.conv3, a2)
    cd = sd = None
    if blk.downsample is not None:
        ds_conv, ds_bn = blk.downsample[0], blk.downsample[1]
        cd = _conv(cache, key + ".ds", ds_conv, x)
        idt, sd = _bn(ds_bn, cd, False)
    else:
        idt = x
    out, s3 = _bn(blk.bn3, c3, True, residual=idt)
    rec = dict(x=x, c1=c1, a1=a1, s1=s1, c2=c2, a2=a2, s2=s2, c3=c3, s3=s3, cd=cd, sd=sd, out=out) if save else None
    return out, rec


def train_forward(model, xs: Tensor, start: Optional[int]) -> Tuple[Tensor, list]:
    """ResNet_features.forward in train mode on NHWC fp32 -> (features NHWC, saved): the
    blocks from ``start`` on keep their activations (``start`` None: none kept)."""
    K.require_device(xs, "network input")
    xs = xs.contiguous()
    if xs.shape[1] != 3:
        raise RuntimeError(f"ResNet stem expects 3 input channels, got {xs.shape[1]}")
    mp = model.maxpool
    if not (mp.kernel_size == 3 and mp.stride == 2 and mp.padding == 1):
        raise RuntimeError(f"ResNet HIP training: unsupported stem pool {mp}")
    cache = model._hip_pack.setdefault("train", {})
    h = K.nchw_to_nhwc(xs, 4)
    c = _conv(cache, "stem", model.conv1, h, cpad=4)
    h, _ = _bn(model.bn1, c, True)
    del c
    h = K.maxpool2d_nhwc(h, 3, 2, 1)
    saved = []
    for i, (key, blk) in enumerate(_blocks(model)):
        keep = start is not None and i >= start
        h, rec = _block_forward(cache, key, blk, h, keep)
        if keep:
            saved.append((key, blk, rec))
    return h, saved


def _set_grad(p: Tensor, g: Tensor) -> None:
    if p.requires_grad:
        p.grad = g.reshape(p.shape).contiguous()


def _bn_grads(bn: nn.BatchNorm2d, dg: Tensor, db: Tensor) -> None:
    _set_grad(bn.weight, dg)
    _set_grad(bn.bias, db)


def _conv_wgrad(conv: nn.Conv2d, dy: Tensor, x: Tensor) -> None:
    if not conv.weight.requires_grad:
        return
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    cout, cin = conv.out_channels, conv.in_channels
    if k == 1 and s == 1:
        _set_grad(conv.weight, K.wgrad(dy.reshape(-1, cout), x.reshape(-1, cin)))
        return
    gp = torch.empty(cout, k * k * cin, device=dy.device, dtype=torch.float32)
    K.wgrad_conv(dy, x, k, k, s, gp, pad=p)
    _set_grad(conv.weight, gp.view(cout, k, k, cin).permute(0, 3, 1, 2))


def _conv_dgrad(cache: Dict, key: str, conv: nn.Conv2d, dy: Tensor, x_shape, into: Optional[Tensor] = None) -> Tensor:
    """d input of a bias-free conv; added into ``into`` (same shape as the input) when given."""
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    b, h, w, cin = x_shape
    cout = conv.out_channels
    if k == 1:
        wt = _packed(cache, key + ".w11t", conv.weight, lambda t: t.view(cout, cin).t())
        if s == 1:
            if into is None:
                return K.linear(dy.reshape(-1, cout), wt).view(b, h, w, cin)
            iv = into.view(-1, cin)
            K.linear(dy.reshape(-1, cout), wt, None, _lib.EPI_RESID, r=iv, out=iv)
            return into
        g = K.linear(dy.reshape(-1, cout), wt).view(dy.shape[0], dy.shape[1], dy.shape[2], cin)
        return K.stride_scatter(g, h, w, s, out=into, accumulate=into is not None)
    if p != (k - 1) // 2:
        raise RuntimeError(f"ResNet HIP training: unsupported conv padding {conv}")
    wf = _packed(cache, key + ".wflip", conv.weight, lambda t: t.flip(2, 3).permute(1, 2, 3, 0))
    src = dy if s == 1 else K.stride_scatter(dy, h, w, s)
    d = K.conv2d_nhwc(src, wf, None, 1, p, _lib.EPI_NONE)
    if tuple(d.shape) != (b, h, w, cin):
        raise RuntimeError(f"ResNet HIP training: dgrad shape {tuple(d.shape)} vs {(b, h, w, cin)}")
    if into is not None:
        into.add_(d)
        return into
    return d


def _block_backward(cache: Dict, key: str, blk, sv: dict, dout: Tensor, need_dx: bool) -> Optional[Tensor]:
    x = sv["x"]
    # bn3 + identity + ReLU: g = dout * (out > 0) feeds both bn3 and the identity path
    dc3, g, dg, db = K.bn_backward(sv["c3"], dout, *sv["s3"], blk.bn3.weight.detach(), relu_out=sv["out"],
                                   want_masked=True)
    _bn_grads(blk.bn3, dg, db)
    dx = None
    if blk.downsample is not None:
        ds_conv, ds_bn = blk.downsample[0], blk.downsample[1]
        dcd, _, dg, db = K.bn_backward(sv["cd"], g, *sv["sd"], ds_bn.weight.detach())
        _bn_grads(ds_bn, dg, db)
        _conv_wgrad(ds_conv, dcd, x)
        if need_dx:
            dx = _conv_dgrad(cache, key + ".ds", ds_conv, dcd, x.shape)
    elif need_dx:
        dx = g
    del g
    _conv_wgrad(blk.conv3, dc3, sv["a2"])
    da2 = _conv_dgrad(cache, key + ".c3", blk.conv3, dc3, sv["a2"].shape)
    del dc3
    dc2, _, dg, db = K.bn_backward(sv["c2"], da2, *sv["s2"], blk.bn2.weight.detach(), relu_out=sv["a2"])
    _bn_grads(blk.bn2, dg, db)
    del da2
    _conv_wgrad(blk.conv2, dc2, sv["a1"])
    da1 = _conv_dgrad(cache, key + ".c2", blk.conv2, dc2, sv["a1"].shape)
    del dc2
    dc1, _, dg, db = K.bn_backward(sv["c1"], da1, *sv["s1"], blk.bn1.weight.detach(), relu_out=sv["a1"])
    _bn_grads(blk.bn1, dg, db)
    del da1
    _conv_wgrad(blk.conv1, dc1, x)
    if need_dx:
        dx = _conv_dgrad(cache, key + ".c1", blk.conv1, dc1, x.shape, into=dx)
    return dx


def backward(model, saved: list, dfeat: Tensor) -> None:
    """Backward from d features (NHWC) through the saved blocks (last to first); every
    backbone parameter with requires_grad gets .grad."""
    cache = model._hip_pack.setdefault("train", {})
    dy = dfeat.contiguous()
    for i in range(len(saved) - 1, -1, -1):
        key, blk, sv = saved[i]
        dy = _block_backward(cache, key, blk, sv, dy, need_dx=i > 0)
        saved[i] = None                          # free the activations as we go
