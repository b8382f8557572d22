"""HIP executor for the ResNet feature backbones (features/resnet_features.py:77-229).

NHWC end to end.  Eval-mode BatchNorm is folded into each convolution at pack time
(w' = w * g/sqrt(v+eps), b' = beta - mu * g/sqrt(v+eps)); every conv is one implicit-GEMM
MFMA launch with bias / ReLU / identity-add+ReLU fused into its epilogue:

  stem:        NCHW->NHWC (channels padded 3->4) -> conv7x7 s2 p3 +BN+ReLU -> maxpool 3x3 s2 p1
  Bottleneck:  conv1x1+BN+ReLU -> conv3x3(s)+BN+ReLU -> conv1x1+BN (+ downsample conv1x1(s)+BN)
               + identity -> ReLU  (the last three in one epilogue)
  BasicBlock:  conv3x3(s)+BN+ReLU -> conv3x3+BN + identity -> ReLU

Folded weights are cached per device and rebuilt whenever any of the conv / BN tensors
changes (storage pointer or in-place version counter).

``model.hip_dtype = torch.bfloat16`` selects the bf16 build (BASELINE C3): activations bf16
NHWC, folded weights rounded to bf16 once at pack time ([Cout][KH*KW*Cin padded to 64]),
biases fp32, fp32 accumulation on v_mfma_f32_32x32x16_bf16, every conv output rounded to
nearest even.  The stem input is padded 3 -> 8 channels (one 16-B chunk per tap).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from .backend import packed_ready
from . import _lib
from . import kernels as K

Tensor = torch.Tensor


def _fold(cache: Dict, key: str, conv: nn.Conv2d, bn: nn.BatchNorm2d, cpad: Optional[int] = None,
          bf16: bool = False):
    ts = [conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var]
    if conv.bias is not None:
        ts.append(conv.bias)
    stamp = tuple((t.data_ptr(), t._version) for t in ts) + (bn.eps,)
    ck = (key, str(conv.weight.device), bf16)
    ent = cache.get(ck)
    if ent is None or ent[0] != stamp:
        with torch.no_grad():
            scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
            w = conv.weight * scale.view(-1, 1, 1, 1)
            b = bn.bias - bn.running_mean * scale
            if conv.bias is not None:
                b = b + conv.bias * scale
            w = w.permute(0, 2, 3, 1)                           # [Cout, KH, KW, Cin]
            if cpad is not None and cpad > w.shape[3]:
                w = torch.nn.functional.pad(w, (0, cpad - w.shape[3]))
            w = w.contiguous().float()
            if bf16:
                w = K.pack_conv_weight_bf16(w)
            ent = (stamp, (w, b.contiguous().float()))
        cache[ck] = ent
        packed_ready()
    return ent[1]


def _stem_s2d(cache: Dict, conv: nn.Conv2d, bn: nn.BatchNorm2d):
    """Folded stem weights re-laid for the space-to-depth 4x4 conv (kernels.stem_weight_s2d),
    bf16-packed; rebuilt whenever the BatchNorm fold is."""
    w, b = _fold(cache, "stem.f32", conv, bn)                   # [64, 7, 7, 3] fp32
    ck = ("stem.s2d", str(w.device))
    ent = cache.get(ck)
    if ent is None or ent[0] is not w:
        with torch.no_grad():
            ent = (w, K.pack_conv_weight_bf16(K.stem_weight_s2d(w)))
        cache[ck] = ent
        packed_ready()
    return ent[1], b


def _conv_bn(cache, key, conv, bn, x, epilogue, r=None, cpad=None):
    if conv.groups != 1 or conv.dilation != (1, 1) or conv.kernel_size[0] != conv.kernel_size[1]:
        raise RuntimeError(f"ResNet HIP path: unsupported conv {conv}")
    if x.dtype == torch.bfloat16:
        w, b = _fold(cache, key, conv, bn, cpad, bf16=True)
        kh, kw = conv.kernel_size
        return K.conv2d_nhwc_bf16(x, w, kh, kw, b, conv.stride[0], conv.padding[0], epilogue, r)
    w, b = _fold(cache, key, conv, bn, cpad)
    return K.conv2d_nhwc(x, w, b, conv.stride[0], conv.padding[0], epilogue, r)


DUAL_1X1 = True      # tools / A-B runs may switch the dual downsample + conv1 launch off
# bf16 stem fused with its max-pool (pipnet_stem_pool_bf16); False = conv + pool launches, bitwise
# the same map (A/B: tools/ab_toggle.py count_pipnet_amd.resnet_hip.STEM_POOL c3)
STEM_POOL = True


def _dual_ok(blk, h) -> bool:
    """A first Bottleneck whose downsample and conv1 are both 1x1 stride-1 convs over h with
    Cout % 256 == 0 (C3's layer3 / layer4 at stride 1): one launch for both (the input read once)."""
    if not DUAL_1X1 or h.dtype != torch.bfloat16 or blk.downsample is None or len(blk.downsample) != 2:
        return False
    ds, c1 = blk.downsample[0], blk.conv1
    return all(isinstance(c, nn.Conv2d) and c.kernel_size == (1, 1) and c.stride == (1, 1) and c.padding == (0, 0)
               and c.groups == 1 and c.out_channels % 256 == 0 for c in (ds, c1)) and isinstance(blk.downsample[1],
                                                                                                   nn.BatchNorm2d)


def _dual_weights(cache, key, blk):
    """Folded + packed downsample and conv1 weights stacked [N_ds + N_c1, Kp], biases stacked."""
    wd, bd = _fold(cache, key + ".ds", blk.downsample[0], blk.downsample[1], bf16=True)
    w1, b1 = _fold(cache, key + ".c1", blk.conv1, blk.bn1, bf16=True)
    ck = (key + ".dual", str(wd.device))
    ent = cache.get(ck)
    if ent is None or ent[0][0] is not wd or ent[0][1] is not w1:
        with torch.no_grad():
            ent = ((wd, w1), (torch.cat([wd, w1]).contiguous(), torch.cat([bd, b1]).contiguous()))
        cache[ck] = ent
        packed_ready()
    return ent[1][0], ent[1][1], wd.shape[0], w1.shape[0]


def _bottleneck(cache, key, blk, h):
    from .resnet_features import BasicBlock, Bottleneck
    if isinstance(blk, Bottleneck) and _dual_ok(blk, h):
        w, b, nd, n1 = _dual_weights(cache, key, blk)
        idt, t = K.conv1x1_bf16_dual(h, w, b, nd, n1)
        t = _conv_bn(cache, key + ".c2", blk.conv2, blk.bn2, t, _lib.EPI_BIAS_RELU)
        return _conv_bn(cache, key + ".c3", blk.conv3, blk.bn3, t, _lib.EPI_BIAS_RESID_RELU, r=idt)
    if blk.downsample is not None:
        ds_conv, ds_bn = blk.downsample[0], blk.downsample[1]
        idt = _conv_bn(cache, key + ".ds", ds_conv, ds_bn, h, _lib.EPI_BIAS)
    else:
        idt = h
    if isinstance(blk, Bottleneck):
        t = _conv_bn(cache, key + ".c1", blk.conv1, blk.bn1, h, _lib.EPI_BIAS_RELU)
        t = _conv_bn(cache, key + ".c2", blk.conv2, blk.bn2, t, _lib.EPI_BIAS_RELU)
        return _conv_bn(cache, key + ".c3", blk.conv3, blk.bn3, t, _lib.EPI_BIAS_RESID_RELU, r=idt)
    if isinstance(blk, BasicBlock):
        t = _conv_bn(cache, key + ".c1", blk.conv1, blk.bn1, h, _lib.EPI_BIAS_RELU)
        return _conv_bn(cache, key + ".c2", blk.conv2, blk.bn2, t, _lib.EPI_BIAS_RESID_RELU, r=idt)
    raise RuntimeError(f"ResNet HIP path: unsupported block {type(blk).__name__}")


def resnet_features_hip(model, x: Tensor, cache: Dict) -> Tensor:
    """ResNet_features.forward (resnet_features.py:211-222) on HIP kernels -> NHWC features
    (fp32, or bf16 when ``model.hip_dtype`` is torch.bfloat16); resnet_features_hip_steps,
    drained."""
    from .convnext_features import drain
    return drain(resnet_features_hip_steps(model, x, cache))


def resnet_features_hip_steps(model, x: Tensor, cache: Dict):
    """Generator form of resnet_features_hip: yields after the stem and after every block
    (their launches enqueued), returns the NHWC features -- concurrent sub-batch forwards
    enqueue block by block (pipnet._forward_hip_split)."""
    K.require_device(x, "network input")
    x = x.contiguous()
    if x.shape[1] != 3:
        raise RuntimeError(f"ResNet stem expects 3 input channels, got {x.shape[1]}")
    mp = model.maxpool
    if not (mp.kernel_size == 3 and mp.stride == 2 and mp.padding == 1):
        raise RuntimeError(f"ResNet HIP path: unsupported stem pool {mp}")
    if getattr(model, "hip_dtype", torch.float32) == torch.bfloat16:
        c1 = model.conv1
        if c1.kernel_size == (7, 7) and c1.stride == (2, 2) and c1.padding == (3, 3) and c1.groups == 1 \
                and c1.dilation == (1, 1):
            # space-to-depth stem: a 4x4 stride-1 conv with K = 256 instead of 7x7x8 -> 448
            w, b = _stem_s2d(cache, c1, model.bn1)
            s2d = K.nchw_to_s2d_bf16(x)
            if STEM_POOL and c1.out_channels == 64 and s2d.shape[2] - 3 <= 112:
                h = K.stem_pool_bf16(s2d, w, b)           # conv + bias + ReLU + max-pool, one launch
            else:
                h = K.maxpool2d_nhwc_bf16(K.conv2d_nhwc_bf16(s2d, w, 4, 4, b, 1, 0, _lib.EPI_BIAS_RELU), 3, 2, 1)
        else:
            h = K.nchw_to_nhwc_bf16(x, 8)
            h = _conv_bn(cache, "stem", c1, model.bn1, h, _lib.EPI_BIAS_RELU, cpad=8)
            h = K.maxpool2d_nhwc_bf16(h, 3, 2, 1)
    else:
        h = K.nchw_to_nhwc(x, 4)
        h = _conv_bn(cache, "stem", model.conv1, model.bn1, h, _lib.EPI_BIAS_RELU, cpad=4)
        h = K.maxpool2d_nhwc(h, 3, 2, 1)
    yield
    for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4)):
        for j, blk in enumerate(layer):
            h = _bottleneck(cache, f"layer{li + 1}.{j}", blk, h)
            yield
    return h
