"""ConvNeXt-tiny feature backbones -- drop-in for ``features/convnext_features.py``.

Module tree, attribute names and ``state_dict`` keys are those of torchvision's
``convnext_tiny`` (``features.{i}.{j}.block.{0,2,3,5}``, ``layer_scale``, stem
``features.0.{0,1}``, downsample ``features.{2,4,6}.{0,1}``), so reference
checkpoints load with ``strict=True``.  torchvision itself is not a dependency.

Eval + no-grad forwards run on the HIP kernels, NHWC end to end:
  stem (conv k4 s4 + LN)  ->  per CNBlock: dwconv7+LN -> Linear+GELU (MFMA) ->
  Linear*layer_scale+residual (MFMA, in place)  ->  downsample: LN -> conv k2 (MFMA implicit GEMM)
and return a ``[B,C,h,w]`` tensor whose storage is NHWC (channels_last strides).
Training / grad-enabled forwards use the plain torch modules (autograd intact).
"""
from __future__ import annotations

import os
import warnings
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import kernels as K
from .backend import use_hip, packed_ready

Tensor = torch.Tensor


# ------------------------------------------------------------------------------------------
# torchvision-compatible module tree (restated; torchvision is absent)
# ------------------------------------------------------------------------------------------
class LayerNorm2d(nn.LayerNorm):
    def forward(self, x: Tensor) -> Tensor:
        x = x.permute(0, 2, 3, 1)
        x = F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)
        return x.permute(0, 3, 1, 2)


class Permute(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.dims = list(dims)

    def forward(self, x: Tensor) -> Tensor:
        return torch.permute(x, self.dims)


class StochasticDepth(nn.Module):
    """Row-mode stochastic depth; identity in eval (torchvision.ops.StochasticDepth)."""

    def __init__(self, p: float, mode: str = "row"):
        super().__init__()
        self.p, self.mode = p, mode

    def forward(self, x: Tensor) -> Tensor:
        if not self.training or self.p == 0.0:
            return x
        keep = 1.0 - self.p
        noise = torch.empty([x.shape[0]] + [1] * (x.ndim - 1), dtype=x.dtype, device=x.device).bernoulli_(keep)
        return x * noise.div_(keep)


class CNBlock(nn.Module):
    def __init__(self, dim: int, layer_scale: float = 1e-6, stochastic_depth_prob: float = 0.0):
        super().__init__()
        self.block = nn.Sequential(
            nn.Conv2d(dim, dim, kernel_size=7, padding=3, groups=dim, bias=True),
            Permute([0, 2, 3, 1]),
            nn.LayerNorm(dim, eps=1e-6),
            nn.Linear(dim, 4 * dim, bias=True),
            nn.GELU(),
            nn.Linear(4 * dim, dim, bias=True),
            Permute([0, 3, 1, 2]),
        )
        self.layer_scale = nn.Parameter(torch.ones(dim, 1, 1) * layer_scale)
        self.stochastic_depth = StochasticDepth(stochastic_depth_prob, "row")

    def forward(self, x: Tensor) -> Tensor:
        result = self.layer_scale * self.block(x)
        result = self.stochastic_depth(result)
        return result + x


class Conv2dNormActivation(nn.Sequential):
    """Stem: Conv2d(3,96,k4,s4,bias) + LayerNorm2d(96) (no activation)."""

    def __init__(self, cin: int, cout: int, kernel_size: int, stride: int):
        super().__init__(nn.Conv2d(cin, cout, kernel_size=kernel_size, stride=stride, padding=0, bias=True),
                         LayerNorm2d(cout, eps=1e-6))


CONVNEXT_TINY_SETTING = [(96, 192, 3), (192, 384, 3), (384, 768, 9), (768, None, 3)]


class ConvNeXt(nn.Module):
    def __init__(self, stochastic_depth_prob: float = 0.1, layer_scale: float = 1e-6):
        super().__init__()
        layers = [Conv2dNormActivation(3, 96, 4, 4)]
        total = sum(n for _, _, n in CONVNEXT_TINY_SETTING)
        bid = 0
        for cin, cout, n in CONVNEXT_TINY_SETTING:
            stage = []
            for _ in range(n):
                stage.append(CNBlock(cin, layer_scale, stochastic_depth_prob * bid / (total - 1.0)))
                bid += 1
            layers.append(nn.Sequential(*stage))
            if cout is not None:
                layers.append(nn.Sequential(LayerNorm2d(cin, eps=1e-6), nn.Conv2d(cin, cout, kernel_size=2, stride=2)))
        self.features = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(LayerNorm2d(768, eps=1e-6), nn.Flatten(1), nn.Linear(768, 1000))
        for m in self.modules():
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
        self._hip_pack: Dict = {}

    def hip_steps(self, x: Tensor):
        """The HIP forward as a block-by-block generator returning NHWC features."""
        return convnext_features_hip_steps(self.features, x, self._hip_pack,
                                           precision=getattr(self, "hip_precision", "fp32"))

    def forward(self, x: Tensor) -> Tensor:
        if use_hip(self):
            return nhwc_as_nchw(convnext_features_hip(self.features, x, self._hip_pack,
                                                      precision=getattr(self, "hip_precision", "fp32")))
        x = self.features(x)
        x = self.avgpool(x)
        return self.classifier(x)


def convnext_tiny(pretrained: bool = False) -> ConvNeXt:
    model = ConvNeXt(stochastic_depth_prob=0.1)
    if pretrained:
        _load_imagenet_weights(model)
    return model


def _load_imagenet_weights(model: nn.Module) -> None:
    """torchvision would download ConvNeXt_Tiny_Weights.DEFAULT (convnext_features.py:50);
    offline we only look in the torch hub cache, and otherwise keep the random init."""
    path = os.path.join(torch.hub.get_dir(), "checkpoints", "convnext_tiny-983f1562.pth")
    if os.path.exists(path):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        model.load_state_dict(sd, strict=True)
    else:
        warnings.warn("ImageNet ConvNeXt-tiny weights are unavailable offline; keeping random init "
                      "(load a trained PIP-Net checkpoint with load_state_dict).")


# ------------------------------------------------------------------------------------------
# reference wrappers (features/convnext_features.py)
# ------------------------------------------------------------------------------------------
def replace_convlayers_convnext(model: nn.Module, threshold: int) -> nn.Module:
    """features/convnext_features.py:5-15: stride-2 convs with in_channels > threshold -> stride 1."""
    for m in model.modules():
        if isinstance(m, nn.Conv2d) and m.stride[0] == 2 and m.in_channels > threshold:
            m.stride = tuple(s // 2 for s in m.stride)
    return model


class MidLayerConvNeXt(nn.Module):
    """features/convnext_features.py:17-36: stem + the first ``num_stages`` entries of features."""

    def __init__(self, original_model: nn.Module, num_stages: int = 2):
        super().__init__()
        self.features = nn.Sequential()
        if hasattr(original_model, "features") and len(original_model.features) > 0:
            self.features.add_module("0", original_model.features[0])
            for i in range(min(num_stages, len(original_model.features) - 1)):
                self.features.add_module(str(i + 1), original_model.features[i + 1])
        self._hip_pack: Dict = {}

    def hip_steps(self, x: Tensor):
        """The HIP forward as a block-by-block generator returning NHWC features."""
        return convnext_features_hip_steps(self.features, x, self._hip_pack,
                                           precision=getattr(self, "hip_precision", "fp32"))

    def forward(self, x: Tensor) -> Tensor:
        if use_hip(self):
            return nhwc_as_nchw(convnext_features_hip(self.features, x, self._hip_pack,
                                                      precision=getattr(self, "hip_precision", "fp32")))
        return self.features(x)


def _convnext_features(threshold: int, pretrained: bool, use_mid_layers: bool, num_stages: int) -> nn.Module:
    model = convnext_tiny(pretrained=pretrained)
    with torch.no_grad():
        model.avgpool = nn.Identity()
        model.classifier = nn.Identity()
        model = replace_convlayers_convnext(model, threshold)
        if use_mid_layers:
            model = MidLayerConvNeXt(model, num_stages=num_stages)
    return model


def convnext_tiny_26_features(pretrained: bool = False, use_mid_layers: bool = False, num_stages: int = 2, **kwargs):
    """features/convnext_features.py:38-65 (threshold 100 -> 26x26 grid at 224)."""
    return _convnext_features(100, pretrained, use_mid_layers, num_stages)


def convnext_tiny_13_features(pretrained: bool = False, use_mid_layers: bool = False, num_stages: int = 2, **kwargs):
    """features/convnext_features.py:67-94 (threshold 300 -> 13x13 grid at 224)."""
    return _convnext_features(300, pretrained, use_mid_layers, num_stages)


def get_feature_dimensions(use_mid_layers: bool = False, num_stages: int = 2, input_size: int = 224):
    """features/convnext_features.py:97-107 (shape probe on the torch path)."""
    model = convnext_tiny_26_features(pretrained=False, use_mid_layers=use_mid_layers, num_stages=num_stages)
    model.eval()
    with torch.no_grad():
        from .backend import torch_backend
        with torch_backend():
            return model(torch.zeros(1, 3, input_size, input_size)).shape


# ------------------------------------------------------------------------------------------
# HIP executor
# ------------------------------------------------------------------------------------------
def nhwc_as_nchw(x_nhwc: Tensor) -> Tensor:
    """[B,h,w,C] contiguous -> [B,C,h,w] view (channels_last strides, no copy)."""
    return x_nhwc.permute(0, 3, 1, 2)


def as_nhwc(x: Tensor) -> Tensor:
    """[B,C,h,w] -> contiguous [B,h,w,C] (free when x is channels_last, e.g. our own output)."""
    y = x.permute(0, 2, 3, 1)
    return y if y.is_contiguous() else y.contiguous()


def packed(cache: Dict, key: str, t: Tensor, fn) -> Tensor:
    """Device-layout copy of a parameter, rebuilt whenever the parameter changes
    (storage pointer or in-place version counter: callers mutate weights, test.py:73)."""
    stamp = (t.data_ptr(), t._version, tuple(t.shape))
    key = (key, str(t.device))          # replicas on several devices share one module dict
    ent = cache.get(key)
    if ent is None or ent[0] != stamp:
        with torch.no_grad():
            ent = (stamp, fn(t.detach()).contiguous())
        cache[key] = ent
        packed_ready()
    return ent[1]


FUSED_MLP = True      # tools / A-B runs may switch the fused narrow-stage MLP off
# (Round 4 measured the CNBlock GELU applied on Linear2's A-load instead of in Linear1's
# epilogue: bitwise the same outputs, C2 22.06 -> 24.31 ms per step, profiles/r04/
# ab_c2_defer_gelu.txt -- the packed GELU VALU between Linear2's MFMAs stalls them more than the
# epilogue does.  Removed from the library in round 5.)
# The fused MLP parallelises over pixels only (16 per wave): on small feature maps (C1's 64^2
# inputs: 256 / 64 pixels per image) the unfused GEMMs, which also spread the hidden dimension
# over workgroups, are faster.  The choice depends on the layer's C and h*w, never on the batch
# size, so per-pixel results stay batch-invariant.  (C = 192 at 16^2, C5's stage 2: fused
# ~100 us vs 115 unfused per block at batch 64, tools/ab_mlp.py.)
MLP_FUSED_MIN_PIXELS = {96: 512, 192: 256}


def _cnblock_hip(blk: CNBlock, h: Tensor, cache: Dict, key: str, row_scale: Optional[Tensor] = None) -> Tensor:
    """One CNBlock in place on NHWC ``h``.  ``row_scale`` (train mode, StochasticDepth "row"):
    device [B] = keep_b / (1 - p); the Linear2 epilogue scales each sample's branch by it
    (0 leaves a dropped sample's rows equal to the residual), so the batch stays one
    full-size GEMM (splitting it into kept runs measured slower: small-M grids underfill
    the 256 CUs)."""
    dw, ln, l1, l2 = blk.block[0], blk.block[2], blk.block[3], blk.block[5]
    b, hh, ww, c = h.shape
    if dw.kernel_size != (7, 7) or dw.padding != (3, 3) or dw.groups != c or dw.stride != (1, 1):
        raise RuntimeError(f"CNBlock {key}: unsupported depthwise conv {dw}")
    wdw = packed(cache, key + ".dw", dw.weight, lambda w: w.reshape(c, 49).t())
    t = K.dwconv7_ln(h, wdw, dw.bias, ln.weight, ln.bias)
    hv = h.view(-1, c)
    if row_scale is None and c in K.MLP_FUSED_CHANNELS and FUSED_MLP \
            and hh * ww >= MLP_FUSED_MIN_PIXELS[c]:
        # narrow stages: Linear1 + GELU + Linear2 + layer_scale + residual in one kernel
        K.cnblock_mlp(t.view(-1, c), l1.weight, l1.bias, l2.weight, l2.bias, blk.layer_scale.view(-1), hv, hw=hh * ww)
        return h
    m, hid = hv.shape[0], l1.weight.shape[0]
    u = K.linear(t.view(-1, c), l1.weight, l1.bias, _lib.EPI_BIAS_GELU)
    if row_scale is None:
        K.linear(u, l2.weight, l2.bias, _lib.EPI_RESID, scale=blk.layer_scale.view(-1), r=hv, out=hv)
    else:
        K.linear_rowscale(u, l2.weight, l2.bias, blk.layer_scale.view(-1), hv, row_scale, hh * ww)
    return h


def _cnblock_s3(blk: CNBlock, h: Tensor, cache: Dict, key: str) -> Tensor:
    """One CNBlock in place on NHWC fp32 ``h`` with split-bf16 GEMMs (precision "bf16x3"):
    dwconv+LN writes split planes [hi|lo], Linear1 (+GELU) reads them and writes its own
    output as split planes, Linear2 adds layer_scale * (.) into the fp32 residual stream."""
    dw, ln, l1, l2 = blk.block[0], blk.block[2], blk.block[3], blk.block[5]
    b, hh, ww, c = h.shape
    if dw.kernel_size != (7, 7) or dw.padding != (3, 3) or dw.groups != c or dw.stride != (1, 1):
        raise RuntimeError(f"CNBlock {key}: unsupported depthwise conv {dw}")
    hid = l1.out_features
    wdw = packed(cache, key + ".dw", dw.weight, lambda w: w.reshape(c, 49).t())
    w1 = packed(cache, key + ".fc1.s3", l1.weight, lambda w: K.split_planes_weight(w.view(hid, 1, 1, c)))
    w2 = packed(cache, key + ".fc2.s3", l2.weight, lambda w: K.split_planes_weight(w.view(c, 1, 1, hid)))
    t3 = K.dwconv7_ln_s3(h, wdw, dw.bias, ln.weight, ln.bias)
    u3 = K.conv_s3(t3, w1, 1, 1, hid, l1.bias, 1, 0, _lib.EPI_S3_GELU)
    K.conv_s3(u3, w2, 1, 1, c, l2.bias, 1, 0, _lib.EPI_F32_RESID, scale=blk.layer_scale.view(-1), r=h, out=h)
    return h


PRECISIONS = ("fp32", "bf16x3")


def stochastic_depth_row_scales(features: nn.Sequential, sd_keep: Dict[int, object], batch: int,
                                device) -> Dict[int, Tensor]:
    """Per-block device vectors keep_b / (1 - p) (float32, as StochasticDepth's
    ``noise.div_(1 - p)``) for the blocks with p > 0, staged through one pinned buffer and
    one asynchronous copy (no per-block synchronisation)."""
    blocks = [blk for mod in features if isinstance(mod, nn.Sequential) for blk in mod if isinstance(blk, CNBlock)]
    ids = [bid for bid, blk in enumerate(blocks) if blk.stochastic_depth.p > 0.0]
    if not ids:
        return {}
    host = torch.empty((len(ids), batch), dtype=torch.float32, pin_memory=torch.device(device).type == "cuda")
    for j, bid in enumerate(ids):
        mask = torch.as_tensor(sd_keep[bid]).reshape(-1)
        if mask.numel() != batch:
            raise RuntimeError(f"stochastic-depth mask of block {bid} has {mask.numel()} entries for batch {batch}")
        host[j] = mask.to(torch.float32).div_(1.0 - blocks[bid].stochastic_depth.p)
    dev = host.to(device, non_blocking=True)
    return {bid: dev[j] for j, bid in enumerate(ids)}


def convnext_features_hip(features: nn.Sequential, x: Tensor, cache: Dict,
                          sd_keep: Optional[Dict[int, object]] = None, precision: str = "fp32") -> Tensor:
    """Run a (possibly truncated, stride-patched) ConvNeXt ``features`` on the HIP kernels
    (convnext_features_hip_steps, drained)."""
    return drain(convnext_features_hip_steps(features, x, cache, sd_keep, precision))


def drain(steps):
    """Run a ``*_hip_steps`` generator to completion; its return value."""
    while True:
        try:
            next(steps)
        except StopIteration as e:
            return e.value


def convnext_features_hip_steps(features: nn.Sequential, x: Tensor, cache: Dict,
                                sd_keep: Optional[Dict[int, object]] = None, precision: str = "fp32"):
    """Generator form of convnext_features_hip: yields after the stem, every CNBlock and every
    downsample (the launches of that stage are enqueued by then), returns the NHWC features --
    so concurrent sub-batch forwards can enqueue block by block (pipnet._forward_hip_split).
    Run a (possibly truncated, stride-patched) ConvNeXt ``features`` on the HIP kernels.
    ``sd_keep``: train-mode stochastic depth, block id (0..17 in module order) -> per-sample
    keep mask for every block with p > 0 (eval / None: no stochastic depth).
    ``precision``: "fp32" (exact fp32 MFMA GEMMs) or "bf16x3" (the CNBlock Linears and the
    downsample convs as split-bf16 GEMMs, include/pipnet_amd.h; inference only -- train-mode
    stochastic depth always runs fp32)."""
    if precision not in PRECISIONS:
        raise ValueError(f"unknown HIP precision {precision!r} (expected one of {PRECISIONS})")
    s3 = precision == "bf16x3" and sd_keep is None
    K.require_device(x, "network input")
    x = x.contiguous()
    h = None
    bid = 0
    scales = None if sd_keep is None else stochastic_depth_row_scales(features, sd_keep, x.shape[0], x.device)
    for idx, mod in enumerate(features):
        name = str(idx)
        if idx == 0:
            conv, ln = mod[0], mod[1]
            if conv.kernel_size != (4, 4) or conv.stride != (4, 4) or conv.in_channels != 3 or conv.out_channels != 96:
                raise RuntimeError(f"unsupported ConvNeXt stem {conv}")
            h = K.convnext_stem(x, conv.weight, conv.bias, ln.weight, ln.bias)
            yield
        elif len(mod) > 0 and isinstance(mod[0], CNBlock):
            for j, blk in enumerate(mod):
                if s3:
                    h = _cnblock_s3(blk, h, cache, f"{name}.{j}")
                else:
                    h = _cnblock_hip(blk, h, cache, f"{name}.{j}", None if scales is None else scales.get(bid))
                bid += 1
                yield
        elif len(mod) == 2 and isinstance(mod[0], LayerNorm2d) and isinstance(mod[1], nn.Conv2d):
            ln, conv = mod[0], mod[1]
            if conv.kernel_size != (2, 2) or conv.padding != (0, 0):
                raise RuntimeError(f"unsupported ConvNeXt downsample {conv}")
            if s3 and conv.in_channels % 32 == 0:
                t3 = K.layernorm_s3(h, ln.weight, ln.bias)
                wp = packed(cache, name + ".conv.s3", conv.weight,
                            lambda w: K.split_planes_weight(w.permute(0, 2, 3, 1)))
                h = K.conv_s3(t3, wp, 2, 2, conv.out_channels, conv.bias, conv.stride[0], 0, _lib.EPI_F32_BIAS)
            else:
                t = K.layernorm(h, ln.weight, ln.bias)
                wp = packed(cache, name + ".conv", conv.weight, lambda w: w.permute(0, 2, 3, 1))
                h = K.conv2x2(t, wp, conv.bias, conv.stride[0])
            yield
        else:
            raise RuntimeError(f"unsupported ConvNeXt features entry {idx}: {type(mod).__name__}")
    return h
