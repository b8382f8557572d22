"""PIP-Net -- drop-in for ``pipnet/pipnet.py`` (model, NonNegLinear, factories).

``PIPNet.forward(xs, inference=False) -> (proto_features, pooled, out)`` keeps the
reference signature, attribute names (``_net``, ``_add_on``, ``_pool``,
``_classification``, ``_multiplier``, ``_num_*``) and ``state_dict`` keys.  In eval mode
with grad disabled the whole forward runs on HIP kernels:

  backbone (NHWC)  ->  [1x1 add-on on MFMA]  ->  fused per-patch softmax + spatial max-pool
  (proto map written once, channels_last)  ->  fused threshold + NonNegLinear.

``_classification.weight`` is read at call time (callers mutate it in place between
batches, ``pipnet/test.py:71-73``).
"""
from __future__ import annotations

import argparse

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from . import _lib
from . import kernels as K
from .backend import cross_stream_forward, use_hip
from .convnext_features import as_nhwc, convnext_tiny_13_features, convnext_tiny_26_features, nhwc_as_nchw
from .resnet_features import (resnet18_features, resnet34_features, resnet50_features, resnet50_features_inat,
                              resnet101_features, resnet152_features)

PRESENCE_THRESHOLD = 0.1   # pipnet.py:36
# The head as ONE launch (softmax_pool_linear: the classifier GEMV in each image's last workgroup)
# or as softmax_pool + nonneg_linear; bitwise equal.  The two-kernel form is the default: the
# one-launch form runs each image's 200-class GEMV serially in one workgroup at the end of the
# pooling kernel and measured C2 -0.5 %, C3 -3.9 % (profiles/r05/ab_fused_head.txt).
FUSED_HEAD = False


class PIPNet(nn.Module):
    def __init__(self, num_classes: int, num_prototypes: int, feature_net: nn.Module, args: argparse.Namespace,
                 add_on_layers: nn.Module, pool_layer: nn.Module, classification_layer: nn.Module):
        super().__init__()
        assert num_classes > 0
        self._num_features = args.num_features
        self._num_classes = num_classes
        self._num_prototypes = num_prototypes
        self._net = feature_net
        self._add_on = add_on_layers
        self._pool = pool_layer
        self._classification = classification_layer
        self._multiplier = classification_layer.normalization_multiplier

    def forward(self, xs: Tensor, inference: bool = False):
        if use_hip(self):
            return self._forward_hip(xs, inference)
        features = self._net(xs)
        proto_features = self._add_on(features)
        pooled = self._pool(proto_features)
        if inference:
            clamped_pooled = torch.where(pooled < PRESENCE_THRESHOLD, 0.0, pooled)
            return proto_features, clamped_pooled, self._classification(clamped_pooled)
        return proto_features, pooled, self._classification(pooled)

    # -- HIP inference path ---------------------------------------------------------------
    def _forward_hip(self, xs: Tensor, inference: bool):
        K.require_device(xs, "input images")
        if not (isinstance(self._pool, nn.Sequential) and isinstance(self._pool[0], nn.AdaptiveMaxPool2d)):
            raise RuntimeError("PIPNet HIP path expects _pool = Sequential(AdaptiveMaxPool2d(1), Flatten())")
        if stream_split(self, xs) > 1:
            with cross_stream_forward():
                return self._forward_hip_split(xs, inference, stream_split(self, xs))
        logits = self._hip_logits(xs)
        proto, pooled, clamped, out = self._hip_head(logits, inference)
        return nhwc_as_nchw(proto), (clamped if inference else pooled), out

    def _hip_logits(self, xs: Tensor) -> Tensor:
        feats = as_nhwc(self._net(xs))                     # [B,h,w,C] NHWC
        return add_on_logits_hip(self._add_on, feats)      # [B,h,w,P]

    def _hip_head(self, logits: Tensor, inference: bool, out=None):
        """softmax + max-pool (pipnet_softmax_pool_*), then threshold + NonNegLinear
        (pipnet_nonneg_linear_f32) -- or the same as one launch (FUSED_HEAD); ``out`` = (proto,
        pooled, clamped, logits) tensors to write into (batch slices of the split forward)."""
        cls = self._classification
        thresh = PRESENCE_THRESHOLD if inference else None
        if FUSED_HEAD:
            return K.softmax_pool_linear(logits, cls.weight, cls.bias, thresh, out=out)
        pool = K.softmax_pool_bf16 if logits.dtype == torch.bfloat16 else K.softmax_pool
        proto, pooled = pool(logits, 0, out=None if out is None else out[:2])
        clamped, res = K.nonneg_linear(pooled, cls.weight, cls.bias, thresh, out=None if out is None else out[2:])
        return proto, pooled, clamped, res

    def _forward_hip_split(self, xs: Tensor, inference: bool, n: int):
        """The batch as n concurrent sub-batches on n HIP streams: one sub-batch's
        bandwidth-bound kernels (depthwise conv + LayerNorm, LayerNorm, head) co-run on the CUs
        with another's MFMA-bound GEMMs.  Every kernel's result per image is independent of
        the batch it runs in (fixed K order, batch-invariant tile choice), so the outputs are
        bit-identical to the one-stream forward; the head writes straight into batch slices of
        the full outputs (no concatenation copy)."""
        dev = xs.device
        main = torch.cuda.current_stream(dev)
        streams = _side_streams(dev, n)
        parts = xs.chunk(n)
        for s in streams:
            s.wait_stream(main)
        net = self._net
        if INTERLEAVE and hasattr(net, "hip_steps") and use_hip(net):
            # enqueue the sub-batch forwards block by block, round robin, so every stream has
            # work from the start (enqueued one after the other, the second stream trailed the
            # first by the host's enqueue time of a whole backbone)
            feats = interleaved_features(net, parts, streams)
            logits = []
            for s, f in zip(streams, feats):
                with torch.cuda.stream(s):
                    logits.append(add_on_logits_hip(self._add_on, f))
        else:
            logits = []
            for s, p in zip(streams, parts):
                with torch.cuda.stream(s):
                    logits.append(self._hip_logits(p))
        b = xs.shape[0]
        _, h, w, pn = logits[0].shape
        k = self._classification.weight.shape[0]
        proto = torch.empty((b, h, w, pn), device=dev, dtype=torch.float32)
        pooled = torch.empty((b, pn), device=dev, dtype=torch.float32)
        clamped = torch.empty((b, pn), device=dev, dtype=torch.float32)
        out = torch.empty((b, k), device=dev, dtype=torch.float32)
        i0 = 0
        for s, lg in zip(streams, logits):
            i1 = i0 + lg.shape[0]
            s.wait_stream(main)                            # outputs allocated on main before any write
            with torch.cuda.stream(s):
                self._hip_head(lg, inference, out=(proto[i0:i1], pooled[i0:i1], clamped[i0:i1], out[i0:i1]))
            i0 = i1
        for s in streams:
            main.wait_stream(s)
        return nhwc_as_nchw(proto), (clamped if inference else pooled), out


# Concurrent sub-batches: batches of at least STREAM_SPLIT_MIN_BATCH images run as n
# half-batch forwards on n HIP streams, so one half's tile-quantisation tails and
# bandwidth-bound kernels co-run with the other half's MFMA tiles.  Default 2 for ResNet
# backbones (C3 bs=128: bf16 17.8k -> 20.1-20.3k img/s; 3 streams 19.6k) and for the full
# ConvNeXt PIP-Net (C2 bs=64: 2,933 -> 2,974-2,977 img/s; 3 streams 2,954-2,964), 1 for
# CountPIPNet / mid-layer backbones (C5 64 images: 55.8-56.1k -> 51.4-51.8k with 2 streams)
# -- profiles/r03/stream_split_ab.txt.  bench.py takes per-kernel roofline timings from a
# separate one-stream pass, where each launch runs alone.
STREAM_SPLIT_MIN_BATCH = 32
# Sub-batch forwards enqueued block by block, round robin (backbones with ``hip_steps``), rather
# than one whole backbone after the other.
INTERLEAVE = True
_SIDE_STREAMS = {}


def interleaved_features(net, parts, streams):
    """Backbone features of each sub-batch ``parts[i]`` on ``streams[i]``, enqueued one block at
    a time, round robin over the streams (``net.hip_steps`` yields after every block)."""
    gens = [net.hip_steps(p) for p in parts]
    feats = [None] * len(parts)
    live = list(range(len(parts)))
    while live:
        for i in list(live):
            with torch.cuda.stream(streams[i]):
                try:
                    next(gens[i])
                except StopIteration as e:
                    feats[i] = e.value
                    live.remove(i)
    return feats


def _side_streams(dev, n):
    key = (dev, n)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in range(n)]
    return _SIDE_STREAMS[key]


def set_stream_split(net: nn.Module, n: int) -> nn.Module:
    """Number of concurrent sub-batch streams for the HIP forward (1 = off; default 2 for
    ResNet and full ConvNeXt PIP-Net backbones, 1 otherwise).  Outputs are bit-identical either way (every kernel is
    batch-invariant)."""
    (net.module if hasattr(net, "module") else net)._hip_stream_split = int(n)
    return net


def stream_split(model: nn.Module, xs: Tensor) -> int:
    n = getattr(model, "_hip_stream_split", None)
    if n is None:
        from .convnext_features import ConvNeXt
        from .resnet_features import ResNet_features
        net = getattr(model, "_net", None)
        full_convnext = isinstance(net, ConvNeXt) and not hasattr(model, "_max_count")
        n = 2 if isinstance(net, ResNet_features) or full_convnext else 1
    if n <= 1 or xs.shape[0] < max(STREAM_SPLIT_MIN_BATCH, n):
        return 1
    return n


def add_on_logits_hip(add_on: nn.Module, feats: Tensor, activation=nn.Softmax) -> Tensor:
    """Apply the (optional) 1x1 prototype projection of ``_add_on`` on MFMA; returns NHWC
    logits.  The trailing activation module is applied by the caller's fused head kernel."""
    mods = list(add_on) if isinstance(add_on, nn.Sequential) else [add_on]
    if not mods or not isinstance(mods[-1], activation) or getattr(mods[-1], "dim", 1) != 1:
        raise RuntimeError(f"HIP head expects _add_on to end with {activation.__name__}(dim=1), got {add_on}")
    if len(mods) == 1:
        return feats
    conv = mods[0]
    if not (len(mods) == 2 and isinstance(conv, nn.Conv2d) and conv.kernel_size == (1, 1)
            and conv.stride == (1, 1) and conv.groups == 1):
        raise RuntimeError(f"HIP head expects _add_on = [Conv2d 1x1, activation], got {add_on}")
    b, h, w, c = feats.shape
    p = conv.out_channels
    if feats.dtype == torch.bfloat16:                    # bf16 build: 1x1 conv on bf16 MFMA
        from .convnext_features import packed
        cache = add_on.__dict__.setdefault("_hip_pack", {})
        wb = packed(cache, "add_on_bf16", conv.weight,
                    lambda t: K.pack_conv_weight_bf16(t.detach().view(p, 1, 1, c).float()))
        bias = conv.bias.detach().float().contiguous() if conv.bias is not None else None
        return K.conv2d_nhwc_bf16(feats, wb, 1, 1, bias, 1, 0, _lib.EPI_BIAS if bias is not None else _lib.EPI_NONE)
    y = K.linear(feats.view(-1, c), conv.weight.view(p, c), conv.bias,
                 _lib.EPI_BIAS if conv.bias is not None else _lib.EPI_NONE)
    return y.view(b, h, w, p)


base_architecture_to_features = {
    "resnet18": resnet18_features,
    "resnet34": resnet34_features,
    "resnet50": resnet50_features,
    "resnet50_inat": resnet50_features_inat,
    "resnet101": resnet101_features,
    "resnet152": resnet152_features,
    "convnext_tiny_26": convnext_tiny_26_features,
    "convnext_tiny_13": convnext_tiny_13_features,
}


class NonNegLinear(nn.Module):
    """pipnet.py:54-71: F.linear(x, relu(W), b); W uninitialised (torch.empty) like the reference."""

    def __init__(self, in_features: int, out_features: int, bias: bool = True, device=None, dtype=None) -> None:
        super().__init__()
        kw = {"device": device, "dtype": dtype}
        self.in_features = in_features
        self.out_features = out_features
        self.weight = nn.Parameter(torch.empty((out_features, in_features), **kw))
        self.normalization_multiplier = nn.Parameter(torch.ones((1,), requires_grad=True))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_features, **kw))
        else:
            self.register_parameter("bias", None)

    def forward(self, input: Tensor) -> Tensor:
        return F.linear(input, torch.relu(self.weight), self.bias)


def get_pip_network(num_classes: int, args: argparse.Namespace):
    """pipnet.py:74-115."""
    if "convnext" in args.net:
        backbone = base_architecture_to_features[args.net](
            pretrained=not args.disable_pretrained,
            use_mid_layers=getattr(args, "use_mid_layers", False),
            num_stages=getattr(args, "num_stages", 2))
    elif "res" in args.net:
        backbone = base_architecture_to_features[args.net](pretrained=not args.disable_pretrained)
    else:
        raise Exception("other base architecture NOT implemented")
    in_ch = [m for m in backbone.modules() if isinstance(m, nn.Conv2d)][-1].out_channels
    if args.num_features == 0:
        num_prototypes = in_ch
        print("Number of prototypes: ", num_prototypes, flush=True)
        add_on = nn.Sequential(nn.Softmax(dim=1))
    else:
        num_prototypes = args.num_features
        print("Number of prototypes set from", in_ch, "to", num_prototypes,
              ". Extra 1x1 conv layer added. Not recommended.", flush=True)
        add_on = nn.Sequential(
            nn.Conv2d(in_channels=in_ch, out_channels=num_prototypes, kernel_size=1, stride=1, padding=0, bias=True),
            nn.Softmax(dim=1))
    pool = nn.Sequential(nn.AdaptiveMaxPool2d(output_size=(1, 1)), nn.Flatten())
    classification = NonNegLinear(num_prototypes, num_classes, bias=bool(args.bias))
    return backbone, add_on, pool, classification, num_prototypes


def set_hip_dtype(model: nn.Module, dtype) -> nn.Module:
    """Select the compute dtype of the HIP inference path:
      * torch.float32 / "fp32" (default): exact fp32 arithmetic, parity with the reference;
      * torch.bfloat16 / "bf16": the BASELINE C3 ResNet build (bf16 activations);
      * "bf16x3": ConvNeXt backbones -- fp32 activations, the CNBlock Linears and downsample
        convs as split-bf16 GEMMs (x = hi + lo, three bf16 products, fp32 accumulation;
        ~1e-5 relative per product, include/pipnet_amd.h pipnet_conv2d_nhwc_s3)."""
    from .convnext_features import ConvNeXt, MidLayerConvNeXt
    from .resnet_features import ResNet_features
    if dtype in ("bf16x3", "split_bf16"):
        found = False
        for m in model.modules():
            if isinstance(m, (ConvNeXt, MidLayerConvNeXt)):
                m.hip_precision = "bf16x3"
                found = True
        if not found:
            raise ValueError("the bf16x3 HIP path is implemented for ConvNeXt backbones only")
        return model
    dtype = {"fp32": torch.float32, "f32": torch.float32, "bf16": torch.bfloat16}.get(dtype, dtype)
    if dtype not in (torch.float32, torch.bfloat16):
        raise ValueError(f"unsupported HIP compute dtype {dtype}")
    found = False
    for m in model.modules():
        if isinstance(m, ResNet_features):
            m.hip_dtype = dtype
            found = True
        if dtype == torch.float32 and isinstance(m, (ConvNeXt, MidLayerConvNeXt)):
            m.hip_precision = "fp32"
    if dtype == torch.bfloat16 and not found:
        raise ValueError("the bf16 HIP path is implemented for ResNet backbones only")
    return model


def get_pipnet(num_classes: int, args: argparse.Namespace):
    """pipnet.py:117-139 -> (PIPNet, num_prototypes).  Optional ``args.hip_dtype``
    ("fp32" | "bf16" | "bf16x3") selects the HIP compute dtype (see set_hip_dtype)."""
    feature_net, add_on, pool, classification, num_prototypes = get_pip_network(num_classes, args)
    model = PIPNet(num_classes=num_classes, num_prototypes=num_prototypes, feature_net=feature_net, args=args,
                   add_on_layers=add_on, pool_layer=pool, classification_layer=classification)
    if getattr(args, "hip_dtype", None):
        set_hip_dtype(model, args.hip_dtype)
    return model, num_prototypes
