"""CountPIPNet -- drop-in for ``pipnet/count_pipnet.py`` (model, NonNegLinear, factory).

``CountPIPNet.forward(xs, inference=False) -> (proto_features, counts | clamped_counts, out)``
keeps the reference signature, attributes (``_max_count`` is the "is count net" probe of
``pipnet/test.py:27``) and ``state_dict`` keys.  Eval + no-grad runs on HIP kernels:

  backbone (NHWC) -> 1x1 add-on (MFMA) -> fused hard Gumbel-softmax + per-prototype count
  (Philox4x32 Exp(1) noise in-kernel, or an injected draw) -> round / clamp ->
  intermediate (identity / one-hot / linear / linear_full / bilinear on MFMA) -> NonNegLinear.
"""
from __future__ import annotations

import argparse
import math
from typing import Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from . import kernels as K
from .backend import cross_stream_forward, packed_ready, use_hip
from .convnext_features import as_nhwc, convnext_tiny_13_features, convnext_tiny_26_features, nhwc_as_nchw
from .count_pipnet_utils import (BilinearIntermediate, ClampSTE, GumbelSoftmax, IdentityIntermediate,
                                 LinearFull, LinearIntermediate, OneHotEncoder, STE_Round)
from . import pipnet as _pipnet
from .pipnet import _side_streams, add_on_logits_hip, interleaved_features, stream_split


class CountPIPNet(nn.Module):
    """count_pipnet.py:14-168."""

    def __init__(self, num_classes: int, num_prototypes: int, feature_net: nn.Module, args: argparse.Namespace,
                 add_on_layers: nn.Module, intermediate_layer: nn.Module, classification_layer: nn.Module,
                 max_count: int = 3, use_ste: bool = True, backward_clamp_strategy: str = "Identity"):
        super().__init__()
        assert num_classes > 0
        self._num_features = args.num_features
        self._num_classes = num_classes
        self._num_prototypes = num_prototypes
        self._net = feature_net
        self._add_on = add_on_layers
        self._classification = classification_layer
        self._intermediate = intermediate_layer
        assert backward_clamp_strategy in ["Identity", "Gated"]
        print(f"Using backward clamp strategy: {backward_clamp_strategy}", flush=True)
        self._is_clamp_backward_identity = backward_clamp_strategy == "Identity"
        self._max_count = max_count
        self._use_ste = use_ste
        self._multiplier = classification_layer.normalization_multiplier
        self.ste_round = STE_Round.apply
        self.ste_clamp = ClampSTE.apply

    def forward(self, xs, inference=False):
        if use_hip(self):
            return self._forward_hip(xs, inference)
        features = self._net(xs)
        proto_features = self._add_on(features)
        counts = proto_features.sum(dim=(2, 3))
        if self._use_ste:
            clamped = self.ste_clamp(self.ste_round(counts), 0, self._max_count, self._is_clamp_backward_identity)
        else:
            clamped = torch.clamp(counts.round() if inference else counts, 0, self._max_count)
        out = self._classification(self._intermediate(clamped))
        return (proto_features, clamped, out) if inference else (proto_features, counts, out)

    # -- HIP inference path ---------------------------------------------------------------
    def _forward_hip(self, xs, inference):
        K.require_device(xs, "input images")
        n = stream_split(self, xs)
        # (the Philox offset of a sub-batch, b0*h*w*P/4 blocks, is exact for P % 4 == 0)
        if n > 1 and self._num_prototypes % 4 == 0 and not torch.cuda.is_current_stream_capturing():
            with cross_stream_forward():
                return self._forward_hip_split(xs, inference, n)
        feats = as_nhwc(self._net(xs))
        act = list(self._add_on)[-1] if isinstance(self._add_on, nn.Sequential) else self._add_on
        do_round = bool(self._use_ste or inference)
        if isinstance(act, GumbelSoftmax):
            logits = add_on_logits_hip(self._add_on, feats, activation=GumbelSoftmax)
            noise = act.exp_noise
            if noise is not None:
                noise = noise.to(device=logits.device, dtype=torch.float32).contiguous()
                proto, hist = K.count_gumbel(logits, act.tau, noise, 0)
            elif torch.cuda.is_current_stream_capturing():
                # HIP-graph capture: the key must live in device memory so that every replay
                # draws fresh noise (count_pipnet_amd.graph)
                proto, hist = K.count_gumbel_devseed(logits, act.tau, self._graph_seed_state(logits.device))
            else:
                seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())   # fresh noise per call
                proto, hist = K.count_gumbel(logits, act.tau, None, seed)
            counts, clamped = K.count_finish(hist, None, self._max_count, do_round)
        else:
            logits = add_on_logits_hip(self._add_on, feats, activation=nn.Softmax)
            proto, sums = K.softmax_pool(logits, pool_mode=1)
            counts, clamped = K.count_finish(None, sums, self._max_count, do_round)
        inter = intermediate_hip(self._intermediate, clamped)
        cls = self._classification
        _, out = K.nonneg_linear(inter, cls.weight, cls.bias, None)
        return nhwc_as_nchw(proto), (clamped if inference else counts), out

    def _forward_hip_split(self, xs, inference, n):
        """The backbone, add-on and count head of n sub-batches on n concurrent HIP streams
        (pipnet.PIPNet._forward_hip_split), joined before the count -> classifier layers, which
        run once on the whole batch (the Bilinear intermediate streams 101 MB of folded weights
        per call).  Per-image results are batch-invariant and the Gumbel noise of sub-batch image
        b0 starts at Philox block b0*h*w*P/4, so the outputs equal the one-stream forward's."""
        dev = xs.device
        main = torch.cuda.current_stream(dev)
        streams = _side_streams(dev, n)
        parts = xs.chunk(n)
        act = list(self._add_on)[-1] if isinstance(self._add_on, nn.Sequential) else self._add_on
        gumbel = isinstance(act, GumbelSoftmax)
        kind = GumbelSoftmax if gumbel else nn.Softmax
        for s in streams:
            s.wait_stream(main)
        if _pipnet.INTERLEAVE and hasattr(self._net, "hip_steps") and use_hip(self._net):
            feats = interleaved_features(self._net, parts, streams)
        else:
            feats = []
            for s, p in zip(streams, parts):
                with torch.cuda.stream(s):
                    feats.append(as_nhwc(self._net(p)))
        logits = []
        for s, f in zip(streams, feats):
            with torch.cuda.stream(s):
                logits.append(add_on_logits_hip(self._add_on, f, activation=kind))
        b = xs.shape[0]
        _, h, w, pn = logits[0].shape
        proto = torch.empty((b, h, w, pn), device=dev, dtype=torch.float32)
        noise = seed = None
        if gumbel:
            hist = torch.empty((b, pn), device=dev, dtype=torch.int32)
            noise = act.exp_noise
            if noise is not None:
                noise = noise.to(device=dev, dtype=torch.float32).contiguous()
            else:
                seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
        else:
            sums = torch.empty((b, pn), device=dev, dtype=torch.float32)
        i0 = 0
        for s, lg in zip(streams, logits):
            i1 = i0 + lg.shape[0]
            s.wait_stream(main)                            # outputs allocated on main before any write
            with torch.cuda.stream(s):
                if gumbel:
                    K.count_gumbel(lg, act.tau, None if noise is None else noise[i0:i1], seed or 0,
                                   offset=i0 * h * w * pn // 4, out=(proto[i0:i1], hist[i0:i1]))
                else:
                    K.softmax_pool(lg, pool_mode=1, out=(proto[i0:i1], sums[i0:i1]))
            i0 = i1
        for s in streams:
            main.wait_stream(s)
        do_round = bool(self._use_ste or inference)
        counts, clamped = K.count_finish(hist if gumbel else None, None if gumbel else sums, self._max_count,
                                         do_round)
        inter = intermediate_hip(self._intermediate, clamped)
        cls = self._classification
        _, out = K.nonneg_linear(inter, cls.weight, cls.bias, None)
        return nhwc_as_nchw(proto), (clamped if inference else counts), out

    def _graph_seed_state(self, device):
        st = getattr(self, "_hip_seed_state", None)
        if st is None or st.device != device:
            seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
            st = torch.tensor([seed, 0], dtype=torch.int64, device=device)
            self._hip_seed_state = st           # plain attribute: not a parameter / buffer
        return st

    def _calculate_counts_for_testing(self, proto_features):
        return proto_features.sum(dim=(2, 3))

    def get_prototype_importance_per_class(self, prototype_idx, classifier_input_scalars=None):
        """count_pipnet.py:126-147."""
        w_in = self._intermediate.prototype_to_classifier_input_weights(prototype_idx)
        if classifier_input_scalars is not None:
            assert classifier_input_scalars.shape == w_in.shape, \
                f"Classifier input scalars must have the same shape as the classifier input weights " \
                f"{tuple(w_in.shape)} vs {tuple(classifier_input_scalars.shape)}"
            w_in = w_in * classifier_input_scalars
        return torch.einsum("d,kd->k", torch.abs(w_in).to(self._classification.weight.device),
                            self._classification.weight)

    def get_prototype_importance(self, prototype_idx):
        return self.get_prototype_importance_per_class(prototype_idx).sum().item()

    def update_temperature(self, new_temperature):
        for module in self._add_on.modules():
            if isinstance(module, GumbelSoftmax):
                module.tau = new_temperature
                break


def intermediate_hip(layer: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """HIP forward of the count -> classifier-input layers (count_pipnet.py:393-417)."""
    if isinstance(layer, IdentityIntermediate):
        return x
    if isinstance(layer, OneHotEncoder):
        return K.count_encode(x, layer.num_bins, kind=0, do_round=layer.use_ste)
    if isinstance(layer, LinearIntermediate):
        w = layer.linear.weight[:, 0].contiguous()
        return K.count_encode(x, layer.expansion_factor, kind=1, do_round=False, w=w)
    if isinstance(layer, LinearFull):
        return K.linear(x, layer.linear.weight)
    if isinstance(layer, BilinearIntermediate):
        wf, vf, pair = _bilinear_folded(layer)
        if (BILINEAR_PAIR and x.shape[1] % 32 == 0 and wf.shape[0] % 4 == 0 and x.stride(0) % 4 == 0
                and x.stride(1) == 1 and x.data_ptr() % 16 == 0):    # else the two-GEMM form
            return K.linear_pair_mul(x, pair)     # one split-K GEMM over [W E; V E] + one product reduction
        we = K.linear(x, wf)
        return K.linear(x, vf, epilogue=_lib.EPI_MUL, r=we)
    raise RuntimeError(f"CountPIPNet HIP path: unsupported intermediate layer {type(layer).__name__}")


# BilinearIntermediate at inference: both folded products as ONE split-K GEMM over the stacked
# [W E; V E] weights whose reduction multiplies the two halves (K.linear_pair_mul; needs P % 32 == 0
# and D % 4 == 0), else as two GEMMs with the product in the second's epilogue (also the A/B arm;
# the same products, slab sums may group differently).
BILINEAR_PAIR = True


def _bilinear_folded(layer: BilinearIntermediate) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """W(embed(x)) * V(embed(x)) (count_pipnet_utils.py:378-385) with the embedding folded into
    both projections: the three Linears carry no bias and nothing sits between embed and W / V,
    so W(E x) = (W E) x.  The folded [D, P] weights (W E, V E; products taken in fp64, rounded
    once to fp32) turn the inference intermediate into two M = batch GEMMs with K = P that
    stream 2 D P instead of D P + 2 D^2 weight floats (C5: 101 MB instead of 352 MB, 3.5x fewer
    FLOPs) -- the same kind of inference-time fold as the BatchNorm fold of the ResNet path.
    Both products run as one launch of the in-tree fp64 MFMA kernel (``K.matmul2_f64acc``), never
    a vendor GEMM.
    Rebuilt whenever any of the three weights changes (storage pointer / in-place version); a
    write through ``param.data`` bypasses the version counter -- call
    ``count_pipnet_amd.invalidate_weight_caches(net)`` after one (backend.py)."""
    ts = (layer.embed.weight, layer.W.weight, layer.V.weight)
    stamp = tuple((t.data_ptr(), t._version, tuple(t.shape)) for t in ts)
    cache = layer.__dict__.setdefault("_hip_fold_cache", {})   # plain attribute, not a buffer
    key = str(layer.W.weight.device)
    ent = cache.get(key)
    if ent is None or ent[0] != stamp:
        with torch.no_grad():
            e = layer.embed.weight.detach().contiguous()
            pair = K.matmul2_f64acc(layer.W.weight.detach().contiguous(), layer.V.weight.detach().contiguous(), e)
        ent = (stamp, (pair[0], pair[1], pair.view(-1, pair.shape[2])))    # [W E; V E] stacked: [2 D, P]
        cache[key] = ent
        packed_ready()
    return ent[1]


base_architecture_to_features = {
    "convnext_tiny_26": convnext_tiny_26_features,
    "convnext_tiny_13": convnext_tiny_13_features,
}


class NonNegLinear(nn.Module):
    """count_pipnet.py:176-224 (Kaiming-uniform init, unlike pipnet.py's uninitialised one)."""

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
        self.reset_parameters()

    def reset_parameters(self) -> None:
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1 / math.sqrt(self.weight.shape[1]) if self.weight.shape[1] > 0 else 0
            nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, input: torch.Tensor) -> torch.Tensor:
        return F.linear(input, torch.relu(self.weight), self.bias)


def detect_output_channels(features: nn.Module) -> int:
    """count_pipnet.py:438-464: out_channels of the last Conv2d of the last features stage."""
    if hasattr(features, "features") and len(features.features) > 0:
        last_conv = None
        for m in features.features[-1].modules():
            if isinstance(m, nn.Conv2d):
                last_conv = m
        if last_conv is not None:
            print(f"Detected {last_conv.out_channels} output channels from last conv layer", flush=True)
            return last_conv.out_channels
    raise RuntimeError("Could not detect output channels from the feature extractor.")


def get_count_network(num_classes: int, args: argparse.Namespace, max_count: int = 3, use_ste: bool = True,
                      device=None):
    """count_pipnet.py:324-436 -> (CountPIPNet, num_prototypes).  Optional ``args.hip_dtype``
    ("fp32" | "bf16x3") selects the HIP compute dtype of the ConvNeXt backbone."""
    if args.net not in base_architecture_to_features:
        raise ValueError(f"Network '{args.net}' is not supported. "
                         f"Supported networks: {list(base_architecture_to_features)}")
    features = base_architecture_to_features[args.net](
        pretrained=not args.disable_pretrained,
        use_mid_layers=getattr(args, "use_mid_layers", False),
        num_stages=getattr(args, "num_stages", 2))
    in_ch = detect_output_channels(features)
    activation = getattr(args, "activation", "gumbel_softmax")
    act = nn.Softmax(dim=1) if activation == "softmax" else GumbelSoftmax(dim=1, tau=1.0)
    if args.num_features == 0:
        num_prototypes = in_ch
        print(f"Number of prototypes: {num_prototypes}", flush=True)
        add_on = nn.Sequential(act)
    else:
        num_prototypes = args.num_features
        print(f"Number of prototypes set from {in_ch} to {num_prototypes}. Extra 1x1 conv layer added.", flush=True)
        add_on = nn.Sequential(nn.Conv2d(in_ch, num_prototypes, kernel_size=1, stride=1, padding=0, bias=True), act)
    kind = getattr(args, "intermediate_layer", "onehot")
    positive_grad_strategy = getattr(args, "positive_grad_strategy", None)
    print(f"Using positive gradient strategy: {positive_grad_strategy}", flush=True)
    backward_clamp_strategy = getattr(args, "backward_clamp_strategy", "Gated")
    if kind == "linear":
        inter, dim = LinearIntermediate(num_prototypes, max_count), num_prototypes * max_count
    elif kind == "linear_full":
        inter, dim = LinearFull(num_prototypes, max_count), num_prototypes * max_count
    elif kind == "bilinear":
        inter, dim = BilinearIntermediate(num_prototypes, max_count), num_prototypes * max_count
    elif kind == "onehot":
        inter = OneHotEncoder(max_count, use_ste=use_ste, respect_active_grad=False, num_prototypes=num_prototypes,
                              device=device, positive_grad_strategy=positive_grad_strategy)
        dim = num_prototypes * max_count
    elif kind == "identity":
        inter, dim = IdentityIntermediate(num_prototypes, device=device), num_prototypes
    else:
        raise ValueError(f"Unknown intermediate layer type: {kind}")
    classification = NonNegLinear(dim, num_classes, bias=getattr(args, "bias", False))
    model = CountPIPNet(num_classes=num_classes, num_prototypes=num_prototypes, feature_net=features, args=args,
                        add_on_layers=add_on, classification_layer=classification, intermediate_layer=inter,
                        max_count=max_count, use_ste=use_ste, backward_clamp_strategy=backward_clamp_strategy)
    if getattr(args, "hip_dtype", None):          # optional HIP compute dtype (pipnet.set_hip_dtype)
        from .pipnet import set_hip_dtype
        set_hip_dtype(model, args.hip_dtype)
    return model, num_prototypes
