"""ORACLE -- CPU restatement of the reference PIP-Net / CountPIPNet inference forward.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the checker
(or the timed CPU baseline) -- never as the product path.  The product path is the HIP
library in ``count_pipnet_amd/csrc`` and fails loudly when it is missing.

Pure functional torch (CPU, fp32, NCHW, the same ATen op sequence as the reference),
driven by a plain ``state_dict`` so it shares no code with the product's modules.
Each function cites the reference lines it restates.  Pinned against golden vectors
recorded from the reference itself (``tests/golden/gen_golden.py``); the ConvNeXt
arithmetic lives in third-party torchvision (absent, unpinned version)
and is restated from its published definition.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]

LN_EPS = 1e-6
# (dim_in, dim_out, n_blocks) of ConvNeXt-tiny, torchvision convnext_tiny
CONVNEXT_TINY = [(96, 192, 3), (192, 384, 3), (384, 768, 9), (768, None, 3)]


def _ln2d(x: Tensor, w: Tensor, b: Tensor) -> Tensor:
    """torchvision LayerNorm2d: permute -> F.layer_norm over C -> permute back."""
    return F.layer_norm(x.permute(0, 2, 3, 1), (x.shape[1],), w, b, LN_EPS).permute(0, 3, 1, 2)


def downsample_stride(net: str, in_channels: int) -> int:
    """features/convnext_features.py:5-15 -- a stride-2 conv whose ``in_channels``
    exceeds the threshold (100 for convnext_tiny_26 :61, 300 for convnext_tiny_13 :90)
    becomes stride 1."""
    threshold = {"convnext_tiny_26": 100, "convnext_tiny_13": 300}[net]
    return 1 if in_channels > threshold else 2


SD_PROB = 0.1          # torchvision convnext_tiny(stochastic_depth_prob=0.1)
N_BLOCKS = sum(n for _, _, n in CONVNEXT_TINY)


def sd_drop_prob(bid: int) -> float:
    """torchvision ConvNeXt: block ``bid`` (0..17 over all stages) drops its residual
    branch with p = 0.1 * bid / 17 in train mode (StochasticDepth "row")."""
    return SD_PROB * bid / (N_BLOCKS - 1.0)


def convnext_features(x: Tensor, sd: SD, prefix: str, net: str = "convnext_tiny_26",
                      use_mid_layers: bool = False, num_stages: int = 2,
                      sd_keep: Optional[Dict[int, Tensor]] = None) -> Tensor:
    """features/convnext_features.py:38-94 (+ MidLayerConvNeXt :17-36) over the
    torchvision ConvNeXt-tiny ``features`` Sequential.  ``sd_keep`` =
    train-mode stochastic depth: block id -> per-sample keep mask {0,1} [B] (blocks with
    p > 0); the branch is scaled by mask / (1 - p) as torchvision's StochasticDepth does."""
    p = prefix + "features."
    # stem: Conv2d k4 s4 + LayerNorm2d  (features.0)
    x = F.conv2d(x, sd[p + "0.0.weight"], sd[p + "0.0.bias"], stride=4)
    x = _ln2d(x, sd[p + "0.1.weight"], sd[p + "0.1.bias"])
    last = 7 if not use_mid_layers else min(num_stages, 7)      # MidLayerConvNeXt :27-31
    idx = 1
    bid = -1
    for cin, cout, n in CONVNEXT_TINY:
        if idx > last:
            break
        for j in range(n):                                       # CNBlock (torchvision)
            bid += 1
            q = f"{p}{idx}.{j}."
            y = F.conv2d(x, sd[q + "block.0.weight"], sd[q + "block.0.bias"], padding=3, groups=cin)
            y = y.permute(0, 2, 3, 1)
            y = F.layer_norm(y, (cin,), sd[q + "block.2.weight"], sd[q + "block.2.bias"], LN_EPS)
            y = F.linear(y, sd[q + "block.3.weight"], sd[q + "block.3.bias"])
            y = F.gelu(y)
            y = F.linear(y, sd[q + "block.5.weight"], sd[q + "block.5.bias"])
            y = y.permute(0, 3, 1, 2)
            y = sd[q + "layer_scale"] * y
            if sd_keep is not None and sd_drop_prob(bid) > 0.0:
                keep = 1.0 - sd_drop_prob(bid)
                y = y * (sd_keep[bid].to(y.dtype) / keep).view(-1, 1, 1, 1)
            x = y + x
        idx += 1
        if cout is None or idx > last:
            break
        q = f"{p}{idx}."                                         # downsample: LN2d + Conv k2
        x = _ln2d(x, sd[q + "0.weight"], sd[q + "0.bias"])
        x = F.conv2d(x, sd[q + "1.weight"], sd[q + "1.bias"], stride=downsample_stride(net, cin))
        idx += 1
    return x


def _bn(x: Tensor, sd: SD, q: str) -> Tensor:
    return F.batch_norm(x, sd[q + "running_mean"], sd[q + "running_var"], sd[q + "weight"],
                        sd[q + "bias"], training=False, momentum=0.0, eps=1e-5)


def resnet50_features(x: Tensor, sd: SD, prefix: str) -> Tensor:
    """features/resnet_features.py:126-229 with Bottleneck :77-124; layer3/layer4 at
    stride 1 (:153-154) so the 224x224 input gives a 28x28 grid; BN in eval mode."""
    p = prefix
    x = F.conv2d(x, sd[p + "conv1.weight"], stride=2, padding=3)
    x = F.relu(_bn(x, sd, p + "bn1."))
    x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
    for li, (n, stride) in enumerate([(3, 1), (4, 2), (6, 1), (3, 1)]):
        for j in range(n):
            q = f"{p}layer{li + 1}.{j}."
            s = stride if j == 0 else 1
            idt = x
            y = F.relu(_bn(F.conv2d(x, sd[q + "conv1.weight"]), sd, q + "bn1."))
            y = F.relu(_bn(F.conv2d(y, sd[q + "conv2.weight"], stride=s, padding=1), sd, q + "bn2."))
            y = _bn(F.conv2d(y, sd[q + "conv3.weight"]), sd, q + "bn3.")
            if (q + "downsample.0.weight") in sd:
                idt = _bn(F.conv2d(x, sd[q + "downsample.0.weight"], stride=s), sd, q + "downsample.1.")
            x = F.relu(y + idt)
    return x


def _bf(x: Tensor) -> Tensor:
    """Round to bfloat16 (nearest even) and back to fp32."""
    return x.to(torch.bfloat16).float()


def _conv_bn_bf16(x: Tensor, sd: SD, wkey: str, bnq: str, stride: int = 1, padding: int = 0) -> Tensor:
    """conv + eval BatchNorm of the bf16 build: BN folded in fp32 (w*g/sqrt(v+eps),
    b - mu*g/sqrt(v+eps)), folded weight rounded to bf16, fp32 accumulation, fp32 bias."""
    scale = sd[bnq + "weight"] / torch.sqrt(sd[bnq + "running_var"] + 1e-5)
    w = _bf(sd[wkey] * scale.view(-1, 1, 1, 1))
    b = sd[bnq + "bias"] - sd[bnq + "running_mean"] * scale
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def resnet50_features_bf16(x: Tensor, sd: SD, prefix: str) -> Tensor:
    """The bf16 build of resnet50_features (BASELINE C3; the reference itself is fp32 only,
    so this restates the build's arithmetic -- input and every conv output rounded to
    bf16, epilogue bias / residual / ReLU in fp32 before the rounding).  Returns fp32
    tensors holding bf16 values."""
    p = prefix
    x = _bf(x)
    x = _bf(F.relu(_conv_bn_bf16(x, sd, p + "conv1.weight", p + "bn1.", 2, 3)))
    x = F.max_pool2d(x, kernel_size=3, stride=2, padding=1)
    for li, (n, stride) in enumerate([(3, 1), (4, 2), (6, 1), (3, 1)]):
        for j in range(n):
            q = f"{p}layer{li + 1}.{j}."
            s = stride if j == 0 else 1
            idt = x
            if (q + "downsample.0.weight") in sd:
                idt = _bf(_conv_bn_bf16(x, sd, q + "downsample.0.weight", q + "downsample.1.", s))
            y = _bf(F.relu(_conv_bn_bf16(x, sd, q + "conv1.weight", q + "bn1.")))
            y = _bf(F.relu(_conv_bn_bf16(y, sd, q + "conv2.weight", q + "bn2.", s, 1)))
            x = _bf(F.relu(_conv_bn_bf16(y, sd, q + "conv3.weight", q + "bn3.") + idt))
    return x


def pipnet_forward_bf16(xs: Tensor, sd: SD, cfg, inference: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """pipnet_forward with the bf16 ResNet build (optional 1x1 add-on also bf16 with fp32
    bias, rounded); softmax / pool / classifier in fp32 as in the build's head."""
    if cfg.net != "resnet50":
        raise ValueError("oracle: the bf16 build covers resnet50 only")
    feats = resnet50_features_bf16(xs, sd, "_net.")
    if getattr(cfg, "num_features", 0):
        feats = _bf(F.conv2d(feats, _bf(sd["_add_on.0.weight"]), sd["_add_on.0.bias"]))
    proto = torch.softmax(feats, dim=1)
    pooled = torch.amax(proto, dim=(2, 3))
    if inference:
        pooled = torch.where(pooled < 0.1, 0.0, pooled)
    out = non_neg_linear(pooled, sd["_classification.weight"], sd.get("_classification.bias"))
    return proto, pooled, out


def backbone(x: Tensor, sd: SD, cfg, sd_keep: Optional[Dict[int, Tensor]] = None) -> Tensor:
    if "convnext" in cfg.net:
        return convnext_features(x, sd, "_net.", cfg.net, getattr(cfg, "use_mid_layers", False),
                                 getattr(cfg, "num_stages", 2), sd_keep)
    if cfg.net == "resnet50":
        return resnet50_features(x, sd, "_net.")
    raise ValueError(f"oracle: unsupported net {cfg.net}")


def non_neg_linear(x: Tensor, w: Tensor, b: Optional[Tensor]) -> Tensor:
    """pipnet/pipnet.py:70-71, pipnet/count_pipnet.py:224 -- F.linear(x, relu(W), b)."""
    return F.linear(x, torch.relu(w), b)


def pipnet_forward(xs: Tensor, sd: SD, cfg, inference: bool = False,
                   sd_keep: Optional[Dict[int, Tensor]] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """pipnet/pipnet.py:31-41 with the add-on / pool of get_pip_network :92-108
    (``sd_keep``: train-mode stochastic depth masks, see convnext_features)."""
    feats = backbone(xs, sd, cfg, sd_keep)
    if getattr(cfg, "num_features", 0):
        feats = F.conv2d(feats, sd["_add_on.0.weight"], sd["_add_on.0.bias"])
    proto = torch.softmax(feats, dim=1)                          # nn.Softmax(dim=1)
    pooled = torch.amax(proto, dim=(2, 3))                       # AdaptiveMaxPool2d(1)+Flatten
    if inference:
        pooled = torch.where(pooled < 0.1, 0.0, pooled)          # pipnet.py:36
    out = non_neg_linear(pooled, sd["_classification.weight"], sd.get("_classification.bias"))
    return proto, pooled, out


def gumbel_softmax_hard(logits: Tensor, exp_noise: Tensor, tau: float = 1.0, dim: int = 1) -> Tensor:
    """torch.nn.functional.gumbel_softmax(hard=True) with the Exp(1) draw injected
    (count_pipnet_utils.py:36-38 -> torch functional.py gumbel_softmax)."""
    gumbels = -exp_noise.log()
    y_soft = ((logits + gumbels) / tau).softmax(dim)
    index = y_soft.max(dim, keepdim=True)[1]
    y_hard = torch.zeros_like(logits).scatter_(dim, index, 1.0)
    return y_hard - y_soft + y_soft


def modified_encoding(x: Tensor, max_count: int) -> Tensor:
    """count_pipnet_utils.py:141-185 -- count c>0.1 -> one-hot at clamp(int(c)-1, 0, C-1)."""
    b, p = x.shape
    enc = torch.zeros(b, p, max_count)
    nz = x > 0.1
    idx = torch.clamp(x.long() - 1, 0, max_count - 1)
    enc.scatter_(2, idx.unsqueeze(2), nz.unsqueeze(2).float())
    return enc


def intermediate(counts: Tensor, sd: SD, cfg, num_prototypes: int) -> Tensor:
    """count_pipnet.py:393-417 -- identity / onehot / bilinear / linear / linear_full."""
    kind = getattr(cfg, "intermediate_layer", "onehot")
    mc = int(getattr(cfg, "max_count", 3))
    if kind == "identity":                                       # count_pipnet_utils.py:446-469
        return counts
    if kind == "onehot":                                         # :86-139 (+ ModifiedSTEFunction :201-217)
        x = counts.round() if getattr(cfg, "use_ste", True) else counts
        return modified_encoding(x, mc).reshape(counts.shape[0], -1)
    if kind == "bilinear":                                       # :323-385
        e = F.linear(counts, sd["_intermediate.embed.weight"])
        return F.linear(e, sd["_intermediate.W.weight"]) * F.linear(e, sd["_intermediate.V.weight"])
    if kind == "linear":                                         # :471-539
        w = sd["_intermediate.linear.weight"]                    # [C, 1]
        return F.linear(counts.reshape(-1, 1), w).reshape(counts.shape[0], -1)
    if kind == "linear_full":                                    # :387-444
        return F.linear(counts, sd["_intermediate.linear.weight"])
    raise ValueError(f"Unknown intermediate layer type: {kind}")


def count_pipnet_forward(xs: Tensor, sd: SD, cfg, inference: bool = False,
                         exp_noise: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor]:
    """pipnet/count_pipnet.py:70-110 (eval mode: GumbelSoftmax hard, count_pipnet_utils.py:36-38)."""
    feats = backbone(xs, sd, cfg)
    if getattr(cfg, "num_features", 0):
        feats = F.conv2d(feats, sd["_add_on.0.weight"], sd["_add_on.0.bias"])
    if getattr(cfg, "activation", "gumbel_softmax") == "softmax":
        proto = torch.softmax(feats, dim=1)
    else:
        if exp_noise is None:
            raise ValueError("oracle: gumbel_softmax needs the injected Exp(1) noise")
        proto = gumbel_softmax_hard(feats, exp_noise, tau=float(getattr(cfg, "tau", 1.0)))
    counts = proto.sum(dim=(2, 3))                                # :88
    mc = int(getattr(cfg, "max_count", 3))
    if getattr(cfg, "use_ste", True):
        clamped = counts.round().clamp(0, mc)                     # STE_Round / ClampSTE forward
    else:
        clamped = torch.clamp(counts.round() if inference else counts, 0, mc)
    inter = intermediate(clamped, sd, cfg, proto.shape[1])
    out = non_neg_linear(inter, sd["_classification.weight"], sd.get("_classification.bias"))
    return (proto, clamped, out) if inference else (proto, counts, out)


def gflop_per_image(cfg, image_size: int) -> float:
    """Algorithmic GFLOP (2 x MAC) of the ConvNeXt backbone + 1x1 add-on per image
    (40.09 for convnext_tiny_26 at 224)."""
    if "convnext" not in cfg.net:
        raise ValueError("gflop_per_image: convnext only")
    h = image_size // 4
    flops = 2.0 * h * h * 96 * 48
    last = 7 if not getattr(cfg, "use_mid_layers", False) else min(getattr(cfg, "num_stages", 2), 7)
    idx, c = 1, 96
    for cin, cout, n in CONVNEXT_TINY:
        if idx > last:
            break
        flops += n * h * h * (2 * 49 * cin + 2 * 2 * cin * 4 * cin)
        idx += 1
        if cout is None or idx > last:
            break
        h = (h - 2) // downsample_stride(cfg.net, cin) + 1
        flops += 2.0 * h * h * cout * 4 * cin
        c = cout
        idx += 1
    nf = getattr(cfg, "num_features", 0)
    if nf:
        flops += 2.0 * h * h * c * nf
    return flops / 1e9


# ---- eval_pipnet metric loop (pipnet/test.py:67-131, 278-319) -------------------------------

def eval_batch_metrics(pooled: Tensor, out: Tensor, w: Tensor, ys: Tensor, multiplier: float,
                       thr: float = 1e-3) -> dict:
    """The per-batch body of eval_pipnet after the forward (test.py:77-131): returns the
    values the reference accumulates (as Python floats, exactly as its ``.item()`` calls)
    and the per-image predictions / confidences.  ``w`` [K, P] is the weight the
    reference multiplies ``pooled`` with (classification weight or count importances)."""
    max_out_score, ys_pred = torch.max(out, dim=1)
    scores_conf = torch.amax(F.softmax(torch.log1p(out ** multiplier), dim=1), dim=1)
    abstained = int(max_out_score.shape[0] - torch.count_nonzero(max_out_score))
    scores = pooled * w.unsqueeze(1).repeat(1, pooled.shape[0], 1)          # [K, B, P]
    relevant = torch.abs(scores) > thr
    any_sizes = relevant.any(dim=0).sum(dim=1).float()
    pred_sizes = torch.diagonal(torch.index_select(relevant.sum(dim=2).float(), 0, ys_pred))
    ppc = torch.count_nonzero(torch.gt(torch.relu(scores - thr).mean(dim=1), 0.).float(), dim=1).float()
    anz = torch.count_nonzero(torch.gt(torch.abs(pooled), thr).float(), dim=1).float()
    _, pred = out.topk(1, 1, True, True)
    top1 = (pred.t() == ys.unsqueeze(0)).reshape(-1).float()
    return dict(pred_size=pred_sizes.mean(0).item(), any_size=any_sizes.mean(0).item(),
                ppc=ppc.mean(0).item(), anz=anz.mean().item(), top1=torch.mean(top1).item(),
                abstained=abstained, ys_pred=ys_pred, conf=scores_conf)


def eval_loop(batches, num_classes: int, multiplier: float, thr: float = 1e-3) -> dict:
    """Accumulate eval_batch_metrics over ``batches`` = [(pooled, out, w, ys)] like
    eval_pipnet (test.py:136-157): running Python-float sums / number of batches."""
    import numpy as np
    cm = np.zeros((num_classes, num_classes), dtype=int)
    s = dict(pred_size=0., any_size=0., ppc=0., anz=0., top1=0.)
    abstained = 0
    for pooled, out, w, ys in batches:
        r = eval_batch_metrics(pooled, out, w, ys, multiplier, thr)
        for k in s:
            s[k] += r[k]
        abstained += r["abstained"]
        for yp, yt in zip(r["ys_pred"].tolist(), ys.tolist()):
            cm[yt][yp] += 1
    n = len(batches)
    total = cm.sum()
    return {"confusion_matrix": cm, "test_accuracy": (np.trace(cm) / total) if total else 1,
            "top1_accuracy": s["top1"] / n, "local_size_for_true_class": s["pred_size"] / n,
            "local_size_for_all_classes": s["any_size"] / n, "prototypes_per_class": s["ppc"] / n,
            "almost_nonzeros": s["anz"] / n, "abstained": abstained}
