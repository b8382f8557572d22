"""Platform-stable synthetic weights and inputs (no network: no checkpoints, no datasets).

Every tensor is drawn from its own numpy PCG64 stream keyed by ``(seed, crc32(name))``,
so the values do not depend on dict order, torch version or host.  Two profiles:

* ``"init"``     -- the reference's own initialisation scales (torchvision ConvNeXt
                    ``trunc_normal_(std=0.02)``, ``layer_scale = 1e-6``).  Inference logits
                    are ~0 with this profile, so it is only a smoke case.
* ``"trained"``  -- "trained-like" magnitudes: fan-in scaled conv/linear weights, O(1)
                    layer scales, classifier ``N(1, 0.1)`` as ``main.py:168`` initialises it.
                    Prototype presence above the 0.1 threshold is a few percent, like a
                    trained PIP-Net, so the threshold / argmax paths are actually exercised.
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Tuple

import numpy as np
import torch


def _rng(seed: int, name: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())]))


def _fan_in(shape: Tuple[int, ...]) -> int:
    fan = 1
    for s in shape[1:]:
        fan *= int(s)
    return max(fan, 1)


def synth_tensor(name: str, shape: Tuple[int, ...], seed: int, profile: str = "trained",
                 layer_scale: Tuple[float, float] = (1.0, 2.0)) -> torch.Tensor:
    """One deterministic tensor for parameter/buffer ``name`` of ``shape``."""
    g = _rng(seed, name)
    shape = tuple(int(s) for s in shape)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return torch.zeros(shape, dtype=torch.long)
    if leaf in ("normalization_multiplier", "_multiplier"):
        return torch.full(shape, 2.0)                     # main.py:171
    if leaf == "layer_scale":
        if profile == "init":
            a = np.full(shape, 1e-6)
        else:
            a = g.uniform(layer_scale[0], layer_scale[1], size=shape)
    elif leaf == "running_mean":
        a = 0.1 * g.standard_normal(shape)
    elif leaf == "running_var":
        a = g.uniform(0.5, 1.5, size=shape)
    elif "_classification" in name and leaf == "weight":
        a = g.normal(1.0, 0.1, size=shape)               # main.py:168
    elif "_classification" in name and leaf == "bias":
        a = 0.1 * g.standard_normal(shape)
    elif len(shape) >= 2:
        if profile == "init":
            a = np.clip(g.normal(0.0, 0.02, size=shape), -0.04, 0.04)
        else:
            a = g.standard_normal(shape) / np.sqrt(_fan_in(shape))
    elif leaf == "weight":                               # LayerNorm / BatchNorm affine scale
        a = np.ones(shape) if profile == "init" else 1.0 + 0.1 * g.standard_normal(shape)
    else:                                                # biases
        a = np.zeros(shape) if profile == "init" else 0.05 * g.standard_normal(shape)
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


def synth_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int,
                     profile: str = "trained", **kw) -> Dict[str, torch.Tensor]:
    return {n: synth_tensor(n, s, seed, profile, **kw) for n, s in shapes}


def fill_module_(module: torch.nn.Module, seed: int, profile: str = "trained", prefix: str = "",
                 skip: Tuple[str, ...] = (), **kw) -> torch.nn.Module:
    """Overwrite every parameter/buffer of ``module`` in place with its synthetic value.

    Keys are the module's own ``state_dict`` names (optionally with ``prefix``, e.g.
    ``"module."`` to mimic the DataParallel checkpoints of ``main.py:118``).  Names
    containing any string in ``skip`` keep their constructor values (e.g. the
    BilinearIntermediate embedding pattern of ``count_pipnet_utils.py:356-363``).
    """
    with torch.no_grad():
        for n, t in module.state_dict(keep_vars=True).items():
            if any(s in n for s in skip):
                continue
            v = synth_tensor(prefix + n, tuple(t.shape), seed, profile, **kw)
            t.copy_(v.to(dtype=t.dtype))
    return module


def synth_images(batch: int, size: int, seed: int = 0, channels: int = 3) -> torch.Tensor:
    """``N(0,1)`` float32 NCHW images (ImageNet-normalised range), SURVEY.md section 8d."""
    g = _rng(seed, f"images/{batch}x{channels}x{size}x{size}")
    a = g.standard_normal((batch, channels, size, size), dtype=np.float32)
    return torch.from_numpy(a)


def synth_exponential(shape: Tuple[int, ...], seed: int) -> torch.Tensor:
    """``Exp(1)`` samples -- the noise source of ``F.gumbel_softmax`` (g = -log E)."""
    g = _rng(seed, "exp/" + "x".join(str(int(s)) for s in shape))
    a = g.standard_exponential(size=tuple(shape), dtype=np.float32)
    return torch.from_numpy(np.maximum(a, np.float32(1e-30)))


def synth_bernoulli(shape: Tuple[int, ...], keep: float, seed: int) -> torch.Tensor:
    """{0, 1} float32 samples with P(1) = keep -- recorded stochastic-depth masks."""
    g = _rng(seed, "bern/" + "x".join(str(int(s)) for s in shape))
    return torch.from_numpy((g.random(size=tuple(shape)) < keep).astype(np.float32))
