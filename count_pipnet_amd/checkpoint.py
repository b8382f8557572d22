"""Checkpoint -> packed device weights.

The reference saves ``{'model_state_dict': net.state_dict(), 'optimizer_net_state_dict': ...}``
with ``net`` wrapped in ``nn.DataParallel`` (``util/checkpoint_manager.py:118-125``, keys
``module.``-prefixed) and loads them with ``torch.load`` + ``load_state_dict(strict=True)``
(``:64-67, :85-88``).  ``load_checkpoint`` reads the same files into this package's modules
-- with the safe loader (``weights_only=True``: tensors and plain containers only) -- moves
the model to the device and builds every device-layout copy the HIP path needs
(BatchNorm-folded ResNet convs, depthwise / downsample repacks, bf16 casts) by one
single-image warm-up forward, so the first real batch pays no packing cost.
"""
from __future__ import annotations

from typing import Mapping, Optional, Union

import torch
import torch.nn as nn

Tensor = torch.Tensor


def model_state_dict(obj) -> Mapping[str, Tensor]:
    """The model weights inside a reference checkpoint object (or a bare state_dict)."""
    if isinstance(obj, Mapping) and "model_state_dict" in obj:
        obj = obj["model_state_dict"]
    if not isinstance(obj, Mapping):
        raise ValueError(f"not a checkpoint / state_dict: {type(obj).__name__}")
    return obj


def adapt_keys(sd: Mapping[str, Tensor], target: nn.Module) -> Mapping[str, Tensor]:
    """Add or strip the DataParallel ``module.`` prefix so ``sd`` matches ``target``."""
    want_prefix = next(iter(target.state_dict().keys()), "").startswith("module.")
    have_prefix = next(iter(sd.keys()), "").startswith("module.")
    if have_prefix and not want_prefix:
        return {k[len("module."):]: v for k, v in sd.items()}
    if want_prefix and not have_prefix:
        return {"module." + k: v for k, v in sd.items()}
    return sd


def load_checkpoint(net: nn.Module, source: Union[str, Mapping], device: Optional[torch.device] = None,
                    strict: bool = True, warmup_image_size: Optional[int] = 224) -> nn.Module:
    """Load a reference checkpoint (path or loaded object) into ``net`` for HIP inference.

    ``net`` may be the bare model or a DataParallel / ShardedInference wrapper.  Returns the
    model in eval mode on ``device`` with its packed weights built (a 1-image forward at
    ``warmup_image_size``; None skips it)."""
    obj = torch.load(source, map_location="cpu", weights_only=True) if isinstance(source, str) else source
    sd = adapt_keys(model_state_dict(obj), net)
    missing, unexpected = net.load_state_dict(sd, strict=strict)
    if device is not None:
        net = net.to(device)
    net.eval()
    if warmup_image_size and device is not None and torch.device(device).type == "cuda":
        prepack(net, warmup_image_size, device)
    return net


@torch.no_grad()
def prepack(net: nn.Module, image_size: int, device) -> None:
    """Build every cached device-layout weight by one single-image inference forward."""
    mod = net.module if hasattr(net, "module") else net
    xs = torch.zeros(1, 3, image_size, image_size, device=device)
    mod.eval()
    mod(xs, inference=True)
    torch.cuda.synchronize(device)
