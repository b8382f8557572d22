"""HIP executor for the ResNet feature backbones (resnet_features.py)."""
from __future__ import annotations

from typing import Dict

import torch


def resnet_features_hip(model, x: torch.Tensor, cache: Dict) -> torch.Tensor:
    raise NotImplementedError(
        "count_pipnet_amd: the ResNet HIP path is not built yet; run ResNet backbones on the "
        "torch path explicitly with `with count_pipnet_amd.backend.torch_backend(): ...`")
