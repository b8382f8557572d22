"""Dispatch rule between the HIP inference path and the autograd (training) path.

Reference semantics: the same ``forward(xs, inference)`` serves training
(``pipnet/train.py:84``, grads + custom STE backward) and evaluation (``pipnet/test.py:75``
under ``@torch.no_grad``, ``net.eval()``).  The MI355X path is inference-only, so

  * eval mode AND grad disabled  ->  HIP kernels (input must be a ROCm float32 tensor;
                                     anything else raises -- there is no CPU fallback);
  * train mode OR grad enabled   ->  the torch autograd path (training is out of scope
                                     for the kernels and keeps the reference's gradients).

``torch_backend()`` lets a caller explicitly ask for the torch path in eval mode (e.g. to
evaluate on a host without a GPU); it is never taken implicitly.
"""
from __future__ import annotations

import contextlib
import threading

import torch

_state = threading.local()


def _forced_torch() -> bool:
    return getattr(_state, "force_torch", False)


@contextlib.contextmanager
def torch_backend():
    """Explicitly run modules on their plain-torch path inside this context."""
    prev = _forced_torch()
    _state.force_torch = True
    try:
        yield
    finally:
        _state.force_torch = prev


def use_hip(module: torch.nn.Module) -> bool:
    return (not module.training) and (not torch.is_grad_enabled()) and (not _forced_torch())
