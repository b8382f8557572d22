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


# Attributes under which modules keep device-layout copies of their parameters (depthwise taps,
# BN-folded convs, bf16 / split-plane weights, the folded bilinear intermediate).
_CACHE_ATTRS = ("_hip_pack", "_hip_fold_cache")


def invalidate_weight_caches(net: torch.nn.Module) -> int:
    """Drop every repacked / folded weight copy under ``net``; the next HIP forward rebuilds them.

    The caches are keyed on each parameter's storage pointer and in-place version counter, which
    every torch in-place op (``optimizer.step()``, ``load_state_dict``, ``param.copy_``) bumps.
    A write through ``param.data`` (``p.data.copy_(...)``, ``p.data[...] = ...``) goes through a
    tensor with its OWN version counter, so it is invisible to that stamp: call this after such a
    write (or write through ``torch.no_grad()`` + ``param.copy_`` instead).  Returns the number
    of cache dicts cleared.  Captured graphs (``graph.GraphedForward``) must be re-captured."""
    n = 0
    for mod in net.modules():
        for attr in _CACHE_ATTRS:
            c = mod.__dict__.get(attr)
            if isinstance(c, dict):
                c.clear()
                n += 1
    return n


def packed_ready() -> None:
    """Call right after a weight cache was (re)built: the repacking kernels ran on the current
    stream, and a concurrent sub-batch forward on another HIP stream (pipnet.set_stream_split)
    would read the new buffers without waiting for them.  Host-synchronises the current stream
    on a cache miss only (first forward, or after a weight change), never during graph capture
    (captures replay warm caches)."""
    if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        torch.cuda.current_stream().synchronize()

