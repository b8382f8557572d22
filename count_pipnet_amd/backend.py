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


_CROSS = threading.local()


@contextlib.contextmanager
def cross_stream_forward():
    """Marks a forward whose sub-batches run on several HIP streams (the split forwards of
    pipnet.py / count_pipnet.py): a weight cache rebuilt inside it is read by the other streams."""
    _CROSS.depth = getattr(_CROSS, "depth", 0) + 1
    try:
        yield
    finally:
        _CROSS.depth -= 1


def packed_ready() -> None:
    """Call right after a weight cache was (re)built.  Inside ``cross_stream_forward`` the
    repacking kernels ran on one sub-batch stream and the other streams would read the new
    buffers without waiting for them, so the current stream is host-synchronised there -- on a
    cache miss only (first forward, or after a weight change), never during graph capture
    (captures replay warm caches).  Everywhere else (one-stream forwards, the training steps,
    whose trainable weights change every step) the rebuilt buffer is stream-ordered before its
    readers already and nothing waits."""
    if getattr(_CROSS, "depth", 0) and torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
        torch.cuda.current_stream().synchronize()
