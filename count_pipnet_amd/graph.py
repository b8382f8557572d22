"""HIP-graph replay of the inference forward (``torch.cuda.CUDAGraph`` is hipGraph on ROCm).

Every HIP kernel of the path is enqueued on torch's current stream with device pointers and
workspaces from torch's caching allocator, so one ``net(xs, inference=True)`` captures into
a single graph: replaying it re-launches the whole forward (≈100 kernels for ConvNeXt-tiny)
with one host call and no per-kernel launch gaps -- what matters for the small, launch-bound
configurations (BASELINE C1: 16 images of 64x64).

Semantics versus the eager forward:
  * the input is copied into the graph's static input buffer; outputs are the graph's static
    output tensors (overwritten by the next replay -- clone them to keep them);
  * weights are read at replay time from the same addresses, so in-place updates of
    parameters (``eval_pipnet``'s classifier sparsification, pipnet/test.py:71-73) are seen;
    repacked copies (depthwise taps, BN-folded ResNet convs, bf16 weights, the folded
    BilinearIntermediate weights W E / V E) are the ones captured -- re-capture after
    ``load_state_dict`` or any weight change other than the classification layer's (and call
    ``invalidate_weight_caches(net)`` first when the change went through ``.data``);
  * the CountPIPNet Gumbel noise is drawn from a device-resident Philox key advanced on the
    stream by every replay (``pipnet_count_gumbel_devseed_f32``): fresh noise per call, as
    the reference draws (count_pipnet_utils.py:36-38);
  * one graph per input shape (batch, size): ``GraphedForward`` keys captures by shape.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch

Tensor = torch.Tensor


class GraphedForward:
    """``g = GraphedForward(net); proto, pooled, out = g(xs)`` == ``net(xs, inference=True)``
    under ``torch.no_grad()`` / eval mode, replayed from a captured HIP graph."""

    def __init__(self, net: torch.nn.Module, inference: bool = True, warmup: int = 2):
        self.net = net
        self.inference = inference
        self.warmup = warmup
        self._graphs: Dict[Tuple, Tuple[torch.cuda.CUDAGraph, Tensor, Tuple[Tensor, ...]]] = {}

    def _capture(self, xs: Tensor):
        if not xs.is_cuda:
            raise RuntimeError("GraphedForward: HIP graphs need a ROCm device tensor (there is no CPU fallback)")
        if self.net.training:
            raise RuntimeError("GraphedForward replays the inference path: call net.eval() first")
        static_x = xs.detach().clone()
        mod = self.net.module if hasattr(self.net, "module") else self.net
        if hasattr(mod, "_graph_seed_state"):     # device Philox key allocated outside the capture
            mod._graph_seed_state(xs.device)
        side = torch.cuda.Stream(device=xs.device)
        side.wait_stream(torch.cuda.current_stream(xs.device))
        with torch.cuda.stream(side), torch.no_grad():
            for _ in range(self.warmup):          # allocator / packed-weight caches settle before capture
                self.net(static_x, inference=self.inference)
        torch.cuda.current_stream(xs.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g):
            outs = self.net(static_x, inference=self.inference)
        return g, static_x, tuple(outs)

    def __call__(self, xs: Tensor):
        key = (tuple(xs.shape), xs.dtype, xs.device)
        if key not in self._graphs:
            self._graphs[key] = self._capture(xs)
        g, static_x, outs = self._graphs[key]
        if xs.data_ptr() != static_x.data_ptr():
            static_x.copy_(xs, non_blocking=True)
        g.replay()
        return outs

    def static_input(self, xs_like: Tensor) -> Tensor:
        """The captured input buffer for this shape (write images here to skip the copy)."""
        key = (tuple(xs_like.shape), xs_like.dtype, xs_like.device)
        if key not in self._graphs:
            self._graphs[key] = self._capture(xs_like)
        return self._graphs[key][1]
