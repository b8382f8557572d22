"""Multi-GPU inference: one process per GPU, batch sharded, RCCL all-gather of the results.

Replaces the reference's single-process ``nn.DataParallel(net)`` (``main.py:117-118``,
``util/interpret_idg.py:175``), which on *every* forward broadcasts all parameters from
GPU 0 (112 MB for ConvNeXt-tiny-26), scatters the batch, runs one Python thread per GPU and
gathers all three outputs back to GPU 0.  Here:

  * weights are loaded once per device (each rank owns a resident replica);
  * the global batch is split exactly like ``DataParallel.scatter`` (``torch.chunk`` along
    dim 0, so shard sizes and order match), or each rank passes its own shard;
  * the only exchange is one all-gather of ``pooled`` [B/N, P] and ``out`` [B/N, K]
    over RCCL/xGMI -- no reduction is needed because images are independent;
  * ``proto_features`` is gathered too when the caller uses DataParallel's call pattern
    (the full batch on every rank), because DataParallel gathers all three outputs and
    callers index ``proto_features[i]`` across the batch (util/vis_pipnet.py:25).  Callers
    that pass their own shard (``global_batch=False``, e.g. bench.py) get their shard's map
    unless they ask for the gather.

``ShardedInference`` keeps DataParallel's ``.module`` attribute, so callers written for
the reference (``net.module._classification``, ``net.module._num_classes`` in
``pipnet/test.py``) work unchanged.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

Tensor = torch.Tensor


def shard_sizes(batch: int, world: int) -> List[int]:
    """Per-rank shard sizes of torch.chunk(batch, world) (DataParallel's scatter)."""
    if batch == 0:
        return [0] * world
    step = -(-batch // world)
    sizes = []
    left = batch
    for _ in range(world):
        s = min(step, left)
        sizes.append(s)
        left -= s
    return sizes


def all_gather_rows(x: Tensor, sizes: List[int], group=None) -> Tensor:
    """Concatenate every rank's ``x`` (rank r holds ``sizes[r]`` rows) on every rank.
    Uneven shards are padded to the largest one for the collective and trimmed after."""
    world = len(sizes)
    if world == 1:
        return x
    mx = max(sizes)
    if x.shape[0] < mx:
        pad = torch.zeros((mx - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        x = torch.cat([x, pad], dim=0)
    bufs = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(bufs, x.contiguous(), group=group)
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0)


class ShardedInference(nn.Module):
    """Data-parallel inference wrapper (DataParallel semantics, one process per GPU)."""

    def __init__(self, module: nn.Module, process_group=None, gather_proto: Optional[bool] = None):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.gather_proto = gather_proto

    @property
    def world(self) -> int:
        return dist.get_world_size(self.process_group) if dist.is_available() and dist.is_initialized() else 1

    @property
    def rank(self) -> int:
        return dist.get_rank(self.process_group) if dist.is_available() and dist.is_initialized() else 0

    def forward(self, xs: Tensor, inference: bool = False, global_batch: bool = True,
                sizes: Optional[List[int]] = None) -> Tuple[Tensor, Tensor, Tensor]:
        """``global_batch=True``: ``xs`` is the full batch on every rank (DataParallel call
        pattern) and this rank takes its ``torch.chunk`` shard.  ``False``: ``xs`` is this
        rank's own shard (pass ``sizes`` -- every rank's shard size -- to skip the size
        exchange and its host sync).  Returns (proto_features, pooled [B, P], out [B, K]) in global
        batch order; proto_features covers the whole batch when ``gather_proto`` is True, or
        when it is None (the default) and ``global_batch`` is True -- DataParallel's outputs --,
        and this rank's shard otherwise."""
        world, rank = self.world, self.rank
        if global_batch:
            sizes = shard_sizes(xs.shape[0], world)
            start = sum(sizes[:rank])
            local = xs[start:start + sizes[rank]]
        elif sizes is not None:
            local = xs
            if len(sizes) != world or sizes[rank] != xs.shape[0]:
                raise ValueError(f"sizes {sizes} inconsistent with world {world} / local batch {xs.shape[0]}")
        else:
            local = xs
            n = torch.tensor([local.shape[0]], device=local.device, dtype=torch.int64)
            if world > 1:
                ns = [torch.empty_like(n) for _ in range(world)]
                dist.all_gather(ns, n, group=self.process_group)
                sizes = [int(v.item()) for v in ns]
            else:
                sizes = [local.shape[0]]
        proto, pooled, out = self.module(local, inference=inference)
        pooled = all_gather_rows(pooled, sizes, self.process_group)
        out = all_gather_rows(out, sizes, self.process_group)
        gather_proto = global_batch if self.gather_proto is None else self.gather_proto
        if gather_proto and world > 1:
            proto = gather_proto_features(proto, sizes, self.process_group)
        return proto, pooled, out


def gather_proto_features(proto: Tensor, sizes: List[int], group=None) -> Tensor:
    """All-gather a [b, P, h, w] prototype map.  The HIP path returns it as a view of NHWC
    storage (channels_last strides); it is exchanged in that storage order (no transpose
    on either side) and handed back with the same strides."""
    if proto.dim() == 4 and proto.permute(0, 2, 3, 1).is_contiguous():
        g = all_gather_rows(proto.permute(0, 2, 3, 1), sizes, group)
        return g.permute(0, 3, 1, 2)
    return all_gather_rows(proto.contiguous(), sizes, group)


def init_from_env(backend: Optional[str] = None, device_index: Optional[int] = None) -> Tuple[int, int, torch.device]:
    """Initialise torch.distributed from torchrun's env (RANK / WORLD_SIZE / LOCAL_RANK /
    MASTER_*); backend "nccl" (= RCCL on ROCm) on GPUs, "gloo" on CPU.  ``device_index``
    puts every rank on one GPU (a multi-rank rehearsal on a 1-GPU box, with backend
    "gloo": RCCL refuses two ranks on one device).  Returns (rank, world, device)."""
    import os
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if device_index is None else device_index
    use_gpu = torch.cuda.is_available()
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if use_gpu:
            torch.cuda.set_device(local)
            if (backend or "nccl") == "nccl":
                dist.init_process_group("nccl", device_id=dev)
            else:
                dist.init_process_group(backend)
        else:
            dist.init_process_group(backend or "gloo")
    rank = dist.get_rank() if dist.is_initialized() else 0
    return rank, world, dev
