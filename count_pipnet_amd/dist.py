"""Multi-GPU inference: one process per GPU, batch sharded, RCCL all-gather of the results.

Replaces the reference's single-process ``nn.DataParallel(net)`` (``main.py:117-118``,
``util/interpret_idg.py:175``), which on *every* forward broadcasts all parameters from
GPU 0 (112 MB for ConvNeXt-tiny-26), scatters the batch, runs one Python thread per GPU and
gathers all three outputs back to GPU 0.  Here:

  * weights are loaded once per device (each rank owns a resident replica);
  * the global batch is split exactly like ``DataParallel.scatter`` (``torch.chunk`` along
    dim 0, so shard sizes and order match), or each rank passes its own shard;
  * the only exchange is ONE all-gather of ``pooled`` [B/N, P] and ``out`` [B/N, K] packed side
    by side into one [B/N, P + K] buffer over RCCL/xGMI (the exchange is latency-bound, tens of us
    per collective, so one collective instead of two halves it) -- no reduction is needed because
    images are independent;
  * ``proto_features`` is gathered to rank 0 when the caller uses DataParallel's call
    pattern (the full batch on every rank): DataParallel gathers all three outputs to
    ``device_ids[0]`` and callers index ``proto_features[i]`` across the batch
    (util/vis_pipnet.py:25).  The other ranks get ``None`` for it -- the full-batch map is not
    on their device, and handing them their own shard beside full-batch pooled / logits would
    make ``proto_features[i]`` silently pick the wrong image -- so the map (133 MB per 64
    ConvNeXt images) crosses xGMI once per shard, not once per rank pair.
    ``gather_proto=True`` all-gathers it to every rank, ``False`` never gathers (each rank keeps
    its shard's map); callers that pass their own shard (``global_batch=False``, e.g.
    bench.py) get their shard's map unless they ask.

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


def _pad_rows(x: Tensor, rows: int) -> Tensor:
    if x.shape[0] < rows:
        pad = torch.zeros((rows - x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        x = torch.cat([x, pad], dim=0)
    return x.contiguous()


def gather_rows_to_root(x: Tensor, sizes: List[int], group=None, root: int = 0) -> Tensor:
    """Rank ``root`` receives every rank's rows concatenated in rank order; the other ranks
    get their own ``x`` back (DataParallel's gather places the outputs on one device)."""
    world = len(sizes)
    if world == 1:
        return x
    xp = _pad_rows(x, max(sizes))
    me = dist.get_rank(group)
    bufs = [torch.empty_like(xp) for _ in range(world)] if me == root else None
    dist.gather(xp, gather_list=bufs, dst=dist.get_global_rank(group, root) if group is not None else root,
                group=group)
    if me != root:
        return x
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)], dim=0)


def all_gather_rows(x: Tensor, sizes: List[int], group=None) -> Tensor:
    """Concatenate every rank's ``x`` (rank r holds ``sizes[r]`` rows) on every rank: ONE
    ``all_gather_into_tensor`` straight into the [world * max(sizes), ...] output (no per-rank
    buffers, no concatenation).  Even shards (the bench and DataParallel's usual case) return
    that output as is; an uneven shard is padded for the collective and the padding rows are
    dropped by one compaction copy."""
    world = len(sizes)
    if world == 1:
        return x
    mx = max(sizes)
    x = _pad_rows(x, mx)
    out = torch.empty((world * mx,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=group)
    if all(s == mx for s in sizes):
        return out
    return torch.cat([out[r * mx:r * mx + s] for r, s in enumerate(sizes)], dim=0)


class ShardedInference(nn.Module):
    """Data-parallel inference wrapper (DataParallel semantics, one process per GPU)."""

    def __init__(self, module: nn.Module, process_group=None, gather_proto: Optional[bool] = None):
        super().__init__()
        self.module = module
        self.process_group = process_group
        self.gather_proto = gather_proto
        # bench.py: when a list, every forward appends the (start, end) HIP events bracketing its
        # pooled + logits exchange on the current stream (the collective's cost per step)
        self.exchange_events: Optional[list] = None

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
        batch order.  proto_features covers the whole batch on every rank when ``gather_proto``
        is True; when it is None (the default) and ``global_batch`` is True -- DataParallel's
        output placement -- it covers the whole batch on rank 0 and is ``None`` on every other
        rank; otherwise it is this rank's shard."""
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
        pooled, out = exchange_outputs(pooled, out, sizes, self.process_group, self.exchange_events)
        if world > 1:
            if self.gather_proto is None and global_batch:
                proto = gather_proto_features(proto, sizes, self.process_group, to_root=True)
                if rank != 0:
                    proto = None          # not this rank's to index (see the module docstring)
            elif self.gather_proto:
                proto = gather_proto_features(proto, sizes, self.process_group)
        return proto, pooled, out


def exchange_outputs(pooled: Tensor, out: Tensor, sizes: List[int], group=None,
                     events: Optional[list] = None) -> Tuple[Tensor, Tensor]:
    """All-gather this rank's ``pooled`` [b, P] and ``out`` [b, K] rows in ONE collective: both
    are written side by side into a [b, P + K] buffer (same dtype), gathered with one
    ``all_gather_into_tensor`` and split back into contiguous [B, P] / [B, K] tensors in global
    batch order.  ``events``: a list that receives the (start, end) events of the exchange."""
    if len(sizes) == 1:
        return pooled, out
    if pooled.dtype != out.dtype:
        raise RuntimeError(f"exchange_outputs: pooled {pooled.dtype} and logits {out.dtype} differ")
    e0 = e1 = None
    if events is not None and pooled.is_cuda:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
    p = pooled.shape[1]
    both = torch.cat([pooled, out], dim=1)
    g = all_gather_rows(both, sizes, group)
    pooled_g, out_g = g[:, :p].contiguous(), g[:, p:].contiguous()
    if e1 is not None:
        e1.record()
        events.append((e0, e1))
    return pooled_g, out_g


def gather_proto_features(proto: Tensor, sizes: List[int], group=None, to_root: bool = False) -> Tensor:
    """Gather a [b, P, h, w] prototype map to every rank (or to rank 0 with ``to_root``).  The
    HIP path returns it as a view of NHWC storage (channels_last strides); it is exchanged in
    that storage order (no transpose on either side) and handed back with the same strides."""
    gather = gather_rows_to_root if to_root else all_gather_rows
    if proto.dim() == 4 and proto.permute(0, 2, 3, 1).is_contiguous():
        g = gather(proto.permute(0, 2, 3, 1), sizes, group)
        return g.permute(0, 3, 1, 2)
    return gather(proto.contiguous(), sizes, group)


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
