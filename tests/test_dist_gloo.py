"""Multi-process data-parallel inference (count_pipnet_amd.dist) on CPU with gloo,
world_size 2: DataParallel-style sharding (torch.chunk order, uneven shards) and the
all-gather of proto / pooled / logits reproduce the single-process full-batch forward.
The HIP path under the same wrapper is tests/test_gpu_dist.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from count_pipnet_amd.dist import ShardedInference, shard_sizes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
        from count_pipnet_amd.backend import torch_backend
        from golden_util import golden_inputs, load_golden
        from model_util import build_model
        meta, _ = load_golden("pipnet_mid_addon")
        net = build_model(meta)
        xs = torch.cat([golden_inputs(meta)] * 2)[:batch]
        wrapped = ShardedInference(net)
        with torch.no_grad(), torch_backend():
            proto, pooled, out = wrapped(xs, inference=True)
            r_proto, r_pooled, r_out = net(xs, inference=True)
            start = sum(shard_sizes(batch, world)[:rank])
            own = shard_sizes(batch, world)[rank]
            # per-rank shard path: each rank passes only its own rows
            proto2, pooled2, out2 = wrapped(xs[start:start + own], inference=True, global_batch=False)
            # bench.py's call: own shard + every rank's size (no size exchange)
            _, pooled3, out3 = wrapped(xs[start:start + own], inference=True, global_batch=False,
                                       sizes=shard_sizes(batch, world))
            # gather_proto=True: the whole map on every rank
            proto4, _, _ = ShardedInference(net, gather_proto=True)(xs, inference=True)
            proto5, _, _ = ShardedInference(net, gather_proto=False)(xs, inference=True)
            try:
                wrapped(xs[start:start + own], inference=True, global_batch=False, sizes=[own + 1] * world)
                bad_sizes_rejected = False
            except ValueError:
                bad_sizes_rejected = True
        ok = (torch.allclose(pooled, r_pooled, atol=1e-6) and torch.allclose(out, r_out, rtol=1e-5, atol=1e-5)
              and torch.equal(pooled, pooled2) and torch.equal(out, out2) and proto2.shape[0] == own
              # DataParallel call pattern: pooled / logits cover the whole batch everywhere, the
              # proto map is gathered to rank 0 (DataParallel's output device); the other ranks
              # get None, so proto[i] over the batch cannot silently pick a wrong image there
              and ((proto.shape == r_proto.shape and torch.allclose(proto, r_proto, atol=1e-6)) if rank == 0
                   else proto is None)
              # gather_proto=False keeps each rank's own shard
              and torch.allclose(proto5, r_proto[start:start + own], atol=1e-6)
              and proto4.shape == r_proto.shape and torch.allclose(proto4, r_proto, atol=1e-6)
              and torch.equal(pooled, pooled3) and torch.equal(out, out3) and bad_sizes_rejected
              and wrapped.module is net)
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch", [4, 5])
def test_sharded_inference_gloo_world2(batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}


def test_shard_sizes_match_torch_chunk():
    for b in range(0, 20):
        for w in (1, 2, 3, 4, 8):
            ref = [c.shape[0] for c in torch.arange(b).chunk(w)] if b else []
            ref += [0] * (w - len(ref))
            assert shard_sizes(b, w) == ref, (b, w)


def _group_worker(rank, world, port, q):
    """bench.py's C5 layout at N = 8: two independent 4-rank groups (dist.new_group), every rank
    passing its own shard; each group's gathered outputs equal its own 4-shard batch."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
        from count_pipnet_amd.backend import torch_backend
        from golden_util import golden_inputs, load_golden
        from model_util import build_model
        meta, _ = load_golden("pipnet_mid_addon")
        net = build_model(meta)
        base = golden_inputs(meta)
        groups = [dist.new_group(list(range(g0, g0 + 4))) for g0 in range(0, world, 4)]
        g = rank // 4
        # group g's batch: 4 shards of 1 image, image i of group g = base[(g + i) % len(base)] * (1 + g)
        imgs = torch.stack([base[(g + i) % base.shape[0]] * (1 + 0.1 * g) for i in range(4)])
        wrapped = ShardedInference(net, process_group=groups[g])
        with torch.no_grad(), torch_backend():
            _, pooled, out = wrapped(imgs[rank % 4:rank % 4 + 1], inference=True, global_batch=False,
                                     sizes=[1] * 4)
            _, r_pooled, r_out = net(imgs, inference=True)
        ok = (pooled.shape[0] == 4 and torch.allclose(pooled, r_pooled, atol=1e-6)
              and torch.allclose(out, r_out, rtol=1e-5, atol=1e-5) and wrapped.world == 4 and wrapped.rank == rank % 4)
        q.put((rank, bool(ok)))
        dist.barrier()          # rank 0 hosts the store: no rank leaves while another group still uses it
    finally:
        dist.destroy_process_group()


def test_sharded_inference_two_groups_world8():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    res = dict(q.get(timeout=5) for _ in range(8))
    assert res == {r: True for r in range(8)}


def _one_collective_worker(rank, world, port, q):
    """One forward of the per-rank shard call (bench.py's) issues exactly ONE collective -- the
    packed [b, P + K] all-gather of pooled and logits -- and its outputs equal the single-process
    full-batch forward (pooled / logits split back out of the packed rows, contiguous)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
        from count_pipnet_amd.backend import torch_backend
        from golden_util import golden_inputs, load_golden
        from model_util import build_model
        meta, _ = load_golden("pipnet_mid_addon")
        net = build_model(meta)
        xs = torch.cat([golden_inputs(meta)] * 2)[:4]
        sizes = shard_sizes(4, world)
        start = sum(sizes[:rank])
        calls = []
        names = ("all_gather_into_tensor", "all_gather", "gather", "all_reduce", "broadcast", "reduce_scatter",
                 "all_to_all", "all_to_all_single")
        orig = {n: getattr(dist, n) for n in names}

        def counted(n):
            def f(*a, **k):
                calls.append(n)
                return orig[n](*a, **k)
            return f
        wrapped = ShardedInference(net, gather_proto=False)
        with torch.no_grad(), torch_backend():
            _, r_pooled, r_out = net(xs, inference=True)
            for n in names:
                setattr(dist, n, counted(n))
            try:
                _, pooled, out = wrapped(xs[start:start + sizes[rank]], inference=True, global_batch=False,
                                         sizes=sizes)
            finally:
                for n in names:
                    setattr(dist, n, orig[n])
        ok = (calls == ["all_gather_into_tensor"] and pooled.is_contiguous() and out.is_contiguous()
              and torch.allclose(pooled, r_pooled, atol=1e-6) and torch.allclose(out, r_out, rtol=1e-5, atol=1e-5))
        q.put((rank, bool(ok), calls))
    finally:
        dist.destroy_process_group()


def test_one_collective_per_forward_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_one_collective_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = {r: (ok, calls) for r, ok, calls in (q.get(timeout=5) for _ in range(2))}
    assert all(ok for ok, _ in res.values()), res
