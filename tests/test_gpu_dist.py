"""The HIP inference path under ShardedInference (count_pipnet_amd.dist), the replacement of
``nn.DataParallel(net, device_ids)`` (/root/reference/main.py:117-118), on the 1-GPU box.

* world 1 over RCCL (``init_process_group("nccl", device_id=cuda:0)``, bench.py's init);
* world 2 and world 3 over gloo with every rank on cuda:0 (RCCL refuses two ranks on one
  device), so the sharding, the uneven shards (5 images -> 3+2 and 2+2+1) and the all-gather
  of proto / pooled / logits run on the HIP kernels' device tensors.

Every rank checks its wrapped outputs against the single-process HIP forward of the full
batch BITWISE: images are independent and the HIP kernels are batch-invariant
(test_gpu_parity.py::test_c2_full_batch_properties), so sharding must not change one bit.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

TESTS = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, backend, case, batch, q):
    import sys
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    sys.path.insert(0, TESTS)
    sys.path.insert(0, os.path.dirname(TESTS))
    import torch.distributed as dist
    res = {"rank": rank}
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from count_pipnet_amd.dist import ShardedInference, shard_sizes
        from golden_util import golden_inputs, load_golden
        from model_util import build_model
        from count_pipnet_amd.synthetic import synth_images
        meta, _ = load_golden(case)
        net = build_model(meta).to(dev)
        size = meta["case"]["size"]
        xs = synth_images(batch, size, seed=41).to(dev)
        wrapped = ShardedInference(net)
        with torch.no_grad():
            r_proto, r_pooled, r_out = net(xs, inference=True)          # single process, full batch
            proto, pooled, out = wrapped(xs, inference=True)            # DataParallel call pattern
            sizes = shard_sizes(batch, world)
            start = sum(sizes[:rank])
            own = xs[start:start + sizes[rank]].contiguous()
            proto2, pooled2, out2 = wrapped(own, inference=True, global_batch=False, sizes=sizes)   # bench.py's
            proto3, _, out3 = wrapped(own, inference=True, global_batch=False)                      # size exchange
        torch.cuda.synchronize()
        res.update(
            proto_full=proto.shape == r_proto.shape and torch.equal(proto, r_proto),
            proto_strides_nhwc=proto.permute(0, 2, 3, 1).is_contiguous(),
            pooled=torch.equal(pooled, r_pooled), out=torch.equal(out, r_out),
            shard_pooled=torch.equal(pooled2, r_pooled), shard_out=torch.equal(out2, r_out),
            shard_proto=torch.equal(proto2, r_proto[start:start + sizes[rank]]),
            exch_out=torch.equal(out3, r_out), exch_proto=proto3.shape[0] == sizes[rank],
            backend=dist.get_backend(), module=wrapped.module is net, device=str(out.device))
    except Exception as e:       # reported to the parent, which fails the test with it
        res["error"] = repr(e)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    q.put(res)


def _run(world, backend, case, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, case, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r = q.get(timeout=300)
            res[r["rank"]] = r
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return res


def _assert_all(res, world, backend):
    assert sorted(res) == list(range(world)), res
    for r in res.values():
        assert "error" not in r, r
        assert r["backend"] == backend and r["module"] and r["device"] == "cuda:0", r
        bad = [k for k, v in r.items() if isinstance(v, bool) and not v]
        assert not bad, (r["rank"], bad)


def test_sharded_hip_rccl_world1(gpu):
    """bench.py's process-group init (RCCL with device_id) around the HIP forward."""
    _assert_all(_run(1, "nccl", "c2_pipnet_convnext26", 3), 1, "nccl")


@pytest.mark.parametrize("world,case,batch", [(2, "c2_pipnet_convnext26", 5), (3, "pipnet_mid_addon", 5),
                                              (2, "pipnet_mid_addon", 4)])
def test_sharded_hip_gloo_shared_gpu(gpu, world, case, batch):
    """Uneven shards (5 -> 3+2, 2+2+1) and the all-gather of all three outputs on device tensors."""
    _assert_all(_run(world, "gloo", case, batch), world, "gloo")
