"""The HIP inference path under ShardedInference (count_pipnet_amd.dist), the replacement of
``nn.DataParallel(net, device_ids)`` (/root/reference/main.py:117-118), on the 1-GPU box.

* world 1 over RCCL (``init_process_group("nccl", device_id=cuda:0)``, bench.py's init);
* world 2 and world 3 over gloo with every rank on cuda:0 (RCCL refuses two ranks on one
  device), so the sharding, the uneven shards (5 images -> 3+2 and 2+2+1) and the all-gather
  of proto / pooled / logits run on the HIP kernels' device tensors.

Every rank checks its wrapped outputs against the single-process HIP forward of the full
batch BITWISE: images are independent and the HIP kernels are batch-invariant
(test_gpu_parity.py::test_c2_full_batch_properties), so sharding must not change one bit.

Two tests pin the sharded path against the reference rather than against itself:

* the ``c2_pipnet_convnext26`` golden (recorded from the reference's own PIPNet.forward,
  /root/reference/pipnet/pipnet.py:31-41) through a world-2 gloo run (2 images -> 1 + 1):
  the gathered proto (rank 0) / pooled / logits of both ranks against the recorded values
  at 1e-3 with test_gpu_parity's near-threshold substitution rule, in inference and raw mode;
* BASELINE configs[3]'s per-rank workload (ConvNeXt-tiny-26, K = 196 CARS classes, 64 images
  of 224x224 on one rank) through RCCL, every image against the oracle.
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
        sizes = shard_sizes(batch, world)
        start = sum(sizes[:rank])
        with torch.no_grad():
            r_proto, r_pooled, r_out = net(xs, inference=True)          # single process, full batch
            proto, pooled, out = wrapped(xs, inference=True)            # DataParallel call pattern
            own = xs[start:start + sizes[rank]].contiguous()
            proto2, pooled2, out2 = wrapped(own, inference=True, global_batch=False, sizes=sizes)   # bench.py's
            proto3, _, out3 = wrapped(own, inference=True, global_batch=False)                      # size exchange
        torch.cuda.synchronize()
        res.update(
            # DataParallel call pattern: the proto map is gathered to rank 0 (DataParallel's
            # output device); the other ranks get None (the full-batch map is not theirs)
            proto_full=(proto.shape == r_proto.shape and torch.equal(proto, r_proto)) if rank == 0
            else proto is None,
            proto_strides_nhwc=(proto if rank == 0 else proto2).permute(0, 2, 3, 1).is_contiguous(),
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


def _golden_worker(rank, world, port, backend, case, batch, out_dir, q):
    """Runs the sharded HIP forward on the golden inputs (``batch`` = 0: the recorded batch)
    or on ``batch`` synthetic images; saves the gathered outputs of every rank to out_dir."""
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
        from count_pipnet_amd.dist import ShardedInference
        from count_pipnet_amd.synthetic import synth_images
        from golden_util import golden_inputs, load_golden
        from model_util import build_model
        meta, _ = load_golden(case)
        net = build_model(meta).to(dev)
        xs = golden_inputs(meta) if batch == 0 else synth_images(batch, meta["case"]["size"], seed=43)
        wrapped = ShardedInference(net)
        saved = {}
        with torch.no_grad():
            for inference in (True, False):
                proto, pooled, out = wrapped(xs.to(dev), inference=inference)
                torch.cuda.synchronize()
                tag = "inf" if inference else "raw"
                saved[tag] = (None if proto is None else proto.float().cpu(), pooled.cpu(), out.cpu())
        saved["w"] = net._classification.weight.detach().cpu()
        saved["sd"] = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        torch.save(saved, os.path.join(out_dir, f"rank{rank}.pt"))
        res["backend"] = dist.get_backend()
    except Exception as e:
        res["error"] = repr(e)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    q.put(res)


def _run_golden(world, backend, case, batch, out_dir):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_golden_worker, args=(r, world, port, backend, case, batch, str(out_dir), q))
             for r in range(world)]
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
    assert sorted(res) == list(range(world)), res
    for r in res.values():
        assert "error" not in r and r["backend"] == backend, r
    return [torch.load(os.path.join(out_dir, f"rank{r}.pt"), weights_only=True) for r in range(world)]


def test_sharded_world2_matches_reference_golden(gpu, tmp_path):
    """a18 pinned to the reference: the c2_pipnet_convnext26 golden (2 images, recorded from
    the reference's PIPNet.forward) sharded 1 + 1 over a world-2 gloo group on cuda:0.  Rank
    0 holds the gathered proto map (rank 1 gets None); both ranks hold the gathered pooled / logits; all are
    checked against the recorded values (1e-3, near-threshold substitution, decisive argmax)."""
    from golden_util import load_golden
    from test_gpu_parity import _check_pipnet
    _, rec = load_golden("c2_pipnet_convnext26")
    saved = _run_golden(2, "gloo", "c2_pipnet_convnext26", 0, tmp_path)
    for tag in ("inf", "raw"):
        proto0 = saved[0][tag][0].numpy()
        assert proto0.shape[0] == 2 and saved[1][tag][0] is None      # rank 1: no proto map
        for r in range(2):
            _, pooled, out = saved[r][tag]
            _check_pipnet(proto0, pooled.numpy(), out.numpy(), rec, tag, saved[r]["w"].numpy())


def test_c4_per_rank_shard_vs_oracle(gpu, tmp_path):
    """BASELINE configs[3] per rank: ConvNeXt-tiny-26 PIP-Net with K = 196 classes (CARS) and
    bias (the pipnet_convnext26_bias golden's model), 64 images of 224x224 through
    ShardedInference over RCCL (world 1, bench.py's init), every image against the oracle."""
    import numpy as np
    from golden_util import golden_args, load_golden
    from oracle import ref_cpu
    from test_gpu_parity import _check_pipnet
    meta, _ = load_golden("pipnet_convnext26_bias")
    assert meta["case"]["num_classes"] == 196
    saved = _run_golden(1, "nccl", "pipnet_convnext26_bias", 64, tmp_path)[0]
    sd = saved["sd"]
    from count_pipnet_amd.synthetic import synth_images
    xs = synth_images(64, 224, seed=43)
    with torch.no_grad():
        feats = ref_cpu.backbone(xs, sd, golden_args(meta))
        r_proto = torch.softmax(feats, dim=1)
        r_raw = r_proto.amax(dim=(2, 3))
        r_inf = torch.where(r_raw < 0.1, torch.zeros_like(r_raw), r_raw)
        b = sd.get("_classification.bias")
        r_out_inf = ref_cpu.non_neg_linear(r_inf, sd["_classification.weight"], b)
        r_out_raw = ref_cpu.non_neg_linear(r_raw, sd["_classification.weight"], b)
    common = {"raw_pooled": r_raw.numpy(), "inf_proto_max": r_raw.numpy(), "raw_proto_max": r_raw.numpy(),
              "inf_proto_sum": r_proto.sum(dim=(2, 3)).numpy(), "raw_proto_sum": r_proto.sum(dim=(2, 3)).numpy(),
              "inf_proto_pixmax": r_proto.amax(dim=1).numpy(), "raw_proto_pixmax": r_proto.amax(dim=1).numpy(),
              "inf_proto_slice": r_proto[0, :8].numpy(), "raw_proto_slice": r_proto[0, :8].numpy()}
    rec = dict(common, inf_pooled=r_inf.numpy(), inf_out=r_out_inf.numpy(), raw_out=r_out_raw.numpy())
    w = sd["_classification.weight"].numpy()
    for tag in ("inf", "raw"):
        proto, pooled, out = (t.numpy() for t in saved[tag])
        assert out.shape == (64, 196) and pooled.shape == (64, 768) and proto.shape == (64, 768, 26, 26)
        _check_pipnet(proto, pooled, out, rec, tag, w)
    # the decisive-argmax comparison is not vacuous on this workload
    srt = np.sort(r_out_inf.numpy(), axis=1)
    assert ((srt[:, -1] - srt[:, -2]) > 2e-3 * np.maximum(1, np.abs(srt)).max(axis=1)).sum() >= 32


def _count_worker(rank, world, port, batch, q):
    """BASELINE configs[4]'s layout: the C5 CountPIPNet (bilinear, hard Gumbel head, 2048
    prototypes) with each rank passing its own shard (bench.py's call pattern) and the Exp(1)
    draw of its images injected; the gathered counts / logits and the rank's proto shard vs
    the single-process forward of the whole batch with the whole draw (bitwise)."""
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
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from count_pipnet_amd.dist import ShardedInference, shard_sizes
        from count_pipnet_amd.synthetic import synth_exponential, synth_images
        from golden_util import load_golden
        from model_util import build_model
        meta, _ = load_golden("c5_count_bilinear_2048")
        net = build_model(meta).to(dev)
        size = meta["case"]["size"]
        xs = synth_images(batch, size, seed=55).to(dev)
        p, h, w = 2048, size // 8, size // 8                  # prototypes, proto grid (16 x 16 at 128^2)
        noise = synth_exponential((batch, p, h, w), seed=56).to(dev)
        sizes = shard_sizes(batch, world)
        start = sum(sizes[:rank])
        wrapped = ShardedInference(net)
        with torch.no_grad():
            net._add_on[-1].exp_noise = noise
            r_proto, r_counts, r_out = net(xs, inference=True)
            net._add_on[-1].exp_noise = noise[start:start + sizes[rank]]
            proto, counts, out = wrapped(xs[start:start + sizes[rank]].contiguous(), inference=True,
                                         global_batch=False, sizes=sizes)
        torch.cuda.synchronize()
        res.update(grid=tuple(r_proto.shape) == (batch, p, h, w),
                   proto=torch.equal(proto, r_proto[start:start + sizes[rank]]),
                   counts=torch.equal(counts, r_counts), out=torch.equal(out, r_out),
                   shapes=tuple(counts.shape) == (batch, p) and tuple(out.shape) == (batch, r_out.shape[1]),
                   backend=dist.get_backend(), module=wrapped.module is net, device=str(out.device))
    except Exception as e:
        res["error"] = repr(e)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    q.put(res)


def test_c5_count_sharded_gloo_world4(gpu):
    """BASELINE configs[4] shards its batch over 4 GPUs: the C5 CountPIPNet through a world-4
    gloo group on cuda:0 (8 images -> 2 per rank), gathered counts / logits bitwise equal to
    the single-process forward on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world, batch = 4, 8
    procs = [ctx.Process(target=_count_worker, args=(r, world, port, batch, q)) for r in range(world)]
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
    _assert_all(res, world, "gloo")
