"""Throughput of the MI355X PIP-Net inference path (BASELINE.json metric).

A "step" = one ``PIPNet.forward(xs, inference=True)`` of ConvNeXt-tiny-26 over one batch of
64 synthetic 224x224 images per GPU (fp32), inputs resident in HBM, plus -- for N > 1 -- the
RCCL all-gather of logits and pooled presence over xGMI that replaces nn.DataParallel's
gather (main.py:118).  Weak scaling: 64 images per GPU.  200 classes (CUB-200, BASELINE
configs[1]) except at N = 8, where the workload is configs[3] (CARS: 196 classes, 512 images
over 8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--no-extra]

With ``--gpus N > 1`` and no torchrun environment, bench.py launches its own N ranks (a
``torch.distributed.run`` child, started before anything touches the GPU) and exits with
its status; under torchrun, ``WORLD_SIZE`` must equal N.

The same run also times the other GPU configs of BASELINE.json (``extra``), each with its own
dominant-kernel roofline; ``value`` / ``config`` stay C2.  C3 (PIP-Net ResNet-50, 128 images
of 224x224, bf16) is a 1-GPU config: at N > 1 every rank runs its own configs[2] batch.  C5
(CountPIPNet bilinear, 2048 prototypes, 128x128) is configs[4] = 256 images over 4 GPUs: at
N = 4k it runs as k independent 4-rank groups of exactly that layout, below 4 GPUs as N
64-image shards of it.  Each ``extra.*.workload`` states which (``extra_layout``).

Prints one JSON line on rank 0 (fields described in DESIGN.md section "Measurement").
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec fwd, CUB-200 224×224 bs=64 ConvNeXt-tiny, 1/2/4/8 MI355X"
PEAK_F32_TFLOPS = 157.3          # MI355X_MICROARCH.md: FP32 matrix (= vector) peak, spec
PEAK_HBM_GBS = 8000.0
PEAK_BF16_TFLOPS = 2500.0        # MI355X_MICROARCH.md: BF16 dense matrix peak
GFLOP_C2 = 40.094159616          # oracle.ref_cpu.gflop_per_image(convnext_tiny_26, 224)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--classes", type=int, default=None,
                    help="classifier width (default: 196 = CARS at N = 8, BASELINE configs[3]; else 200 = CUB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the C3 / C5 timings")
    ap.add_argument("--precision", choices=["fp32", "bf16x3"], default="fp32",
                    help="fp32: exact fp32 MFMA GEMMs; bf16x3: split-bf16 GEMMs (fp32 in/out, ~1e-5 per product)")
    ap.add_argument("--alt-precision", choices=["none", "fp32", "bf16x3"], default="bf16x3",
                    help="also time this precision on the same network (reported under alt_precision)")
    ap.add_argument("--stream-split", type=int, default=None,
                    help="override the models' default stream split for the throughput pass, C3 / C5 included "
                         "(profiling runs use 1 so every launch of a kernel is a full-batch launch, as in the "
                         "roofline pass)")
    ap.add_argument("--dist-backend", default=None,
                    help="rehearsal only: torch.distributed backend (default nccl = RCCL on GPUs)")
    ap.add_argument("--device-index", type=int, default=None,
                    help="rehearsal only: put every rank on this GPU (multi-rank runs on a 1-GPU box)")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks_if_needed(a) -> None:
    """``--gpus N`` is authoritative.  Under torchrun (WORLD_SIZE set) it must match the world
    size; without it and N > 1, start N ranks as a ``torch.distributed.run`` child process
    (one process per GPU, RCCL over xGMI) and exit with its status.  Nothing here touches the
    GPU, so the parent never holds a HIP context while its ranks run."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={ws} (torchrun's world size); "
                             "they must agree")
        return
    if a.gpus <= 1:
        return
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.run(cmd, env=env).returncode)


def make_net(device, num_classes=200, precision="fp32"):
    from count_pipnet_amd.pipnet import get_pipnet, set_hip_dtype
    from count_pipnet_amd.synthetic import fill_module_
    args = argparse.Namespace(net="convnext_tiny_26", disable_pretrained=True, num_features=0, bias=False)
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_pipnet(num_classes, args)
    fill_module_(net, 21, "trained")
    set_hip_dtype(net, precision)
    return net.eval().to(device), args


# the other GPU configs of BASELINE.json, timed per rank after the headline (tools/bench_configs.py
# holds the same definitions for stand-alone runs)
EXTRA = {
    # C3: the bf16 stem runs as a 4x4 conv over the 2x2 space-to-depth image (K = 256 with exact
    # zeros instead of the 7x7x3 = 147 products) fused with the max-pool (5 stem rows computed per
    # 2 pooled rows): 2*112^2*64*(1.25*256 - 147) more flops per image than the reference's stem
    "c3": dict(baseline="configs[2]", model="pipnet", batch=128, size=224, classes=200, gflop=38.16,
               gflop_executed=38.16 + 2 * 112 * 112 * 64 * (1.25 * 256 - 147) / 1e9,
               dtype="bf16", peak=PEAK_BF16_TFLOPS,
               workload_base="PIP-Net ResNet-50 forward(inference=True), 224x224, 200 classes, bf16 activations / "
                             "weights with fp32 accumulation, 128 images per GPU",
               args=dict(net="resnet50", num_features=0, bias=False, hip_dtype="bf16")),
    # C5: 1.374 GFLOP/img is the reference algorithm's work; the HIP path folds the bilinear
    # intermediate's embedding into W / V (count_pipnet.py _bilinear_folded: 2*(P*D + 2*D^2) ->
    # 2*2*P*D flops per image, P = 2048, D = 6144), so it executes 1.248 GFLOP/img
    "c5": dict(baseline="configs[4]", model="count", batch=64, size=128, classes=9, gflop=1.374,
               gflop_executed=1.374 - 2 * (2048 * 6144 + 2 * 6144 * 6144 - 2 * 2048 * 6144) / 1e9,
               dtype="f32", peak=PEAK_F32_TFLOPS,
               workload_base="CountPIPNet bilinear forward(inference=True), 2048 prototypes, hard Gumbel head "
                             "(Philox noise), 128x128, 9 classes, 64 images per GPU",
               args=dict(net="convnext_tiny_26", use_mid_layers=True, num_stages=3, num_features=2048,
                         activation="gumbel_softmax", intermediate_layer="bilinear", max_count=3, use_ste=True,
                         bias=False)),
}


def extra_layout(name, world, rank):
    """How BASELINE config ``name`` runs on ``world`` ranks, and the label that says so exactly.
    Returns (group ranks or None for the whole world, ranks per group, workload label).
    * c3 = configs[2], a 1-GPU config: every rank runs its own 128-image configs[2] batch (a
      per-rank replica), the N shards joined by the all-gather of logits / pooled.
    * c5 = configs[4], 256 images over 4 GPUs (64 per GPU): for N a multiple of 4 the world is cut
      into N / 4 independent 4-rank groups, each running configs[4] exactly (all-gather inside its
      group); for N < 4 (or not a multiple of 4) the N ranks run 64-image shards of its layout."""
    cfg = EXTRA[name]
    if name == "c5":
        if world >= 4 and world % 4 == 0:
            g = rank // 4
            label = (f"{cfg['workload_base']}, BASELINE configs[4] exactly: 256 images over 4 GPUs (64 per GPU), "
                     f"run as {world // 4} independent 4-rank group(s) with the all-gather inside each group "
                     f"({world * cfg['batch']} images per step in all)")
            return (list(range(4 * g, 4 * g + 4)) if world > 4 else None), 4, label
        label = (f"{cfg['workload_base']}, {world} rank(s) x 64-image shards of BASELINE configs[4]'s layout "
                 f"(configs[4] itself is 256 images over 4 GPUs)"
                 + (", all-gather over the ranks" if world > 1 else ""))
        return None, world, label
    if world == 1:
        return None, 1, f"{cfg['workload_base']}, BASELINE configs[2] (1 GPU)"
    return None, world, (f"{cfg['workload_base']}; BASELINE configs[2] is a 1-GPU config: each of the {world} ranks "
                         f"runs its own configs[2] batch (per-rank replica, {world * cfg['batch']} images per step), "
                         f"all-gather of logits / pooled over the {world} ranks")


def make_extra(cfg, dev):
    from count_pipnet_amd.count_pipnet import get_count_network
    from count_pipnet_amd.pipnet import get_pipnet
    from count_pipnet_amd.synthetic import fill_module_
    a = argparse.Namespace(disable_pretrained=True, backward_clamp_strategy="Gated", **cfg["args"])
    with contextlib.redirect_stdout(io.StringIO()):
        if cfg["model"] == "pipnet":
            net, _ = get_pipnet(cfg["classes"], a)
        else:
            net, _ = get_count_network(cfg["classes"], a, max_count=a.max_count, use_ste=a.use_ste)
    fill_module_(net, 7, "trained")
    return net.eval().to(dev)


class GemmTimer:
    """Brackets every MFMA GEMM / conv launch with HIP events on the launching stream."""

    def __init__(self):
        self.rec = []
        self.enabled = False

    def __call__(self, kname, flops, fn):
        if not self.enabled:
            fn()
            return
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        fn()
        e1.record(s)
        self.rec.append((kname, flops, e0, e1))

    def summary(self):
        agg = {}
        for kname, flops, e0, e1 in self.rec:
            a = agg.setdefault(kname, [0, 0.0, 0.0])
            a[0] += 1
            a[1] += flops
            a[2] += e0.elapsed_time(e1) * 1e-3
        return agg


def measured_traffic(dom):
    """HBM bytes per launch of the dominant kernel from the committed PMC measurement
    (tools/pmc.sh -> tools/pmc_summary.py -> profiles/traffic_latest.json for the headline's
    GEMM, profiles/traffic_kernels.json for the C3 / C5 kernels), used only when it was
    measured on this exact kernel: same kernel name AND same sha256 of the kernel family's
    sources.  Otherwise (kernel changed since the PMC pass) traffic is null."""
    from count_pipnet_amd.build import kernel_source_digest
    tr = None
    for name in ("traffic_latest.json", "traffic_kernels.json"):
        path = os.path.join(REPO, "profiles", name)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            d = json.load(f)
        if name == "traffic_latest.json" and d.get("kernel_key") == dom:
            tr, src = d, name
            break
        if name == "traffic_kernels.json" and dom in d:
            tr, src = d[dom], name
            break
    if tr is None:
        return None, "no PMC measurement of this kernel"
    if not tr.get("source_digest") or tr["source_digest"] != kernel_source_digest(dom):
        return None, "PMC measurement predates the current kernel sources (digest mismatch)"
    return tr.get("hbm_bytes_per_launch"), f"profiles/{src} (" + tr.get("method", "") + ")"


def _cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def host_cpu_share():
    """The host cores this process may actually use: its scheduler affinity and its cgroup
    CPU quota (v2 ``cpu.max`` or v1 ``cpu.cfs_quota_us / cpu.cfs_period_us``).  Returns
    (cores, affinity, quota_cpus or None, source)."""
    aff = len(os.sched_getaffinity(0))
    quota, src = None, "no cgroup CPU quota found"
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as f:
                q, p = f.read().split()[:2]
            if q != "max":
                quota, src = float(q) / float(p), f"{path} = {q} {p}"
            else:
                src = f"{path} = max"
            break
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            if q > 0:
                quota, src = q / p, f"cgroup v1 cfs_quota_us/cfs_period_us = {q}/{p}"
        except (OSError, ValueError):
            pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return cores, aff, quota, src


def cpu_baseline(batch=64, repeats=3):
    """The oracle (pure-torch CPU restatement of the reference forward, parity-pinned to the
    reference's goldens) on the host cores, by SURVEY.md 8(d) / BASELINE.md's protocol:
    the same 64-image 224x224 batch as the GPU step, 1 warm-up forward, then the median of
    3 timed forwards, on as many torch threads as the process has host cores (affinity and
    cgroup quota)."""
    import statistics
    from oracle import ref_cpu
    from count_pipnet_amd.synthetic import synth_images
    cores, aff, quota, src = host_cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    try:
        net, args = make_net(torch.device("cpu"))
        sd = {k: v for k, v in net.state_dict().items()}
        xs = synth_images(batch, 224, seed=1)
        times = []
        with torch.no_grad():
            ref_cpu.pipnet_forward(xs, sd, args, inference=True)       # warm-up
            for _ in range(repeats):
                t0 = time.perf_counter()
                ref_cpu.pipnet_forward(xs, sd, args, inference=True)
                times.append(time.perf_counter() - t0)
        threads = torch.get_num_threads()
    finally:
        torch.set_num_threads(prev)
    med = statistics.median(times)
    return {"value": batch / med, "unit": "images/sec", "cores": threads, "kind": "port",
            "affinity_cpus": aff, "cgroup_quota_cpus": quota, "quota_source": src,
            "nproc": os.cpu_count(), "cpu_model": _cpu_model(), "torch_threads": threads,
            "batch_seconds": times,
            "sample": f"one {batch}-image 224x224 batch (ConvNeXt-tiny-26 PIP-Net fp32, inference=True), "
                      f"1 warm-up + median of {repeats} = {med:.2f} s/batch; oracle/ref_cpu.py pipnet_forward "
                      f"on {threads} torch threads = the process's host-core share (affinity {aff} CPUs, "
                      f"cgroup quota {quota if quota is not None else 'none'}); nproc={os.cpu_count()}, "
                      f"CPU: {_cpu_model()}"}


def main():
    a = parse_args()
    launch_ranks_if_needed(a)

    from count_pipnet_amd import build, kernels
    from count_pipnet_amd.dist import ShardedInference, init_from_env
    rank, world, dev = init_from_env(a.dist_backend, a.device_index)
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the process group has {world} ranks")
    build.build()
    from count_pipnet_amd.synthetic import synth_images
    classes = a.classes if a.classes is not None else (196 if world == 8 else 200)
    net, _ = make_net(dev, num_classes=classes, precision=a.precision)
    # one process per GPU, weights resident, this rank's 64-image shard already in HBM; the
    # step ends with the RCCL all-gather of pooled + logits (DataParallel's gather)
    sharded = ShardedInference(net)
    xs = synth_images(a.batch, 224, seed=100 + rank).to(dev)
    if a.stream_split is not None:
        from count_pipnet_amd.pipnet import set_stream_split as _sss
        _sss(net, a.stream_split)

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(model, inp, batch, steps, warmup, instrument=False, gw=None):
        """W warm-up steps, then K steps bracketed by barrier + synchronize, max over ranks.
        ``instrument``: every MFMA GEMM / conv launch in the timed region is bracketed by HIP
        events on the stream it is launched on (torch's current stream) for the
        dominant-kernel roofline -- a separate pass, so the events' own cost never enters
        ``value``."""
        def step():
            with torch.no_grad():
                model(inp, inference=True, global_batch=False, sizes=[batch] * (gw or world))
        for _ in range(warmup):
            step()
        timer = GemmTimer()
        if instrument:
            kernels.set_launch_hook(timer)
            if world > 1:
                model.exchange_events = []      # the pooled + logits all-gather, event-timed per step
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        timer.enabled = instrument
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        timer.enabled = False
        kernels.set_launch_hook(None)
        agg = timer.summary()
        ev = getattr(model, "exchange_events", None)
        if ev:
            # the last `steps` exchanges are the timed ones; mean ms per step, max over ranks below
            agg["__exchange_ms__"] = sum(e0.elapsed_time(e1) for e0, e1 in ev[-steps:]) / min(steps, len(ev))
            model.exchange_events = None
        if world > 1:
            t = torch.tensor([elapsed, agg.get("__exchange_ms__", 0.0)], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t[0].item())
            if "__exchange_ms__" in agg:
                agg["__exchange_ms__"] = float(t[1].item())
        return elapsed, agg

    def roofline(agg, steps, peak_of):
        agg = {k: v for k, v in agg.items() if not k.startswith("__")}
        # dominant kernel = largest total time per step (the one definition: tools/pmc_summary.py's
        # `dominant:` line uses the same rule)
        dom = max(agg, key=lambda k: agg[k][2])
        n_l, fl, tt = agg[dom]
        peak = peak_of(dom)
        traffic, source = measured_traffic(dom)
        return dom, {"bound": "mfma", "kernel": dom, "achieved": fl / tt / 1e12, "peak": peak, "unit": "TFLOP/s",
                     "frac": fl / tt / 1e12 / peak, "traffic": traffic, "traffic_source": source,
                     "launches_per_step": n_l / steps,
                     "avg_launch_us": tt / n_l * 1e6, "algorithmic_gflop_per_launch": fl / n_l / 1e9}

    def peak_for(split):
        # split-bf16 GEMMs run 3 bf16 products per fp32 product: their fp32-equivalent ceiling
        # is the bf16 dense peak / 3 (achieved counts the algorithmic 2*M*N*K fp32 flops)
        return lambda dom: PEAK_BF16_TFLOPS / 3.0 if split and "bf16" in dom else PEAK_F32_TFLOPS

    from count_pipnet_amd.pipnet import set_stream_split, stream_split

    def measure(model, inner, inp, batch, steps, peak_of, gw=None):
        """Throughput with the model's default stream split (clean pass), then the roofline
        pass: one stream (per-kernel events must not overlap another stream's kernels),
        instrumented.  ``gw``: ranks in the model's process group (default: the world); the
        barriers and the max-over-ranks time always span the whole world.  Returns (elapsed,
        roofline dict, agg, extra fields)."""
        nsplit = stream_split(inner, inp)
        el, _ = timed(model, inp, batch, steps, a.warmup, gw=gw)
        set_stream_split(inner, 1)
        el1, agg = timed(model, inp, batch, steps, max(1, a.warmup // 2), instrument=True, gw=gw)
        set_stream_split(inner, nsplit)
        exch = agg.pop("__exchange_ms__", None)
        _, roof = roofline(agg, steps, peak_of)
        info = {"stream_split": nsplit, "roofline_pass": {"streams": 1, "instrumented": True,
                                                          "ms_per_step": el1 / steps * 1e3}}
        if exch is not None:
            info["exchange_ms_per_step"] = exch
        return el, roof, agg, info

    split = a.precision == "bf16x3"
    elapsed, roof, agg, info = measure(sharded, net, xs, a.batch, a.steps, peak_for(split))
    dom = roof["kernel"]
    gemm_flops = sum(v[1] for v in agg.values())
    gemm_time = sum(v[2] for v in agg.values())
    imgs = a.batch * world * a.steps
    ms = elapsed / a.steps * 1e3
    cfg_name = "configs[3]: CARS, 196 classes, 512 images over 8 GPUs" if (world == 8 and classes == 196) \
        else f"configs[1]: CUB-200, {classes} classes"
    result = {
        "metric": METRIC,
        "value": imgs / elapsed,
        "unit": "images/sec",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (bf16x3 split-product GEMMs)" if split else "f32",
        "data": "synthetic",
        "config": {"workload": f"PIP-Net ConvNeXt-tiny-26 forward(inference=True), 224x224, fp32, "
                               f"BASELINE {cfg_name}" + (", split-bf16 GEMMs" if split else ""),
                   "num_classes": classes, "global_batch": a.batch * world, "per_gpu_batch": a.batch,
                   "image_size": 224, "parallelism": f"dp{world}",
                   "exchange": {"collective": ("rccl" if dist.get_backend() == "nccl" else dist.get_backend())
                                + " all_gather_into_tensor([pooled | logits])", "collectives_per_step": 1,
                                "ms_per_step": info.get("exchange_ms_per_step"),
                                "timing": "HIP events around the packed all-gather on the current stream, "
                                          "roofline pass, mean over the timed steps, max over ranks"}
                               if world > 1 else None},
        "roofline": roof,
        "model_tflops": GFLOP_C2 * a.batch / (ms * 1e-3) / 1e3,
        "model_frac_of_f32_peak": GFLOP_C2 * a.batch / (ms * 1e-3) / 1e3 / PEAK_F32_TFLOPS,
        "gemm_all": {"tflops": gemm_flops / gemm_time / 1e12,
                     "ms_per_step": gemm_time / a.steps * 1e3, "pass": "roofline pass (one stream)"},
    }
    result.update(info)
    if a.alt_precision != "none" and a.alt_precision != a.precision:
        # the same network and inputs with the other GEMM precision, timed the same way
        from count_pipnet_amd.pipnet import set_hip_dtype
        set_hip_dtype(net, a.alt_precision)
        el2, roof2, _, info2 = measure(sharded, net, xs, a.batch, a.steps, peak_for(a.alt_precision == "bf16x3"))
        ms2 = el2 / a.steps * 1e3
        result["alt_precision"] = {
            "precision": a.alt_precision,
            "dtype": "f32 (bf16x3 split-product GEMMs)" if a.alt_precision == "bf16x3" else "f32",
            "value": imgs / el2, "ms_per_step": ms2, "roofline": roof2,
            "model_tflops_f32_equivalent": GFLOP_C2 * a.batch / (ms2 * 1e-3) / 1e3,
            "accuracy": "fp32 inputs/outputs and accumulation; products of hi+lo bf16 splits (~1e-5 relative "
                        "per product); parity vs the reference goldens at the north-star 1e-3 "
                        "(tests/test_gpu_parity.py::test_hip_bf16x3_*)" if a.alt_precision == "bf16x3" else "exact"}
        result["alt_precision"].update(info2)
    del sharded, net, xs
    torch.cuda.empty_cache()

    if not a.no_extra:
        extra = {}
        for name, cfg in EXTRA.items():
            enet = make_extra(cfg, dev)
            granks, gw, label = extra_layout(name, world, rank)
            group = None
            if world > 1 and granks is not None:
                # every rank creates every group, in the same order (torch.distributed contract)
                groups = [dist.new_group(list(range(g0, g0 + gw))) for g0 in range(0, world, gw)]
                group = groups[rank // gw]
            if a.stream_split is not None:
                set_stream_split(enet, a.stream_split)
            ewrap = ShardedInference(enet, process_group=group)
            exs = synth_images(cfg["batch"], cfg["size"], seed=200 + rank).to(dev)
            esteps = max(a.steps, 10)
            el, eroof, _, einfo = measure(ewrap, enet, exs, cfg["batch"], esteps, lambda dom, p=cfg["peak"]: p,
                                          gw=gw)
            gx = cfg.get("gflop_executed", cfg["gflop"])
            gm = min(gx, cfg["gflop"])   # model TF/s: the smaller of the reference's and the executed FLOPs
            rec = {"baseline": cfg["baseline"], "workload": label, "dtype": cfg["dtype"],
                   "ranks_per_group": gw, "groups": world // gw,
                   "per_gpu_batch": cfg["batch"], "global_batch": cfg["batch"] * world, "image_size": cfg["size"],
                   "value": cfg["batch"] * world * esteps / el, "unit": "images/sec",
                   "ms_per_step": el / esteps * 1e3, "steps": esteps,
                   "model_tflops": gm * cfg["batch"] / (el / esteps) / 1e3,
                   "model_frac_of_peak": gm * cfg["batch"] / (el / esteps) / 1e3 / cfg["peak"],
                   "model_gflop_per_image": {"reference": cfg["gflop"], "executed": gx, "counted": gm},
                   "roofline": eroof}
            rec.update(einfo)
            extra[name] = rec
            del ewrap, enet, exs
            torch.cuda.empty_cache()
        result["extra"] = extra
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
