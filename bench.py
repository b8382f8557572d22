"""Throughput of the MI355X PIP-Net inference path (BASELINE.json metric).

A "step" = one ``PIPNet.forward(xs, inference=True)`` of ConvNeXt-tiny-26 over one batch of
64 synthetic 224x224 images per GPU (CUB-200 shape, 200 classes, fp32), inputs resident in
HBM, plus -- for N > 1 -- the RCCL all-gather of logits and pooled presence over xGMI that
replaces nn.DataParallel's gather (main.py:118).  Weak scaling: 64 images per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints one JSON line on rank 0 (fields described in DESIGN.md section "Measurement").
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
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


def make_net(device, num_classes=200, precision="fp32"):
    from count_pipnet_amd.pipnet import get_pipnet, set_hip_dtype
    from count_pipnet_amd.synthetic import fill_module_
    args = argparse.Namespace(net="convnext_tiny_26", disable_pretrained=True, num_features=0, bias=False)
    with contextlib.redirect_stdout(io.StringIO()):
        net, _ = get_pipnet(num_classes, args)
    fill_module_(net, 21, "trained")
    set_hip_dtype(net, precision)
    return net.eval().to(device), args


class GemmTimer:
    """Brackets every MFMA GEMM launch with HIP events on the launching stream."""

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
    (tools/pmc.sh -> tools/pmc_summary.py -> profiles/traffic_latest.json), used only when it
    was measured on this exact kernel: same kernel name AND same sha256 of the kernel
    family's sources.  Otherwise (kernel changed since the PMC pass) traffic is null."""
    from count_pipnet_amd.build import kernel_source_digest
    path = os.path.join(REPO, "profiles", "traffic_latest.json")
    if not os.path.exists(path):
        return None, "no PMC measurement"
    with open(path) as f:
        tr = json.load(f)
    if tr.get("kernel_key") != dom:
        return None, f"PMC measurement is of another kernel ({tr.get('kernel_key')})"
    if not tr.get("source_digest") or tr["source_digest"] != kernel_source_digest(dom):
        return None, "PMC measurement predates the current kernel sources (digest mismatch)"
    return tr.get("hbm_bytes_per_launch"), "profiles/traffic_latest.json (" + tr.get("method", "") + ")"


def _cpu_model():
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def cpu_baseline(batch=64, repeats=3):
    """The oracle (pure-torch CPU restatement of the reference forward, parity-pinned to the
    reference's goldens) on the host cores, by SURVEY.md 8(d) / BASELINE.md's protocol:
    the same 64-image 224x224 batch as the GPU step, 1 warm-up forward, then the median of
    3 timed forwards.  Reports nproc, the lscpu model name and torch's thread count."""
    import statistics
    from oracle import ref_cpu
    from count_pipnet_amd.synthetic import synth_images
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
    med = statistics.median(times)
    threads = torch.get_num_threads()
    return {"value": batch / med, "unit": "images/sec", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "cpu_model": _cpu_model(), "torch_threads": threads,
            "batch_seconds": times,
            "sample": f"one {batch}-image 224x224 batch (ConvNeXt-tiny-26 PIP-Net fp32, inference=True), "
                      f"1 warm-up + median of {repeats} = {med:.2f} s/batch; oracle/ref_cpu.py pipnet_forward "
                      f"on {threads} torch threads; nproc={os.cpu_count()}, CPU: {_cpu_model()}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--precision", choices=["fp32", "bf16x3"], default="fp32",
                    help="fp32: exact fp32 MFMA GEMMs; bf16x3: split-bf16 GEMMs (fp32 in/out, ~1e-5 per product)")
    ap.add_argument("--alt-precision", choices=["none", "fp32", "bf16x3"], default="bf16x3",
                    help="also time this precision on the same network (reported under alt_precision)")
    ap.add_argument("--dist-backend", default=None,
                    help="rehearsal only: torch.distributed backend (default nccl = RCCL on GPUs)")
    ap.add_argument("--device-index", type=int, default=None,
                    help="rehearsal only: put every rank on this GPU (multi-rank runs on a 1-GPU box)")
    a = ap.parse_args()

    from count_pipnet_amd import build, kernels
    from count_pipnet_amd.dist import ShardedInference, init_from_env
    rank, world, dev = init_from_env(a.dist_backend, a.device_index)
    build.build()
    from count_pipnet_amd.synthetic import synth_images
    net, _ = make_net(dev, precision=a.precision)
    # one process per GPU, weights resident, this rank's 64-image shard already in HBM; the
    # step ends with the RCCL all-gather of pooled + logits (DataParallel's gather)
    sharded = ShardedInference(net)
    xs = synth_images(a.batch, 224, seed=100 + rank).to(dev)

    def step():
        with torch.no_grad():
            _, pooled, out = sharded(xs, inference=True, global_batch=False, sizes=[a.batch] * world)
        return out

    def barrier():
        if world > 1:
            dist.barrier()

    def timed():
        """W warm-up steps, then K steps bracketed by barrier + synchronize; every MFMA GEMM
        launch in the timed region is bracketed by HIP events on the stream it is launched
        on (torch's current stream) for the dominant-kernel roofline.  Max over ranks."""
        for _ in range(a.warmup):
            step()
        timer = GemmTimer()
        kernels.set_launch_hook(timer)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        timer.enabled = True
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        timer.enabled = False
        kernels.set_launch_hook(None)
        if world > 1:
            t = torch.tensor([elapsed], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, timer.summary()

    def roofline(agg, split):
        dom = max(agg, key=lambda k: agg[k][2])
        n_l, fl, tt = agg[dom]
        # split-bf16 GEMMs run 3 bf16 products per fp32 product: their fp32-equivalent ceiling
        # is the bf16 dense peak / 3 (achieved counts the algorithmic 2*M*N*K fp32 flops)
        peak = PEAK_BF16_TFLOPS / 3.0 if split and "bf16" in dom else PEAK_F32_TFLOPS
        return dom, {"bound": "mfma", "kernel": dom, "achieved": fl / tt / 1e12, "peak": peak, "unit": "TFLOP/s",
                     "frac": fl / tt / 1e12 / peak, "traffic": None, "launches_per_step": n_l / a.steps,
                     "avg_launch_us": tt / n_l * 1e6, "algorithmic_gflop_per_launch": fl / n_l / 1e9}

    gflop_img = 40.094159616       # oracle.ref_cpu.gflop_per_image(convnext_tiny_26, 224)
    elapsed, agg = timed()
    split = a.precision == "bf16x3"
    dom, roof = roofline(agg, split)
    gemm_flops = sum(v[1] for v in agg.values())
    gemm_time = sum(v[2] for v in agg.values())
    imgs = a.batch * world * a.steps
    ms = elapsed / a.steps * 1e3
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
        "config": {"workload": "PIP-Net ConvNeXt-tiny-26 forward(inference=True), 224x224, 200 classes, fp32 "
                               "(BASELINE configs[1]; configs[3] at N=8)" + (", split-bf16 GEMMs" if split else ""),
                   "global_batch": a.batch * world, "per_gpu_batch": a.batch, "image_size": 224,
                   "parallelism": f"dp{world}", "exchange": (("rccl" if dist.get_backend() == "nccl" else dist.get_backend())
                                + " all_gather(logits, pooled)") if world > 1 else None},
        "roofline": roof,
        "model_tflops": gflop_img * a.batch * world / (ms * 1e-3) / 1e3 / world,
        "model_frac_of_f32_peak": gflop_img * a.batch / (ms * 1e-3) / 1e3 / PEAK_F32_TFLOPS,
        "gemm_all": {"tflops": gemm_flops / gemm_time / 1e12, "ms_per_step": gemm_time / a.steps * 1e3},
    }
    if a.alt_precision != "none" and a.alt_precision != a.precision:
        # the same network and inputs with the other GEMM precision, timed the same way
        from count_pipnet_amd.pipnet import set_hip_dtype
        set_hip_dtype(net, a.alt_precision)
        el2, agg2 = timed()
        _, roof2 = roofline(agg2, a.alt_precision == "bf16x3")
        ms2 = el2 / a.steps * 1e3
        result["alt_precision"] = {
            "precision": a.alt_precision,
            "dtype": "f32 (bf16x3 split-product GEMMs)" if a.alt_precision == "bf16x3" else "f32",
            "value": imgs / el2, "ms_per_step": ms2, "roofline": roof2,
            "model_tflops_f32_equivalent": gflop_img * a.batch / (ms2 * 1e-3) / 1e3,
            "accuracy": "fp32 inputs/outputs and accumulation; products of hi+lo bf16 splits (~1e-5 relative "
                        "per product); parity vs the reference goldens at the north-star 1e-3 "
                        "(tests/test_gpu_parity.py::test_hip_bf16x3_*)" if a.alt_precision == "bf16x3" else "exact"}
    result["roofline"]["traffic"], result["roofline"]["traffic_source"] = measured_traffic(dom)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
