"""Throughput of the backward building blocks at the trainable-stage shapes of C2 training
(128 images of 26x26 pixels = 86,528 rows, C = 768, hidden 3072)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from count_pipnet_amd import kernels as K  # noqa: E402


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


def main():
    dev = torch.device("cuda:0")
    m = 128 * 26 * 26
    res = {}
    for n1, n2 in [(768, 3072), (3072, 768)]:
        a = torch.randn(m, n1, device=dev)
        b = torch.randn(m, n2, device=dev)
        out = torch.empty(n1, n2, device=dev)
        t = timeit(lambda: K.wgrad(a, b, out=out))
        tt = timeit(lambda: torch.mm(a.t(), b, out=out))
        res[f"wgrad_{n1}x{n2}"] = {"ms": t * 1e3, "tflops": 2.0 * m * n1 * n2 / t / 1e12,
                                    "torch_mm_ms": tt * 1e3, "torch_tflops": 2.0 * m * n1 * n2 / tt / 1e12}
    a = torch.randn(m, 3072, device=dev)
    t = timeit(lambda: K.colsum(a))
    res["colsum_86528x3072"] = {"ms": t * 1e3, "GBps": m * 3072 * 4 / t / 1e9}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
