"""A/B the fused CNBlock MLP instantiations of tools/mlp_lab.hip on the C2 / C5 stage-1/2 shapes
(interleaved rounds in one process); variant 0 = the product's choice.  Every variant's output
is checked against the product library's.

    python tools/mlp_lab.py
"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402

from count_pipnet_amd import build  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

SO = os.path.join(HERE, "libmlp_lab.so")
VARIANTS = {96: [0], 192: [0, 21]}
if os.environ.get("LAB_VARIANTS"):
    VARIANTS = json.loads(os.environ["LAB_VARIANTS"])
    VARIANTS = {int(k): v for k, v in VARIANTS.items()}


def main():
    src = os.path.join(HERE, "mlp_lab.hip")
    dep = os.path.join(HERE, "..", "count_pipnet_amd", "csrc", "mlp_f32.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(dep)):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", src,
                        "-o", SO, "-I", os.path.join(HERE, "..", "include")], check=True)
    if "--build-only" in sys.argv:
        return
    build.build()
    lab = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lab.pipnet_cnblock_mlp_f32.argtypes = [P, P, P, P, P, P, P, ctypes.c_int64, ctypes.c_int, P]
    lab.mlp_lab_set.argtypes = [ctypes.c_int]
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    rounds = int(os.environ.get("LAB_ROUNDS", "5"))
    shapes = [(96, 64 * 56 * 56), (192, 64 * 28 * 28), (96, 64 * 32 * 32), (192, 64 * 16 * 16)]
    if os.environ.get("LAB_SHAPES"):      # e.g. "96x100352,192x25088" (C x M): the two-stream half batches
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["LAB_SHAPES"].split(",")]
    for c, m in shapes:
        t = torch.randn(m, c, device=dev, generator=g)
        x0 = torch.randn(m, c, device=dev, generator=g)
        w1 = torch.randn(4 * c, c, device=dev, generator=g) * 0.1
        b1 = torch.randn(4 * c, device=dev, generator=g) * 0.1
        w2 = torch.randn(c, 4 * c, device=dev, generator=g) * 0.05
        b2 = torch.randn(c, device=dev, generator=g)
        gm = torch.randn(c, device=dev, generator=g)
        ref = x0.clone()
        K.cnblock_mlp(t, w1, b1, w2, b2, gm, ref)
        res = {}
        for _ in range(rounds):
            for v in VARIANTS[c]:
                lab.mlp_lab_set(v)
                x = x0.clone()

                def run():
                    st = lab.pipnet_cnblock_mlp_f32(t.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                                                    b2.data_ptr(), gm.data_ptr(), x.data_ptr(), m, c, stream)
                    assert st == 0, st
                run()
                torch.cuda.synchronize()
                ok = torch.allclose(x, ref, rtol=1e-5, atol=1e-5)
                for _ in range(2):
                    run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    run()
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(v, []).append((e0.elapsed_time(e1) / 10, ok))
        fl = 2.0 * 2 * m * 4 * c * c
        rec = {"C": c, "M": m}
        for v, lst in res.items():
            ms = sorted(x[0] for x in lst)[len(lst) // 2]
            rec[f"v{v}"] = {"us": round(ms * 1e3, 1), "tflops": round(fl / (ms * 1e-3) / 1e12, 1),
                            "ok": all(x[1] for x in lst)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
