"""A/B the bf16 GEMM lab kernels (tools/bf16_lab.hip) on square and ResNet50 (C3) GEMM shapes,
interleaved rounds in one process (cdna_hip_programming.md rule 24), uniform [-1, 1) data.

    python tools/bf16_lab.py                 # builds tools/libbf16_lab.so if missing
    LAB_ABL=0,1,2,4 LAB_SHAPES=sq8192,l4ds python tools/bf16_lab.py
    LAB_ABL=0,1040,-1 ...   (1040 / 1042: the four-wave tile with AGPR accumulators; -1: hipBLASLt)
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402

SO = os.path.join(HERE, "libbf16_lab.so")
SHAPES = {   # name: (M, N, K)
    "sq4096": (4096, 4096, 4096), "sq8192": (8192, 8192, 8192),
    "l3c1": (100352, 256, 1024), "l3c3": (100352, 1024, 256), "l4c1": (100352, 512, 2048),
    "l4c3": (100352, 2048, 512), "l4ds": (100352, 2048, 1024), "l3c2eq": (100352, 256, 2304),
    "l4c2eq": (100352, 512, 4608),
}


def build():
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(
            os.path.getmtime(os.path.join(HERE, "bf16_lab.hip")),
            os.path.getmtime(os.path.join(HERE, "..", "count_pipnet_amd", "csrc", "gemm_bf16_impl.hpp"))):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        os.path.join(HERE, "bf16_lab.hip"), "-o", SO, "-I", os.path.join(HERE, "..", "include")],
                       check=True)
    lib = ctypes.CDLL(SO)
    lib.lab_pp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    return lib


def main():
    lib = build()
    if "--build-only" in sys.argv:
        return
    dev = torch.device("cuda:0")
    abls = [int(v) for v in os.environ.get("LAB_ABL", "0,1,2,4,8").split(",")]
    budgets = [float(v) * 1024 * 1024 for v in os.environ.get("LAB_BUDGET", "2").split(",")]
    names = os.environ.get("LAB_SHAPES", ",".join(SHAPES)).split(",")
    rounds = int(os.environ.get("LAB_ROUNDS", "3"))
    reps = int(os.environ.get("LAB_REPS", "10"))
    stream = torch.cuda.current_stream().cuda_stream
    for name in names:
        m, n, k = SHAPES[name]
        a = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
        c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        res = {}
        # correctness: the full-line kernel accumulates in the same k order as the 32-deep one
        for alt in (32, 256, 512, 1024, 1040):
            if alt not in abls or 0 not in abls:
                continue
            c2 = torch.empty_like(c)
            assert lib.lab_pp(0, a.data_ptr(), w.data_ptr(), c.data_ptr(), m, n, k, budgets[0], stream) == 0
            assert lib.lab_pp(alt, a.data_ptr(), w.data_ptr(), c2.data_ptr(), m, n, k, budgets[0], stream) == 0
            torch.cuda.synchronize()
            ref = (a[:512].float() @ w.float().t())
            err = (c[:512].float() - ref).abs().max().item() / ref.abs().max().item()
            print(f"{name}: variant {alt} == pp bitwise: {torch.equal(c, c2)}; pp vs fp32 matmul (first 512 rows) "
                  f"max rel err {err:.2e}", flush=True)
        for _ in range(rounds):
            for abl in abls:
                for bud in budgets:
                    def run():
                        if abl < 0:                                  # -1: hipBLASLt (torch matmul)
                            torch.matmul(a, w.t(), out=c)
                            return
                        st = lib.lab_pp(abl, a.data_ptr(), w.data_ptr(), c.data_ptr(), m, n, k, bud, stream)
                        assert st == 0, st
                    for _ in range(2):
                        run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(reps):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    res.setdefault((abl, bud), []).append(2.0 * m * n * k / (e0.elapsed_time(e1) / reps) / 1e9)
        line = f"{name:7s} M={m:6d} N={n:5d} K={k:5d}"
        for (abl, bud), v in res.items():
            v = sorted(v)
            line += f" | abl{abl}{'' if len(budgets) == 1 else f'/g{bud / 2**20:.0f}'}: {v[len(v) // 2]:6.0f}"
        print(line + "  TF (median of rounds)", flush=True)


if __name__ == "__main__":
    main()
