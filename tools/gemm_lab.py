"""A/B the GEMM variants of tools/gemm_lab.hip on every network shape, interleaved rounds
in one process (cdna_hip_programming.md rule 24).  python tools/gemm_lab.py"""
import ctypes
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libgemm_lab.so"))
P, I32, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lib.lab_linear.argtypes = [I32, I32, P, I64, P, P, P, P, I64, P, I64, I32, I32, I32, I32, P]

VARIANTS = [int(v) for v in os.environ.get("LAB_VARIANTS", "0,1,2,3").split(",")]
GROUPS = [int(v) for v in os.environ.get("LAB_GROUPS", "1,4,8,16").split(",")]
# epilogues to run per shape: "native" = the network's own, or EPI codes (A/B the epilogue cost)
EPIS = os.environ.get("LAB_EPIS", "native").split(",")
ONLY = os.environ.get("LAB_SHAPES")


def shapes(batch=64):
    out = []
    for d, hw in [(96, 56), (192, 28), (384, 27), (768, 26)]:
        m = batch * hw * hw
        out.append((f"s{d}_fc1", m, 4 * d, d, _lib.EPI_BIAS_GELU))
        out.append((f"s{d}_fc2", m, d, 4 * d, _lib.EPI_RESID))
    out.append(("c5_addon", 64 * 16 * 16, 2048, 192, _lib.EPI_BIAS))    # C5: 1x1 add-on 192 -> 2048
    return out


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    stream = torch.cuda.current_stream().cuda_stream
    for name, m, n, k, epi0 in shapes():
        if ONLY and name not in ONLY.split(","):
            continue
        A = torch.randn(m, k, device=dev, generator=g)
        W = torch.randn(n, k, device=dev, generator=g) * 0.05
        b = torch.randn(n, device=dev, generator=g)
        s = torch.randn(n, device=dev, generator=g)
        R = torch.randn(m, n, device=dev, generator=g)
        C = torch.empty(m, n, device=dev)
        ref = {}
        times = {}
        epis = [epi0 if e == "native" else int(e) for e in EPIS]
        cfgs = list(itertools.product(VARIANTS, GROUPS, epis))
        for rnd in range(int(os.environ.get("LAB_ROUNDS", "3"))):
            for v, gm, epi in cfgs:
                def run():
                    st = lib.lab_linear(v, gm, A.data_ptr(), k, W.data_ptr(), b.data_ptr(), s.data_ptr(), R.data_ptr(),
                                        n, C.data_ptr(), n, m, n, k, epi, stream)
                    assert st == 0
                run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times.setdefault((v, gm, epi), []).append(e0.elapsed_time(e1) / 5 * 1e-3)
                if rnd == 0 and (v < 10 or 40 <= v < 70):
                    if epi not in ref:
                        ref[epi] = C.clone()
                    else:
                        err = (C - ref[epi]).abs().max().item()
                        assert err < 1e-3 * (1 + ref[epi].abs().max().item()), (v, gm, epi, err)
        f = 2.0 * m * n * k
        line = [f"{name:9s}"]
        best = min(times, key=lambda c: min(times[c]))
        for c in cfgs:
            t = min(times[c])
            line.append(f"v{c[0]}g{c[1]}e{c[2]}:{f / t / 1e12:5.1f}")
        print(" ".join(line), f"| best v{best[0]} g{best[1]} e{best[2]} {f / min(times[best]) / 1e12:.1f} TF", flush=True)
        del A, W, R, C, ref


if __name__ == "__main__":
    main()
