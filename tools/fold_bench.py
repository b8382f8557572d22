"""Times the C5 bilinear fold (W.E and V.E, fp64 MFMA, csrc/fold_f64.hip) at its own shape:
M = 6144 (D), K = 6144 (D), N = 2048 (P), as two single launches and as the one-launch pair.
fp64 matrix peak of gfx950 taken as 78.6 TF/s (AMD spec; 32 FLOP/clk/SIMD at 2.4 GHz)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from count_pipnet_amd import kernels as K  # noqa: E402

PEAK_F64 = 78.6e12


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / reps * 1e-3


def main():
    d, p = 6144, 2048
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(d, d, generator=g) * 0.01).cuda()
    v = (torch.randn(d, d, generator=g) * 0.01).cuda()
    e = (torch.randn(d, p, generator=g) * 0.01).cuda()
    flop = 2.0 * d * d * p
    t1 = timed(lambda: K.matmul_f64acc(w, e))
    t2 = timed(lambda: K.matmul2_f64acc(w, v, e))
    print(json.dumps({"shape": [d, p, d], "single_ms": round(t1 * 1e3, 3), "pair_ms": round(t2 * 1e3, 3),
                      "pair_ms_per_product": round(t2 * 1e3 / 2, 3),
                      "single_frac_f64_peak": round(flop / t1 / PEAK_F64, 3),
                      "pair_frac_f64_peak": round(2 * flop / t2 / PEAK_F64, 3)}))


if __name__ == "__main__":
    main()
