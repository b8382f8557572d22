"""Per-workgroup phase timing of the fp32 GEMM on the network's shapes (lab variants 30/32/33
= product variants with in-kernel s_memtime stamps, tools/gemm_lab.hip).  For each shape:
prologue (first K-tile DMA wait), cycles per K-tile in the main loop, epilogue, and how the
CU slots are used over the kernel's span (tail / dispatch gaps).
    python tools/gemm_stamps.py [shape,...]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libgemm_lab.so"))
P, I32, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lib.lab_linear.argtypes = [I32, I32, P, I64, P, P, P, P, I64, P, I64, I32, I32, I32, I32, P]
lib.lab_set_stamps.argtypes = [P]


def shapes(batch=64):
    batch *= int(os.environ.get("STAMP_MSCALE", "1"))     # longer dispatches (clock reconciliation)
    out = []
    for d, hw in [(96, 56), (192, 28), (384, 27), (768, 26)]:
        m = batch * hw * hw
        out.append((f"s{d}_fc1", m, 4 * d, d, _lib.EPI_BIAS_GELU))
        out.append((f"s{d}_fc2", m, d, 4 * d, _lib.EPI_RESID))
    return out


def variant_for(m, n, k):      # mirrors gemm_variant in csrc/gemm_f32.hip
    if k % 16 == 0 and k <= 96 and n > 192 and m > 64:
        return 33, 128, 16
    if n <= 384 or k <= 192 or m <= 64:
        return 32, 64, 32
    return 30, 128, 32


def main():
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    stream = torch.cuda.current_stream().cuda_stream
    for name, m, n, k, epi in shapes():
        if only and name not in only:
            continue
        v, bm, bk = variant_for(m, n, k)
        if os.environ.get("STAMP_VAR"):            # e.g. 37 = the 3-workgroup BK16 tile (lab v7)
            v, bm, bk = int(os.environ["STAMP_VAR"]), 128, 16
        if os.environ.get("STAMP_V16") == "1" and v == 30:
            v = 70                      # the same tile on v_mfma_f32_16x16x4_f32
        mt, nt = -(-m // bm), -(-n // 128)
        nwg = mt * nt
        nk = k // bk
        A = torch.randn(m, k, device=dev, generator=g)
        W = torch.randn(n, k, device=dev, generator=g) * 0.05
        b = torch.randn(n, device=dev, generator=g)
        s = torch.randn(n, device=dev, generator=g)
        R = torch.randn(m, n, device=dev, generator=g)
        C = torch.empty(m, n, device=dev)
        st = torch.zeros(nwg * 16, dtype=torch.int64, device=dev)
        lib.lab_set_stamps(st.data_ptr())
        for _ in range(4):
            assert lib.lab_linear(v, 8, A.data_ptr(), k, W.data_ptr(), b.data_ptr(), s.data_ptr(), R.data_ptr(), n,
                                  C.data_ptr(), n, m, n, k, epi, stream) == 0
        torch.cuda.synchronize()
        a = st.view(nwg, 16).cpu().numpy()
        lib.lab_set_stamps(None)
        pro, main_, epi_ = a[:, 1] - a[:, 0], a[:, 2] - a[:, 1], a[:, 3] - a[:, 2]
        rt0, rt1 = a[:, 6], a[:, 7]
        span_rt = rt1.max() - rt0.min()                       # 100 MHz ticks
        life_rt = rt1 - rt0
        hw, xcc = a[:, 4], a[:, 5]
        cu = xcc * 4096 + ((hw >> 8) & 0xFF)
        ncu = len(np.unique(cu))
        per_cu = np.bincount(np.unique(cu, return_inverse=True)[1])
        clk = (a[:, 3] - a[:, 0]).sum() / max(life_rt.sum(), 1) * 100e6
        occ = life_rt.sum() / (span_rt * ncu)
        print(f"{name:9s} v{v} M={m} N={n} K={k} wg={nwg} grid={nwg * 256} nk={nk} CUs={ncu} wg/CU={per_cu.min()}..{per_cu.max()} "
              f"clk={clk / 1e9:.2f}GHz span={span_rt / 100:.1f}us", flush=True)
        print(f"   cycles median: prologue {np.median(pro):.0f}  main {np.median(main_):.0f} "
              f"({np.median(main_) / nk:.0f}/K-tile)  epilogue {np.median(epi_):.0f} | "
              f"p90 prologue {np.percentile(pro, 90):.0f} epi {np.percentile(epi_, 90):.0f}", flush=True)
        if (a[:, 8] > 0).all():          # vector epilogue sub-phases (wave 0's view), cycles
            ph = [a[:, 8] - a[:, 2], a[:, 9] - a[:, 8]]
            names = ["relayout0", "math+stores0"]
            if (a[:, 10] > 0).all():
                ph += [a[:, 10] - a[:, 9], a[:, 11] - a[:, 10], a[:, 3] - a[:, 11]]
                names += ["relayout1", "math+stores1", "to end"]
            else:
                ph += [a[:, 3] - a[:, 9]]
                names += ["to end"]
            print("   epilogue median cycles: " + "  ".join(f"{nm} {np.median(v):.0f}" for nm, v in zip(names, ph)),
                  flush=True)
            if (a[:, 12] > 0).all() and (a[:, 15] > 0).all():   # first slab, per store iteration
                it = [a[:, 12] - a[:, 8], a[:, 13] - a[:, 12], a[:, 14] - a[:, 13], a[:, 15] - a[:, 14],
                      a[:, 9] - a[:, 15]]
                print("   first slab median cycles: it0 {:.0f}  it1 {:.0f}  it2-3 {:.0f}  it4-5 {:.0f}  it6-7 {:.0f}".format(
                    *[np.median(v) for v in it]), flush=True)
        share = (pro.sum(), main_.sum(), epi_.sum())
        tot = sum(share)
        print(f"   wg-time share: prologue {share[0] / tot:.3f} main {share[1] / tot:.3f} epilogue {share[2] / tot:.3f}"
              f" | resident WGs/CU avg {occ:.2f} over the span", flush=True)
        # epilogue coincidence: per CU, how much of its workgroups' epilogue time overlaps another
        # resident workgroup's epilogue (both slots off the MFMA pipe), memtime -> realtime per WG
        scale = (rt1 - rt0) / np.maximum(a[:, 3] - a[:, 0], 1)
        e0 = rt0 + (a[:, 2] - a[:, 0]) * scale
        e1 = rt1
        both = tot_e = 0.0
        for c in np.unique(cu):
            idx = np.nonzero(cu == c)[0]
            ev = sorted([(e0[i], 1) for i in idx] + [(e1[i], -1) for i in idx])
            depth, last = 0, None
            for t, d in ev:
                if last is not None and depth >= 2:
                    both += t - last
                depth += d
                last = t
            tot_e += (e1[idx] - e0[idx]).sum()
        print(f"   epilogue coincidence: {2 * both / max(tot_e, 1):.3f} of epilogue time overlaps another epilogue on the CU "
              f"(random phases at this share: ~{share[2] / tot:.3f})", flush=True)
        # tail: fraction of span after the first WG slot goes permanently idle
        order = np.sort(rt1)
        print(f"   tail: last 5% of WGs finish over {(order[-1] - order[int(0.95 * nwg)]) / 100:.1f}us, "
              f"first end {(order[0] - rt0.min()) / 100:.1f}us", flush=True)
        del A, W, R, C, st


if __name__ == "__main__":
    main()
