"""A/B the dwconv7+LN variants of tools/dw_lab.hip on the network's stage shapes (C2 224^2
and C5 128^2 inputs, batch 64): v0 = register-tile kernel, v1.. = row-ring variants, each
at a few (min workgroups, min rows per chunk) chunkings.  Prints us and HBM-algorithmic
TB/s (input read + output write once)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libdw_lab.so"))
P, I32 = ctypes.c_void_p, ctypes.c_int
lib.lab_dw.argtypes = [I32, P, I32, I32, I32, I32, P, P, P, P, P, P, I32, I32]

dev = torch.device("cuda:0")
stream = torch.cuda.current_stream().cuda_stream
CHUNKS = [(2048, 7), (1024, 7), (4096, 4), (512, 14)]
SHAPES = [(96, 56), (192, 28), (384, 27), (768, 26), (96, 32), (192, 16)]
if os.environ.get("DW_SHAPES"):
    SHAPES = [tuple(int(v) for v in t.split("x")) for t in os.environ["DW_SHAPES"].split(",")]
VARIANTS = [int(v) for v in os.environ.get("DW_VARIANTS", "0,5,6,7").split(",")]
for c, hw in SHAPES:
    x = torch.randn(64, hw, hw, c, device=dev)
    w = torch.randn(49, c, device=dev) * 0.2
    b, lw, lb = torch.randn(c, device=dev), torch.randn(c, device=dev), torch.randn(c, device=dev)
    y = torch.empty_like(x)
    ref = None
    res = {}
    combos = [(v, 2048, 7) for v in VARIANTS] + ([(v, mw, mr) for v in (1, 3) for mw, mr in CHUNKS[:2]]
                                                 if os.environ.get("DW_RING") else [])
    for rnd in range(3):
        for v, mw, mr in combos:
            args = (v, x.data_ptr(), 64, hw, hw, c, w.data_ptr(), b.data_ptr(), lw.data_ptr(), lb.data_ptr(),
                    y.data_ptr(), stream, mw, mr)
            y.fill_(float("nan"))
            assert lib.lab_dw(*args) == 0
            if rnd == 0:
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.clone()
                else:
                    err = (y - ref).abs().max().item()
                    assert err < 1e-3 or 32 <= v <= 39, (c, hw, v, mw, mr, err)   # v32-v39: ablations
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                lib.lab_dw(*args)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault((v, mw, mr), []).append(e0.elapsed_time(e1) / 10 * 1e3)
    gb = 2 * x.numel() * 4 / 1e9
    items = sorted(res.items(), key=lambda kv: min(kv[1]))
    print(f"C={c:4d} H=W={hw}: v0 {min(res[(0, 2048, 7)]):7.1f}us  best: " +
          " ".join(f"v{v}/{mw}/{mr}:{min(t):6.1f}us({gb / min(t) * 1e6 / 1e3:4.2f}TB/s)"
                   for (v, mw, mr), t in items[:6]), flush=True)

# ablations of v1 (no LN / no FMAs / no loads) at the C2 stage-1 and stage-3 shapes
if "--abl" in sys.argv:
    for c, hw in [(96, 56), (384, 27)]:
        x = torch.randn(64, hw, hw, c, device=dev)
        w = torch.randn(49, c, device=dev) * 0.2
        b, lw, lb = torch.randn(c, device=dev), torch.randn(c, device=dev), torch.randn(c, device=dev)
        y = torch.empty_like(x)
        out = []
        for v in (1, 11, 12, 14, 13, 16):
            args = (v, x.data_ptr(), 64, hw, hw, c, w.data_ptr(), b.data_ptr(), lw.data_ptr(), lb.data_ptr(),
                    y.data_ptr(), stream, 2048, 7)
            assert lib.lab_dw(*args) == 0
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    lib.lab_dw(*args)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 10 * 1e3)
            out.append(f"v{v}:{min(ts):6.1f}us")
        print(f"ablation C={c} ({'full', 'noLN', 'noFMA', 'noLoad', 'noLN+noFMA', 'noFMA+noLoad'}): " + " ".join(out),
              flush=True)

# round 6: ablation of the PRODUCT kernel bodies (v60 = product, checked bitwise against the library's
# pipnet_dwconv7_ln_f32) at C2's stage-3 / stage-4 / stage-1 shapes, batch 64
if "--abl6" in sys.argv:
    from count_pipnet_amd import kernels as K
    names = {60: "product", 61: "noLNstats", 62: "1FMA/row", 63: "noLoads", 64: "noStores", 65: "noWeights",
             66: "noLDStile", 67: "noLDS+noLN", 68: "noFMA+noLoads", 69: "noW+noLd+noFMA", 70: "noLDS+noSt+noLN",
             71: "noLN+noSt", 72: "LN+stores only", 73: "noLoads+noW"}
    for c, hw in [(384, 27), (768, 26), (96, 56)]:
        g = torch.Generator(device=dev).manual_seed(c)
        x = torch.randn(64, hw, hw, c, device=dev, generator=g)
        w = torch.randn(49, c, device=dev, generator=g) * 0.2
        b, lw, lb = (torch.randn(c, device=dev, generator=g) for _ in range(3))
        y = torch.empty_like(x)
        ref = K.dwconv7_ln(x, w, b, lw, lb)
        assert lib.lab_dw(60, x.data_ptr(), 64, hw, hw, c, w.data_ptr(), b.data_ptr(), lw.data_ptr(), lb.data_ptr(),
                          y.data_ptr(), stream, 2048, 7) == 0
        torch.cuda.synchronize()
        same = torch.equal(y, ref)
        gb = 2 * x.numel() * 4 / 1e9
        ts = {v: [] for v in names}
        for _ in range(3):
            for v in names:
                args = (v, x.data_ptr(), 64, hw, hw, c, w.data_ptr(), b.data_ptr(), lw.data_ptr(), lb.data_ptr(),
                        y.data_ptr(), stream, 2048, 7)
                assert lib.lab_dw(*args) == 0, v
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    lib.lab_dw(*args)
                e1.record()
                torch.cuda.synchronize()
                ts[v].append(e0.elapsed_time(e1) / 10 * 1e3)
        med = {v: sorted(t)[1] for v, t in ts.items()}
        print(f"C={c} H=W={hw} batch 64 ({gb * 1e3:.0f} MB algorithmic; v60 bitwise the library: {same}): " +
              "  ".join(f"{names[v]} {med[v]:.1f}us/{gb / med[v] * 1e6 / 1e3:.2f}TB/s" for v in names), flush=True)
