"""A/B the dwconv7+LN variants of tools/dw_lab.hip on the network's stage shapes."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libdw_lab.so"))
P, I32 = ctypes.c_void_p, ctypes.c_int
lib.lab_dw.argtypes = [I32, P, I32, I32, I32, I32, P, P, P, P, P, P]

dev = torch.device("cuda:0")
stream = torch.cuda.current_stream().cuda_stream
for c, hw in [(96, 56), (192, 28), (384, 27), (768, 26)]:
    x = torch.randn(64, hw, hw, c, device=dev)
    w = torch.randn(49, c, device=dev) * 0.2
    b, lw, lb = torch.randn(c, device=dev), torch.randn(c, device=dev), torch.randn(c, device=dev)
    y = torch.empty_like(x)
    ref = None
    res = {}
    for rnd in range(3):
        for v in range(5):
            args = (v, x.data_ptr(), 64, hw, hw, c, w.data_ptr(), b.data_ptr(), lw.data_ptr(), lb.data_ptr(),
                    y.data_ptr(), stream)
            assert lib.lab_dw(*args) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                lib.lab_dw(*args)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(v, []).append(e0.elapsed_time(e1) / 10 * 1e3)
            if rnd == 0:
                if ref is None:
                    ref = y.clone()
                else:
                    assert (y - ref).abs().max().item() < 1e-3, (c, v)
    gb = 2 * x.numel() * 4 / 1e9
    print(f"C={c:4d} " + " ".join(f"v{v}:{min(t):7.1f}us({gb / min(t) * 1e6 / 1e3:4.2f}TB/s)" for v, t in res.items()),
          flush=True)
