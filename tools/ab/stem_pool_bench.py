"""Time the bf16 stem: fused conv + max-pool (pipnet_stem_pool_bf16) vs conv (tile 6) + pool."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


dev = torch.device("cuda:0")
for b in (64, 128):
    x = torch.randn(b, 3, 224, 224, device=dev)
    wp = K.pack_conv_weight_bf16(K.stem_weight_s2d(torch.randn(64, 7, 7, 3) * 0.1).to(dev))
    bias = torch.randn(64, device=dev) * 0.1
    s2d = K.nchw_to_s2d_bf16(x)
    conv = lambda: K.conv2d_nhwc_bf16(s2d, wp, 4, 4, bias, 1, 0, _lib.EPI_BIAS_RELU)  # noqa: E731
    h = conv()
    t_conv = timeit(conv)
    t_pool = timeit(lambda: K.maxpool2d_nhwc_bf16(h, 3, 2, 1))
    t_fused = timeit(lambda: K.stem_pool_bf16(s2d, wp, bias))
    print(f"images {b}: conv {t_conv:.1f} us + pool {t_pool:.1f} us = {t_conv + t_pool:.1f} us; fused {t_fused:.1f} us",
          flush=True)
