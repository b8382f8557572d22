import os
import sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from count_pipnet_amd import kernels as K
dev = torch.device('cuda:0')
for (b, h) in [(64, 224), (16, 64), (64, 128)]:
    x = torch.randn(b, 3, h, h, device=dev)
    w = torch.randn(96, 3, 4, 4, device=dev); bb = torch.randn(96, device=dev)
    lw = torch.randn(96, device=dev); lb = torch.randn(96, device=dev)
    for _ in range(3): K.convnext_stem(x, w, bb, lw, lb)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): K.convnext_stem(x, w, bb, lw, lb)
    e1.record(); torch.cuda.synchronize()
    print(b, h, 'stem us', e0.elapsed_time(e1) / 20 * 1e3, flush=True)
