"""Digest of the bf16 ping-pong tiles' outputs (halo 8, pp 5, persistent 9 incl. the dual 1x1 and a
224-row-free ragged M) on C3's layer shapes and of the C3 network's outputs -- A/B library builds
(tools/ab_build.py, loaded with PIPNET_AMD_LIB) must print the same digests to be bitwise equal.

    PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=tools/ab/libpipnet_X.so python tools/bf16_digest.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import torch  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from count_pipnet_amd import kernels as K  # noqa: E402

# (name, batch, H, Cin, Cout, k, stride, pad, epilogue, tile)
LAYERS = [
    ("l3.c2", 64, 28, 256, 256, 3, 1, 1, _lib.EPI_BIAS_RELU, 8),
    ("l4.c2r", 7, 28, 512, 512, 3, 1, 1, _lib.EPI_BIAS_RESID_RELU, 8),        # ragged M, residual
    ("l3.c3", 64, 28, 256, 1024, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 9),
    ("l4.c1", 64, 28, 1024, 512, 1, 1, 0, _lib.EPI_BIAS_RELU, 9),
    ("l2.c3s", 3, 28, 128, 512, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU, 9),        # short K (4 K-tiles), ragged
    ("l2.ds", 64, 56, 256, 512, 1, 2, 0, _lib.EPI_BIAS, 5),
    ("l3.c1p", 64, 28, 512, 256, 1, 1, 0, _lib.EPI_BIAS, 5),
    ("kshort", 5, 28, 64, 256, 1, 1, 0, _lib.EPI_NONE, 5),                  # K = 64: 2 K-tiles
]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, b, h, cin, cout, k, s, pad, epi, tile in LAYERS:
        x = (torch.rand(b, h, h, cin, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = K.pack_conv_weight_bf16(torch.randn(cout, k, k, cin, device=dev, generator=g) * 0.05)
        bias = torch.randn(cout, device=dev, generator=g)
        oh = (h + 2 * pad - k) // s + 1
        r = ((torch.rand(b, oh, oh, cout, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
             if epi == _lib.EPI_BIAS_RESID_RELU else None)
        y = K.conv2d_nhwc_bf16(x, w, k, k, bias if epi != _lib.EPI_NONE else None, s, pad, epi, r, tile=tile)
        res[name] = hashlib.sha256(y.cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16]
    x = (torch.rand(64, 28, 28, 512, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    w = K.pack_conv_weight_bf16(torch.randn(1536, 1, 1, 512, device=dev, generator=g) * 0.05)
    bias = torch.randn(1536, device=dev, generator=g)
    y1, y2 = K.conv1x1_bf16_dual(x, w, bias, 1024, 512)
    res["dual"] = hashlib.sha256(y1.cpu().view(torch.int16).numpy().tobytes()
                                 + y2.cpu().view(torch.int16).numpy().tobytes()).hexdigest()[:16]
    # the C3 network (bf16 ResNet-50 PIP-Net, 128 images, default two streams)
    import bench_configs as bc
    from count_pipnet_amd.synthetic import synth_images
    net = bc.make(bc.CONFIGS["c3"], dev)
    xs = synth_images(128, 224, seed=300).to(dev)
    with torch.no_grad():
        proto, pooled, out = net(xs, inference=True)
    hsh = hashlib.sha256()
    for t in (proto, pooled, out):
        hsh.update(t.contiguous().cpu().numpy().tobytes())
    res["c3_net"] = hsh.hexdigest()[:16]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
