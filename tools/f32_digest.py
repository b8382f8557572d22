"""Digest of the fp32 GEMM's outputs on C2's CNBlock / downsample shapes (ragged M included) and of
the C2 network's outputs -- A/B library builds (tools/ab_build.py, loaded with PIPNET_AMD_LIB) print
the same digests when they are bitwise equal.

    PIPNET_AMD_ALLOW_STALE=1 PIPNET_AMD_LIB=tools/ab/libpipnet_X.so python tools/f32_digest.py
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


def h(t):
    return hashlib.sha256(t.contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, m, n, k, epi in [("s384_fc2", 46656, 384, 1536, _lib.EPI_RESID), ("s384_fc2r", 46656 - 77, 384, 1536,
                                _lib.EPI_RESID), ("s384_bias", 40001, 384, 768, _lib.EPI_BIAS),
                               ("s384_none", 38400, 384, 1536, _lib.EPI_NONE), ("s768_fc2", 43264, 768, 3072,
                                                                                _lib.EPI_RESID)]:
        a = torch.randn(m, k, device=dev, generator=g)
        w = torch.randn(n, k, device=dev, generator=g) * 0.05
        b = torch.randn(n, device=dev, generator=g)
        s = torch.randn(n, device=dev, generator=g)
        r = torch.randn(m, n, device=dev, generator=g)
        if epi == _lib.EPI_RESID:
            K.linear(a, w, b, epi, scale=s, r=r, out=r)
            y = r
        else:
            y = K.linear(a, w, b, epi, scale=s)
        res[name] = (K.gemm_variant(m, n, k), h(y))
    x = torch.randn(64, 27, 27, 192, device=dev, generator=g)
    wk = torch.randn(384, 2, 2, 192, device=dev, generator=g) * 0.05
    b = torch.randn(384, device=dev, generator=g)
    res["ds_2x2"] = (K.gemm_variant(64 * 26 * 26, 384, 768), h(K.conv2x2(x, wk, b, 1)))
    import bench_configs as bc
    from count_pipnet_amd.synthetic import synth_images
    net = bc.make(bc.CONFIGS["c2"], dev)
    xs = synth_images(64, 224, seed=300).to(dev)
    with torch.no_grad():
        out = net(xs, inference=True)
    hs = hashlib.sha256()
    for t in out:
        hs.update(t.contiguous().cpu().numpy().tobytes())
    res["c2_net"] = hs.hexdigest()[:16]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
