"""bf16 ResNet build (BASELINE C3 "ResNet50 ... bf16 inference") through the C-ABI.

Kernel level: against the same arithmetic restated in torch -- bf16-valued operands, fp32
conv (fp64 here), fp32 bias / residual / ReLU, one rounding to bf16.  The only freedom
left is the fp32 accumulation order, so an output may differ from the restatement by one
bf16 rounding step where the fp32 value sits next to a rounding boundary: tolerance 1
bf16 ulp (<= 2^-7 relative) + 1e-6, and >= 99 % of the elements bit-identical.

End to end (golden C3 input): such one-ulp flips re-randomise the rounding of every later
layer, so two bf16 evaluations that differ only in accumulation order drift apart by the
same amount as bf16 drifts from fp32 (measured: pooled 0.028 both ways).  The end-to-end
bar is therefore the bf16 tolerance against the reference's fp32 golden, the same one the
oracle's own restatement of the build meets (tests/test_oracle_golden.py::
test_bf16_build_tolerance_vs_reference): pooled 5e-2 abs, logits 5e-2 of scale, decisive
argmax equal -- applied to both the fp32 golden and the bf16 restatement.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from count_pipnet_amd import _lib
from count_pipnet_amd import kernels as K

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).double()


def _close_bf16(out, ref):
    out, ref = out.double(), ref.double()
    err = (out - ref).abs()
    assert torch.all(err <= ref.abs() * 2.0 ** -7 + 1e-6), err.max()
    assert (err == 0).double().mean() >= 0.99, (err == 0).double().mean()


@pytest.mark.parametrize("cin,cout,h,k,s,pad,epi", [
    (64, 64, 14, 1, 1, 0, _lib.EPI_BIAS_RELU),          # 1x1 dense
    (256, 128, 13, 1, 2, 0, _lib.EPI_BIAS),             # 1x1 stride 2 (downsample)
    (64, 64, 15, 3, 1, 1, _lib.EPI_BIAS_RELU),          # 3x3
    (128, 128, 16, 3, 2, 1, _lib.EPI_BIAS_RELU),        # 3x3 stride 2
    (64, 256, 9, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU),    # bottleneck conv3 + identity
    (8, 64, 30, 7, 2, 3, _lib.EPI_BIAS_RELU),           # stem 7x7 (K 392 -> 448 padded)
    (24, 72, 11, 3, 1, 1, _lib.EPI_NONE),               # K = 216 (not a 64 multiple), N = 72
    (512, 2048, 7, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU),  # layer4 conv3
])
def test_conv2d_nhwc_bf16(gpu, cin, cout, h, k, s, pad, epi):
    g = torch.Generator().manual_seed(cin * 3 + cout + h * 5 + k)
    x = _bf(torch.randn(3, cin, h, h, generator=g).abs() if epi else torch.randn(3, cin, h, h, generator=g))
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    wb = _bf(w)
    b = torch.randn(cout, generator=g).double()
    y = F.conv2d(x, wb, b if epi != _lib.EPI_NONE else None, stride=s, padding=pad)
    r = _bf(torch.randn(*y.shape, generator=g))
    if epi == _lib.EPI_BIAS_RELU:
        y = torch.relu(y)
    if epi == _lib.EPI_BIAS_RESID_RELU:
        y = torch.relu(y + r)
    ref = _bf(y.float()).permute(0, 2, 3, 1)
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu)  # noqa: E731
    wp = K.pack_conv_weight_bf16(w.permute(0, 2, 3, 1).contiguous().to(gpu))
    out = K.conv2d_nhwc_bf16(nhwc(x), wp, k, k, b.float().to(gpu) if epi != _lib.EPI_NONE else None, s, pad, epi,
                             nhwc(r) if epi == _lib.EPI_BIAS_RESID_RELU else None)
    torch.cuda.synchronize()
    assert out.dtype == torch.bfloat16 and tuple(out.shape) == tuple(ref.shape)
    _close_bf16(out.cpu(), ref)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 8])
@pytest.mark.parametrize("cin,cout,h,k,s,pad,epi", [
    (64, 256, 19, 3, 1, 1, _lib.EPI_BIAS_RESID_RELU),   # M = 1083: ragged in every tile size
    (256, 520, 10, 1, 2, 0, _lib.EPI_BIAS),             # N = 520: ragged N tile, strided 1x1
    (96, 264, 21, 1, 1, 0, _lib.EPI_BIAS_RELU),         # dense 1x1, K = 96 -> 128 padded (K tail of zeros)
    (512, 512, 12, 3, 1, 1, _lib.EPI_BIAS_RELU),        # layer4 3x3: 144 K-tiles, padding taps
    (8, 64, 37, 7, 2, 3, _lib.EPI_BIAS_RELU),           # stem 7x7 s2, K 392 -> 448 (taps straddle K tiles)
    (64, 40, 17, 3, 1, 1, _lib.EPI_BIAS),               # N = 40 < 64: ragged N in the 256x64 tile
])
def test_conv2d_nhwc_bf16_every_tile(gpu, tile, cin, cout, h, k, s, pad, epi):
    """Each workgroup tile (64x128, 128x128, 256x256, ping-pong 256x256, 256x64) forced on ragged shapes."""
    if tile == 5 and not ((k == 1 and s == 1 and pad == 0) or cin % 32 == 0):
        pytest.skip("the ping-pong tile needs whole-tap K tiles (Cin % 32 == 0)")
    if tile == 8 and not (k == 3 and s == 1 and pad == 1 and cin % 64 == 0 and h <= 31 and cout >= 256):
        pytest.skip("the halo tile serves 3x3 stride-1 pad-1 convs with Cin % 64 == 0, W <= 31, N >= 256")
    g = torch.Generator().manual_seed(tile * 11 + cout)
    x = _bf(torch.randn(3, cin, h, h, generator=g))
    w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g).double()
    y = F.conv2d(x, _bf(w), b, stride=s, padding=pad)
    r = _bf(torch.randn(*y.shape, generator=g))
    if epi == _lib.EPI_BIAS_RELU:
        y = torch.relu(y)
    if epi == _lib.EPI_BIAS_RESID_RELU:
        y = torch.relu(y + r)
    ref = _bf(y.float()).permute(0, 2, 3, 1)
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu)  # noqa: E731
    out = K.conv2d_nhwc_bf16(nhwc(x), K.pack_conv_weight_bf16(w.permute(0, 2, 3, 1).contiguous().to(gpu)), k, k,
                             b.float().to(gpu), s, pad, epi, nhwc(r) if epi == _lib.EPI_BIAS_RESID_RELU else None,
                             tile=tile)
    _close_bf16(out.cpu(), ref)


@pytest.mark.parametrize("b,cin,cout,h,w,epi", [
    (3, 64, 256, 7, 9, _lib.EPI_BIAS_RESID_RELU),   # non-square, several images per 256-pixel tile
    (2, 128, 264, 5, 1, _lib.EPI_BIAS_RELU),        # W = 1 (every kx != 1 tap is padding), ragged N
    (1, 64, 256, 31, 31, _lib.EPI_BIAS),            # widest halo (256 + 2*31 + 2 = 320 rows)
    (5, 256, 256, 28, 28, _lib.EPI_BIAS_RELU),      # layer3 conv2 at 28^2 (C3), ragged last tile
    (2, 512, 512, 28, 13, _lib.EPI_NONE),           # layer4 conv2 channels: 16 chunks x 9 taps
])
def test_conv_bf16_halo(gpu, b, cin, cout, h, w, epi):
    """3x3 stride-1 convolutions on the LDS-halo ping-pong tile (automatic choice, tile 8):
    K walked chunk-major / tap-minor, taps across row and image boundaries of the linear
    pixel index read the zero block.  Same one-ulp bar as every other tile, and the
    automatic choice must be the halo kernel."""
    g = torch.Generator().manual_seed(b * 7 + cin + cout + h * 3 + w)
    x = _bf(torch.randn(b, cin, h, w, generator=g))
    wt = torch.randn(cout, cin, 3, 3, generator=g) / (cin * 9) ** 0.5
    bias = torch.randn(cout, generator=g).double()
    y = F.conv2d(x, _bf(wt), bias if epi != _lib.EPI_NONE else None, stride=1, padding=1)
    r = _bf(torch.randn(*y.shape, generator=g))
    if epi == _lib.EPI_BIAS_RELU:
        y = torch.relu(y)
    if epi == _lib.EPI_BIAS_RESID_RELU:
        y = torch.relu(y + r)
    ref = _bf(y.float()).permute(0, 2, 3, 1)
    nhwc = lambda t: t.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(gpu)  # noqa: E731
    wp = K.pack_conv_weight_bf16(wt.permute(0, 2, 3, 1).contiguous().to(gpu))
    assert K.bf16_conv_plan(b, h, w, cin, cout, 3, 3, 1, 1, epi) == 8
    outs = [K.conv2d_nhwc_bf16(nhwc(x), wp, 3, 3, bias.float().to(gpu) if epi != _lib.EPI_NONE else None, 1, 1, epi,
                               nhwc(r) if epi == _lib.EPI_BIAS_RESID_RELU else None, tile=t) for t in (-1, 8)]
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    _close_bf16(outs[0].cpu(), ref)


@pytest.mark.parametrize("m,cin,cout,epi", [
    (1083, 64, 256, _lib.EPI_BIAS_RESID_RELU),      # ragged M, 2 K-tiles (short-K path), one tile per WG
    (1083, 96, 512, _lib.EPI_BIAS_RELU),            # K 96 -> 128 padded (re-read last A columns vs zero W)
    (70000, 512, 512, _lib.EPI_BIAS_RESID_RELU),    # 548 tiles: several tiles per persistent workgroup
    (70000, 256, 1024, _lib.EPI_BIAS),              # 1096 tiles, 8 K-tiles
    (9000, 1024, 256, _lib.EPI_NONE),               # long K
    (12544, 256, 1024, _lib.EPI_BIAS_RESID_RELU),   # layer3 conv3 + identity (16 images)
    (3337, 512, 2048, _lib.EPI_BIAS_RESID_RELU),    # layer4 conv3 + identity, ragged M
])
def test_conv_bf16_persistent_pp(gpu, m, cin, cout, epi):
    """Persistent ping-pong tile (tile 9, 1x1 convs with N % 256 == 0): same K order as the
    pp tile, so bitwise equal to it -- including the tile switches, where the next tile's
    first K-tiles are in flight during the previous epilogue -- and within one bf16 ulp of
    the restated arithmetic."""
    g = torch.Generator().manual_seed(m + cin + cout)
    x = torch.randn(m, 1, 1, cin, generator=g).to(torch.bfloat16).to(gpu)
    w = (torch.randn(cout, 1, 1, cin, generator=g) / cin ** 0.5).to(gpu)
    wp = K.pack_conv_weight_bf16(w)
    b = torch.randn(cout, generator=g).to(gpu)
    r = torch.randn(m, 1, 1, cout, generator=g).to(torch.bfloat16).to(gpu) if epi == _lib.EPI_BIAS_RESID_RELU else None
    bias = b if epi != _lib.EPI_NONE else None
    outs = [K.conv2d_nhwc_bf16(x, wp, 1, 1, bias, 1, 0, epi, r, tile=t) for t in (5, 9)]
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    if m <= 9000:
        y = x.double().view(m, cin) @ wp[:, :cin].double().t()
        if bias is not None:
            y = y + b.double()
        if r is not None:
            y = y + r.double().view(m, cout)
        if epi in (_lib.EPI_BIAS_RELU, _lib.EPI_BIAS_RESID_RELU):
            y = torch.relu(y)
        _close_bf16(outs[1].cpu().view(m, cout), _bf(y.float().cpu()))


def test_conv_bf16_halo_batch_invariant(gpu):
    """The halo kernel's per-pixel arithmetic does not depend on the batch a pixel is in."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(6, 28, 28, 256, generator=g).to(torch.bfloat16).to(gpu)
    wp = K.pack_conv_weight_bf16((torch.randn(256, 3, 3, 256, generator=g) / 48.0).to(gpu))
    bias = torch.randn(256, generator=g).to(gpu)
    full = K.conv2d_nhwc_bf16(x, wp, 3, 3, bias, 1, 1, _lib.EPI_BIAS_RELU)
    part = K.conv2d_nhwc_bf16(x[2:5].contiguous(), wp, 3, 3, bias, 1, 1, _lib.EPI_BIAS_RELU)
    torch.cuda.synchronize()
    assert torch.equal(full[2:5], part)


def test_conv_bf16_layout_asymmetric(gpu):
    """1x1 conv with identity input and an asymmetric exactly-representable weight: any
    transposed or mis-swizzled fragment shows up as a wrong element."""
    n = 128
    x = torch.eye(n).view(1, n, 1, n)                                # [1, H=n, W=1, C=n] NHWC: pixel i = e_i
    w = ((torch.arange(n * n) % 251) / 8.0).view(n, n)              # multiples of 1/8 < 32: exact in bf16
    out = K.conv2d_nhwc_bf16(x.contiguous().to(torch.bfloat16).to(gpu),
                             K.pack_conv_weight_bf16(w.view(n, 1, 1, n).to(gpu)), 1, 1, None, 1, 0, _lib.EPI_NONE)
    assert torch.equal(out.float().cpu().view(n, n), w.t().contiguous())


@pytest.mark.parametrize("n", [256, 320])
def test_conv_bf16_pp_layout_asymmetric(gpu, n):
    """The ping-pong tile (16x16x32 operand map, 64-B swizzled rows, per-wave epilogue
    re-layout) on an identity input: out[i] = column i of an asymmetric exact weight."""
    x = torch.eye(n).view(1, n, 1, n)
    w = ((torch.arange(n * n) % 253) / 8.0).view(n, n)
    out = K.conv2d_nhwc_bf16(x.contiguous().to(torch.bfloat16).to(gpu),
                             K.pack_conv_weight_bf16(w.view(n, 1, 1, n).to(gpu)), 1, 1, None, 1, 0, _lib.EPI_NONE,
                             tile=5)
    assert torch.equal(out.float().cpu().view(n, n), w.t().contiguous())


def test_maxpool_relayout_softmax_bf16(gpu):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 23, 23, generator=g).to(torch.bfloat16)
    out = K.maxpool2d_nhwc_bf16(x.permute(0, 2, 3, 1).contiguous().to(gpu), 3, 2, 1).cpu()
    assert torch.equal(out, F.max_pool2d(x.float(), 3, 2, 1).to(torch.bfloat16).permute(0, 2, 3, 1))
    xin = torch.randn(2, 3, 17, 19, generator=g)
    y = K.nchw_to_nhwc_bf16(xin.to(gpu), 8).cpu()
    assert torch.equal(y[..., :3], xin.to(torch.bfloat16).permute(0, 2, 3, 1)) and torch.all(y[..., 3:] == 0)
    for p in (2048, 200, 1000, 36):          # vectorised NV = 4 / 1 / 2, and the P % 8 != 0 fallback
        f = (torch.randn(2, 5, 7, p, generator=g) * 3).to(torch.bfloat16)
        ref = torch.softmax(f.double(), dim=-1)
        for mode in (0, 1):
            proto, pooled = K.softmax_pool_bf16(f.to(gpu), mode)
            assert torch.allclose(proto.double().cpu(), ref, atol=1e-6, rtol=1e-5)
            rp = ref.amax(dim=(1, 2)) if mode == 0 else ref.sum(dim=(1, 2))
            assert torch.allclose(pooled.double().cpu(), rp, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("h,w", [(224, 224), (37, 30), (17, 19)])
def test_stem_s2d_bf16(gpu, h, w):
    """The space-to-depth stem of the bf16 ResNet path: the relayout kernel bit-exact against
    its CPU restatement (tests/test_stem_s2d.py), and relayout + regrouped weights + the 4x4
    bf16 conv (+ bias + ReLU) against the fp64 7x7 stride-2 conv of the same bf16 values."""
    from test_stem_s2d import s2d_reference
    g = torch.Generator().manual_seed(h + 7 * w)
    x = torch.randn(2, 3, h, w, generator=g)
    s = K.nchw_to_s2d_bf16(x.to(gpu)).cpu()
    assert torch.equal(s, s2d_reference(x).to(torch.bfloat16))
    wt = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    b = torch.randn(64, generator=g)
    wp = K.pack_conv_weight_bf16(K.stem_weight_s2d(wt.permute(0, 2, 3, 1).contiguous()).to(gpu))
    out = K.conv2d_nhwc_bf16(K.nchw_to_s2d_bf16(x.to(gpu)), wp, 4, 4, b.to(gpu), 1, 0, _lib.EPI_BIAS_RELU)
    xb, wb = x.to(torch.bfloat16).double(), wt.to(torch.bfloat16).double()
    ref = torch.relu(F.conv2d(xb, wb, b.double(), stride=2, padding=3)).permute(0, 2, 3, 1)
    assert out.shape == ref.shape
    err = (out.double().cpu() - ref).abs()
    assert torch.all(err <= 1e-2 * (1 + ref.abs())), err.max()      # bf16 output rounding (2^-8)


@pytest.mark.parametrize("m,cin,n1,n2", [(2 * 28 * 28, 512, 1024, 256), (3 * 17 * 11, 1024, 2048, 512), (300, 256, 256, 256)])
def test_conv1x1_bf16_dual_matches_single(gpu, m, cin, n1, n2):
    """The dual 1x1 launch (a first Bottleneck's downsample + conv1 over one input read) gives
    each output bit for bit as its own persistent-tile conv."""
    g = torch.Generator().manual_seed(m + n1)
    x = torch.randn(1, m, 1, cin, generator=g).to(torch.bfloat16).to(gpu)
    w1 = K.pack_conv_weight_bf16((torch.randn(n1, 1, 1, cin, generator=g) * 0.05).to(gpu))
    w2 = K.pack_conv_weight_bf16((torch.randn(n2, 1, 1, cin, generator=g) * 0.05).to(gpu))
    b1, b2 = torch.randn(n1, generator=g).to(gpu), torch.randn(n2, generator=g).to(gpu)
    y1, y2 = K.conv1x1_bf16_dual(x, torch.cat([w1, w2]), torch.cat([b1, b2]), n1, n2)
    r1 = K.conv2d_nhwc_bf16(x, w1, 1, 1, b1, 1, 0, _lib.EPI_BIAS)
    r2 = K.conv2d_nhwc_bf16(x, w2, 1, 1, b2, 1, 0, _lib.EPI_BIAS_RELU)
    assert torch.equal(y1, r1) and torch.equal(y2, r2)


@pytest.mark.parametrize("cin,b,h,w,epi", [
    (64, 2, 56, 56, _lib.EPI_BIAS_RELU), (64, 3, 17, 13, _lib.EPI_BIAS_RELU), (64, 1, 9, 63, _lib.EPI_BIAS),
    (64, 2, 11, 7, _lib.EPI_BIAS_RESID_RELU), (64, 1, 5, 5, _lib.EPI_NONE), (64, 5, 1, 1, _lib.EPI_BIAS_RELU),
    (128, 3, 28, 28, _lib.EPI_BIAS_RELU), (128, 2, 13, 31, _lib.EPI_BIAS_RESID_RELU), (128, 1, 7, 3, _lib.EPI_BIAS),
    (128, 4, 2, 1, _lib.EPI_NONE)])
def test_conv3x3_n64_halo(gpu, cin, b, h, w, epi):
    """Tile 11 (3x3 s1 p1, Cin = N = 64 / 128, LDS input halo) is bitwise equal to the generic
    tile of the layer (6 at N = 64; 4 and 0 at N = 128) -- same MFMA shape, same K order, same
    epilogue -- so choosing it changes no output bit; also against the fp64 conv of the same
    bf16 values (bf16 output rounding), image-boundary taps, ragged M (rows past the last tile),
    every epilogue; and batch invariance (image 1 alone == image 1 in the batch)."""
    cout = cin
    g = torch.Generator().manual_seed(cin + h * w + b)
    x = torch.randn(b, h, w, cin, generator=g).to(torch.bfloat16)
    wt = (torch.randn(cout, 3, 3, cin, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn(cout, generator=g)
    r = torch.randn(b, h, w, cout, generator=g).to(torch.bfloat16) if epi == _lib.EPI_BIAS_RESID_RELU else None
    wp = K.pack_conv_weight_bf16(wt.float().to(gpu))
    run = lambda xx, rr, t: K.conv2d_nhwc_bf16(xx.to(gpu), wp, 3, 3, bias.to(gpu), 1, 1, epi,  # noqa: E731
                                               None if rr is None else rr.to(gpu), tile=t)
    out11 = run(x, r, 11)
    for t in ((6,) if cin == 64 else (4, 0)):
        assert torch.equal(out11, run(x, r, t)), t
    out = out11.double().cpu()
    ref = F.conv2d(x.double().permute(0, 3, 1, 2), wt.double().permute(0, 3, 1, 2), padding=1)
    if epi != _lib.EPI_NONE:
        ref = ref + bias.double().view(1, -1, 1, 1)
    ref = ref.permute(0, 2, 3, 1)
    if r is not None:
        ref = ref + r.double()
    if epi in (_lib.EPI_BIAS_RELU, _lib.EPI_BIAS_RESID_RELU):
        ref = torch.relu(ref)
    err = (out - ref).abs()
    assert torch.all(err <= 1e-2 * (1 + ref.abs())), err.max()
    if b > 1:
        one = run(x[1:2], None if r is None else r[1:2], 11).cpu()
        assert torch.equal(one[0], out11[1].cpu())


def test_conv3x3_n64_halo_rejects(gpu):
    """Tile 11 forced on a layer outside its scope (Cin != N, Cin not 64 / 128, W over the halo)
    is an argument error."""
    for cin, cout, w in ((32, 64, 8), (64, 64, 64), (128, 128, 32), (64, 128, 8), (256, 256, 8)):
        x = torch.zeros(1, 4, w, cin, dtype=torch.bfloat16, device=gpu)
        wp = K.pack_conv_weight_bf16(torch.zeros(cout, 3, 3, cin, device=gpu))
        with pytest.raises(RuntimeError):
            K.conv2d_nhwc_bf16(x, wp, 3, 3, None, 1, 1, _lib.EPI_NONE, None, tile=11)


@pytest.mark.parametrize("b,h,w", [(3, 224, 224), (2, 37, 53), (1, 9, 9), (2, 224, 100), (1, 5, 224)])
def test_stem_pool_bf16_matches_unfused(gpu, b, h, w):
    """The fused stem + max-pool (pipnet_stem_pool_bf16) is bitwise the unfused pair: the 4x4
    s2d conv on its automatic tile (6) with bias + ReLU, then pipnet_maxpool2d_nhwc_bf16 --
    odd sizes put pooled rows past the image, partial last row pairs and 1-row maps in play."""
    g = torch.Generator().manual_seed(b * 1000 + h * 7 + w)
    x = torch.randn(b, 3, h, w, generator=g).to(gpu)
    w7 = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    wp = K.pack_conv_weight_bf16(K.stem_weight_s2d(w7.permute(0, 2, 3, 1).contiguous()).to(gpu))
    bias = (torch.randn(64, generator=g) * 0.1).to(gpu)
    s2d = K.nchw_to_s2d_bf16(x)
    fused = K.stem_pool_bf16(s2d, wp, bias)
    ref = K.maxpool2d_nhwc_bf16(K.conv2d_nhwc_bf16(s2d, wp, 4, 4, bias, 1, 0, _lib.EPI_BIAS_RELU), 3, 2, 1)
    torch.cuda.synchronize()
    assert fused.shape == ref.shape
    assert torch.equal(fused, ref)


def _c3_bf16(gpu, num_features=0):
    from golden_util import golden_args, golden_inputs, golden_state_dict, load_golden
    from model_util import build_model
    from count_pipnet_amd.pipnet import set_hip_dtype
    meta, rec = load_golden("c3_pipnet_resnet50")
    net = set_hip_dtype(build_model(meta), torch.bfloat16).to(gpu)
    return meta, rec, net, golden_inputs(meta), golden_state_dict(meta), golden_args(meta)


# bf16 error budget of the C3 build against the reference's fp32 arithmetic, measured on the
# golden model (scratch study: oracle bf16 restatement vs oracle fp32 on 16 images of 224x224):
# pooled |d| <= 0.039, presence flips only within 0.008 of the 0.1 threshold, logits |d| <= 0.156
# of a 6.2 scale -- but almost all of that is common to every class of an image (the classifier
# rows are N(1, 0.1), main.py:168, so a pooled error moves every logit alike) -- while the error
# of the logit *differences* that decide the argmax (d_c - d_top) is <= 0.045, against class
# margins (top-2 gaps) of 0.07-0.13.  The bounds below sit at about 2x those measurements.
BF16_POOLED_TOL = 0.06          # present in both: |pooled - pooled_fp32|
BF16_PRESENCE_BAND = 1e-2       # presence flags must agree where |pooled_fp32 - 0.1| > band
BF16_MARGIN_TOL = 0.08          # max_c |(out_c - out_top) - (ref_c - ref_top)|, < the median class margin
BF16_LOGIT_TOL = 0.05           # |out - ref| <= tol * max|ref| (common mode included)


def _check_bf16_vs_fp32(pooled, out, r_raw, r_out, min_decisive):
    """HIP bf16 inference outputs against the reference's fp32 arithmetic (oracle, pinned to
    the reference goldens): presence flags, pooled values, logits, class-margin error, argmax
    on every image whose fp32 top-2 gap exceeds the margin bound.  Returns the measured
    errors so the test log shows the budget actually used."""
    pooled, out, r_raw, r_out = (t.double() for t in (pooled, out, r_raw, r_out))
    r_inf = torch.where(r_raw < 0.1, torch.zeros_like(r_raw), r_raw)
    band = (r_raw - 0.1).abs() <= BF16_PRESENCE_BAND
    flags_ok = ((pooled > 0) == (r_raw >= 0.1)) | band
    assert flags_ok.all(), ("presence flag flipped outside the band", r_raw[~flags_ok], pooled[~flags_ok])
    both = (pooled > 0) & (r_inf > 0)
    perr = (pooled - r_inf).abs()[both].max().item() if both.any() else 0.0
    assert perr <= BF16_POOLED_TOL, perr
    d = out - r_out
    scale = r_out.abs().max().clamp(min=1.0)
    assert d.abs().max() <= BF16_LOGIT_TOL * scale, (d.abs().max(), scale)
    top = r_out.argmax(1)
    merr = (d - d.gather(1, top[:, None])).abs().max(1).values
    assert merr.max() <= BF16_MARGIN_TOL, merr
    srt = r_out.sort(dim=1).values
    gap = srt[:, -1] - srt[:, -2]
    decisive = gap > BF16_MARGIN_TOL
    assert int(decisive.sum()) >= min_decisive, (gap, decisive.sum())
    assert torch.equal(out.argmax(1)[decisive], top[decisive]), (out.argmax(1), top, gap)
    return {"pooled_err": perr, "logit_err": d.abs().max().item(), "margin_err": merr.max().item(),
            "decisive": int(decisive.sum()), "present": int((r_inf > 0).sum()), "band": int(band.sum())}


def test_c3_bf16_matches_bf16_oracle_and_reference(gpu):
    """The golden's 2 images: vs the bf16 restatement of the build's arithmetic and vs the
    reference's recorded fp32 outputs under the bf16 budget (argmax compared on both images:
    their fp32 class margins 0.10 / 0.14 exceed BF16_MARGIN_TOL)."""
    from oracle import ref_cpu
    meta, rec, net, xs, sd, args = _c3_bf16(gpu)
    torch.set_num_threads(8)
    with torch.no_grad():
        proto, pooled, out = net(xs.to(gpu), inference=True)
        r_proto, r_pooled, r_out = ref_cpu.pipnet_forward_bf16(xs, sd, args, inference=True)
    proto, pooled, out = proto.float().cpu(), pooled.cpu(), out.cpu()
    assert proto.dtype == torch.float32 and tuple(proto.shape) == tuple(r_proto.shape)
    # vs the build's arithmetic restated on the CPU
    near = (r_pooled - 0.1).abs() < 5e-2
    assert torch.all((pooled - r_pooled).abs()[~near] <= 5e-2), (pooled - r_pooled).abs().max()
    scale = r_out.abs().max().clamp(min=1.0)
    assert (out - r_out).abs().max() <= 5e-2 * scale
    assert (proto.amax(dim=(2, 3)) - r_proto.amax(dim=(2, 3))).abs().max() <= 5e-2
    # vs the reference's fp32 outputs (golden)
    got = _check_bf16_vs_fp32(pooled, out, torch.from_numpy(rec["raw_pooled"]), torch.from_numpy(rec["inf_out"]),
                              min_decisive=2)
    print("C3 golden bf16 budget:", got)


def _fp32_oracle_head(xs, sd, args):
    from oracle import ref_cpu
    with torch.no_grad():
        feats = ref_cpu.backbone(xs, sd, args)
        r_raw = torch.softmax(feats, dim=1).amax(dim=(2, 3))
        r_out = ref_cpu.non_neg_linear(torch.where(r_raw < 0.1, torch.zeros_like(r_raw), r_raw),
                                       sd["_classification.weight"], sd.get("_classification.bias"))
    return r_raw, r_out


def test_c3_bf16_16_images_vs_fp32_oracle(gpu):
    """16 committed-seed images of 224x224 through the HIP bf16 build and the fp32 oracle:
    presence flags, pooled, logits, class-margin error and argmax under the bf16 budget;
    at least 8 images must be decisive (the comparison is never empty)."""
    from count_pipnet_amd.synthetic import synth_images
    meta, rec, net, _, sd, args = _c3_bf16(gpu)
    torch.set_num_threads(8)
    xs = synth_images(16, 224, seed=11)
    with torch.no_grad():
        _, pooled, out = net(xs.to(gpu), inference=True)
    r_raw, r_out = _fp32_oracle_head(xs, sd, args)
    got = _check_bf16_vs_fp32(pooled.cpu(), out.cpu(), r_raw, r_out, min_decisive=8)
    print("C3 16-image bf16 budget:", got)


def test_c3_bf16_full_batch_properties(gpu):
    """BASELINE C3 size (bs=128, 224x224), raw and inference mode: shapes, softmax
    normalisation, pooled = max of proto (and its 0.1 clamp), logits = NonNegLinear(pooled),
    per-image determinism (image 0 alone == image 0 in the batch), and 4 images spread over
    the batch against the fp32 oracle under the bf16 budget."""
    from count_pipnet_amd.synthetic import synth_images
    meta, rec, net, _, sd, args = _c3_bf16(gpu)
    xs = synth_images(128, 224, seed=11).to(gpu)
    with torch.no_grad():
        proto, pooled, out = net(xs, inference=False)
        p1, pl1, o1 = net(xs[:1], inference=False)
        _, ipooled, iout = net(xs, inference=True)
    assert tuple(proto.shape) == (128, 2048, 28, 28) and tuple(out.shape) == (128, 200)
    s = proto.sum(dim=1)
    assert torch.allclose(s, torch.ones_like(s), atol=1e-4)
    assert torch.equal(pooled, proto.amax(dim=(2, 3)))
    assert torch.equal(pl1[0], pooled[0]) and torch.equal(o1[0], out[0])
    assert torch.isfinite(out).all()
    assert torch.equal(ipooled, torch.where(pooled < 0.1, torch.zeros_like(pooled), pooled))
    w = net._classification.weight
    assert torch.allclose(iout, ipooled @ torch.relu(w).t(), rtol=1e-5, atol=1e-4)
    pick = [0, 37, 64, 127]
    torch.set_num_threads(8)
    r_raw, r_out = _fp32_oracle_head(xs[pick].cpu(), sd, args)
    got = _check_bf16_vs_fp32(ipooled[pick].cpu(), iout[pick].cpu(), r_raw, r_out, min_decisive=1)
    print("C3 bs=128 sample bf16 budget:", got)


@pytest.mark.parametrize("kind,m_or_b,cin,cout,epi", [
    ("1x1", 2352, 256, 256, _lib.EPI_BIAS_RELU),            # 3 images of 28x28: ragged for 224 and 256
    ("1x1", 50176, 1024, 256, _lib.EPI_BIAS_RELU),          # C3 l3.c1 at 64 images (224 / 196 row tiles)
    ("1x1", 5000, 256, 1024, _lib.EPI_BIAS_RESID_RELU),     # conv3 + identity, ragged
    ("1x1", 777, 512, 512, _lib.EPI_BIAS),
    ("1x1", 300, 128, 256, _lib.EPI_NONE),                  # a single, partial 224-row tile
    ("3x3", 3, 256, 256, _lib.EPI_BIAS_RELU),
    ("3x3", 5, 512, 512, _lib.EPI_BIAS_RESID_RELU),
    ("3x3", 2, 256, 512, _lib.EPI_BIAS),
    ("dual", 4704, 512, (1024, 256), None)])
def test_pp_tiles_ragged_vs_fp32(gpu, kind, m_or_b, cin, cout, epi):
    """The persistent 1x1 tile, the LDS-halo 3x3 tile and the dual 1x1 launch (256-row tiles) on
    ragged M, every epilogue and the halo image borders, against torch's fp32 conv of the same
    bf16 operands: within one bf16 rounding of the output (+ fp32 summation-order noise)."""
    gg = torch.Generator().manual_seed(7)
    if kind == "dual":
        n1, n2 = cout
        x = torch.randn(1, m_or_b, 1, cin, generator=gg).to(torch.bfloat16)
        w = (torch.randn(n1 + n2, 1, 1, cin, generator=gg) * 0.05)
        b = torch.randn(n1 + n2, generator=gg)
        wp = K.pack_conv_weight_bf16(w.to(gpu))
        y1, y2 = K.conv1x1_bf16_dual(x.to(gpu), wp, b.to(gpu), n1, n2)
        wq = wp[:, :cin].float().cpu().view(n1 + n2, cin)
        ref = x.float().view(-1, cin) @ wq.t() + b
        got = torch.cat([y1.float().view(-1, n1), y2.float().view(-1, n2)], 1).cpu()
        ref[:, n1:] = ref[:, n1:].clamp_min(0)
    else:
        if kind == "1x1":
            x = torch.randn(1, m_or_b, 1, cin, generator=gg).to(torch.bfloat16)
            w = torch.randn(cout, 1, 1, cin, generator=gg) / cin ** 0.5
            r = torch.randn(1, m_or_b, 1, cout, generator=gg).to(torch.bfloat16)
            kk, pad = 1, 0
        else:
            x = torch.randn(m_or_b, 28, 28, cin, generator=gg).to(torch.bfloat16)
            w = torch.randn(cout, 3, 3, cin, generator=gg) / (3 * cin ** 0.5)
            r = torch.randn(m_or_b, 28, 28, cout, generator=gg).to(torch.bfloat16)
            kk, pad = 3, 1
        b = torch.randn(cout, generator=gg)
        wp = K.pack_conv_weight_bf16(w.to(gpu))
        out = K.conv2d_nhwc_bf16(x.to(gpu), wp, kk, kk, None if epi == _lib.EPI_NONE else b.to(gpu), 1, pad, epi,
                                 r.to(gpu) if epi == _lib.EPI_BIAS_RESID_RELU else None)
        wq = wp[:, :kk * kk * cin].float().cpu().view(cout, kk, kk, cin).permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wq, None, 1, pad).permute(0, 2, 3, 1)
        if epi != _lib.EPI_NONE:
            ref = ref + b
        if epi == _lib.EPI_BIAS_RESID_RELU:
            ref = ref + r.float()
        if epi in (_lib.EPI_BIAS_RELU, _lib.EPI_BIAS_RESID_RELU):
            ref = ref.clamp_min(0)
        got = out.float().cpu()
    err = (got - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-3 * max(1.0, ref.abs().max().item())).all(), err.max().item()


@pytest.mark.parametrize("b,hw,p", [(3, 784, 2048), (2, 49, 512), (1, 37, 1000), (2, 10, 8)])
def test_head_bf16_quad_layout(gpu, b, hw, p):
    """The bf16 head (4 channels per lane, whole-line proto stores; P % 8 != 0 falls back to the
    lane-strided kernel) against an fp32 torch softmax + max-pool of the same bf16 logits."""
    x = (torch.randn(b, 1, hw, p, generator=torch.Generator().manual_seed(3)) * 3).to(torch.bfloat16).to(gpu)
    proto, pooled = K.softmax_pool_bf16(x, pool_mode=0)
    torch.cuda.synchronize()
    ref = torch.softmax(x.float().view(b, hw, p), dim=-1)
    torch.testing.assert_close(proto.view(b, hw, p), ref, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(pooled, ref.amax(dim=1), rtol=1e-5, atol=1e-7)
