"""Per-kernel numerics through the C-ABI against plain PyTorch fp32/fp64 references
(asymmetric, non-tile-multiple shapes; every epilogue; every supported channel count)."""
import pytest
import torch
import torch.nn.functional as F

from count_pipnet_amd import _lib
from count_pipnet_amd import kernels as K

pytestmark = pytest.mark.gpu


def _rand(*shape, gen, scale=1.0):
    return (torch.randn(*shape, generator=gen, dtype=torch.float64) * scale)


def _gemm_tol(a, w):
    # fp32 fma-chain error bound ~ K * eps * sum|a||w|  (loose constant)
    return 2e-6 * (a.abs() @ w.abs().t()) + 1e-6


@pytest.mark.parametrize("m,n,k", [(1, 1, 4), (37, 53, 48), (128, 128, 32), (300, 200, 96), (1000, 384, 1536),
                                   (64, 6144, 2048), (2, 9, 16), (129, 257, 772),
                                   # NPAD tiles (N % 128 != 0, K % 32 == 0): padded 32-column
                                   # MFMA blocks skipped, wave -> column half flipped per workgroup
                                   (500, 96, 384), (257, 160, 64), (64, 32, 256), (1000, 100, 512), (3, 4, 32)])
def test_linear_plain(gpu, m, n, k):
    g = torch.Generator().manual_seed(m * 7 + n * 13 + k)
    a, w = _rand(m, k, gen=g), _rand(n, k, gen=g)
    ref = a @ w.t()
    out = K.linear(a.float().to(gpu), w.float().to(gpu)).double().cpu()
    assert torch.all((out - ref).abs() <= _gemm_tol(a, w)), (out - ref).abs().max()


def test_mfma_layout_asymmetric(gpu):
    """A = I with an asymmetric W catches a transposed C-write (cdna guide section 3)."""
    n = 128
    a = torch.eye(n)
    w = torch.arange(n * n, dtype=torch.float32).view(n, n) / 1000.0
    out = K.linear(a.to(gpu), w.to(gpu)).cpu()
    assert torch.equal(out, w.t().contiguous())


@pytest.mark.parametrize("epi", [_lib.EPI_BIAS, _lib.EPI_BIAS_GELU, _lib.EPI_RESID, _lib.EPI_MUL])
def test_linear_epilogues(gpu, epi):
    g = torch.Generator().manual_seed(epi)
    m, n, k = 333, 192, 384
    a, w, b = _rand(m, k, gen=g), _rand(n, k, gen=g, scale=0.05), _rand(n, gen=g)
    s, r = _rand(n, gen=g), _rand(m, n, gen=g)
    acc = a @ w.t()
    if epi == _lib.EPI_BIAS:
        ref = acc + b
    elif epi == _lib.EPI_BIAS_GELU:
        ref = F.gelu(acc + b)
    elif epi == _lib.EPI_RESID:
        ref = r + s * (acc + b)
    else:
        ref = acc * r
    d = lambda t: t.float().to(gpu)  # noqa: E731
    out = K.linear(d(a), d(w), d(b), epi, scale=d(s), r=d(r)).double().cpu()
    tol = 4e-6 * (1 + ref.abs()) + 4e-6 * ((a.abs() @ w.abs().t()) * (1 + s.abs() + r.abs()))
    assert torch.all((out - ref).abs() <= tol), (out - ref).abs().max()


def test_linear_inplace_residual(gpu):
    g = torch.Generator().manual_seed(5)
    m, c = 700, 96
    a, w, b, s = _rand(m, 4 * c, gen=g), _rand(c, 4 * c, gen=g, scale=0.05), _rand(c, gen=g), _rand(c, gen=g)
    x = _rand(m, c, gen=g)
    ref = x + s * (a @ w.t() + b)
    xd = x.float().to(gpu)
    K.linear(a.float().to(gpu), w.float().to(gpu), b.float().to(gpu), _lib.EPI_RESID, scale=s.float().to(gpu),
             r=xd, out=xd)
    assert torch.allclose(xd.double().cpu(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cin,cout,h,stride", [(96, 192, 56, 2), (192, 384, 28, 1), (384, 768, 27, 1),
                                               (192, 384, 28, 2), (96, 192, 9, 2)])
def test_conv2x2(gpu, cin, cout, h, stride):
    g = torch.Generator().manual_seed(cin + h)
    x, w, b = _rand(3, cin, h, h, gen=g), _rand(cout, cin, 2, 2, gen=g, scale=0.05), _rand(cout, gen=g)
    ref = F.conv2d(x, w, b, stride=stride).permute(0, 2, 3, 1)
    xn = x.permute(0, 2, 3, 1).contiguous().float().to(gpu)
    wp = w.permute(0, 2, 3, 1).contiguous().float().to(gpu)
    out = K.conv2x2(xn, wp, b.float().to(gpu), stride).double().cpu()
    assert torch.allclose(out, ref, rtol=2e-5, atol=2e-5), (out - ref).abs().max()


@pytest.mark.parametrize("bsz,h,wd", [(2, 224, 224), (2, 64, 64), (2, 128, 128), (3, 36, 20), (1, 4, 8), (5, 68, 132)])
def test_stem(gpu, bsz, h, wd):
    """MFMA stem: 32-pixel tiles, so pixel counts that are not a multiple of 32 (3*9*5, 1*1*2,
    5*17*33) exercise the ragged last tile; non-square images the (oy, ox) decomposition."""
    g = torch.Generator().manual_seed(h * 1000 + wd)
    x, w, b = _rand(bsz, 3, h, wd, gen=g), _rand(96, 3, 4, 4, gen=g, scale=0.2), _rand(96, gen=g)
    lw, lb = 1 + 0.1 * _rand(96, gen=g), 0.1 * _rand(96, gen=g)
    y = F.conv2d(x, w, b, stride=4).permute(0, 2, 3, 1)
    ref = F.layer_norm(y, (96,), lw, lb, 1e-6)
    d = lambda t: t.float().to(gpu)  # noqa: E731
    out = K.convnext_stem(d(x), d(w), d(b), d(lw), d(lb)).double().cpu()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-4), (out - ref).abs().max()


@pytest.mark.parametrize("c,h,ww", [(96, 56, 56), (192, 28, 28), (384, 27, 27), (768, 26, 26), (768, 13, 13),
                                    (384, 14, 14), (96, 16, 16), (192, 8, 8),
                                    # small-map tiles (W <= 32 / 16): exact, ragged and non-square maps
                                    (96, 32, 32), (96, 13, 29), (96, 33, 30), (192, 16, 16), (192, 11, 7),
                                    (192, 20, 15)])
def test_dwconv7_ln(gpu, c, h, ww):
    g = torch.Generator().manual_seed(c + h + 7 * ww)
    x, w, b = _rand(2, c, h, ww, gen=g), _rand(c, 1, 7, 7, gen=g, scale=0.2), _rand(c, gen=g)
    lw, lb = 1 + 0.1 * _rand(c, gen=g), 0.1 * _rand(c, gen=g)
    y = F.conv2d(x, w, b, padding=3, groups=c).permute(0, 2, 3, 1)
    ref = F.layer_norm(y, (c,), lw, lb, 1e-6)
    d = lambda t: t.float().to(gpu)  # noqa: E731
    xn = x.permute(0, 2, 3, 1).contiguous()
    out = K.dwconv7_ln(d(xn), d(w.reshape(c, 49).t().contiguous()), d(b), d(lw), d(lb)).double().cpu()
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-4), (out - ref).abs().max()


@pytest.mark.parametrize("c", [96, 192, 384, 768, 100])
def test_layernorm(gpu, c):
    g = torch.Generator().manual_seed(c)
    x, lw, lb = _rand(517, c, gen=g, scale=3.0), 1 + 0.1 * _rand(c, gen=g), 0.1 * _rand(c, gen=g)
    ref = F.layer_norm(x, (c,), lw, lb, 1e-6)
    d = lambda t: t.float().to(gpu)  # noqa: E731
    out = K.layernorm(d(x), d(lw), d(lb)).double().cpu()
    assert torch.allclose(out, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("p,hw,mode", [(768, 676, 0), (2048, 784, 0), (16, 64, 1), (200, 33, 0), (2048, 256, 1),
                                        (1000, 50, 1), (1500, 20, 0), (30, 49, 0)])   # P % 4 != 0: lane-strided kernel
def test_softmax_pool(gpu, p, hw, mode):
    g = torch.Generator().manual_seed(p + hw)
    x = _rand(3, hw, p, gen=g, scale=4.0)
    proto = torch.softmax(x, dim=2)
    pooled = proto.amax(dim=1) if mode == 0 else proto.sum(dim=1)
    pr, po = K.softmax_pool(x.float().to(gpu).view(3, hw, 1, p), mode)
    assert torch.allclose(pr.double().cpu().view(3, hw, p), proto, rtol=1e-5, atol=1e-7)
    assert torch.allclose(po.double().cpu(), pooled, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("thresh", [None, 0.1])
def test_nonneg_linear(gpu, thresh):
    g = torch.Generator().manual_seed(3)
    x = torch.rand(64, 768, generator=g, dtype=torch.float64) * 0.3
    w, b = _rand(200, 768, gen=g), _rand(200, gen=g)
    xc = torch.where(x < 0.1, 0.0, x) if thresh else x
    ref = xc @ torch.relu(w).t() + b
    d = lambda t: t.float().to(gpu)  # noqa: E731
    xo, out = K.nonneg_linear(d(x), d(w), d(b), thresh)
    assert torch.equal(xo.cpu(), xc.float())
    assert torch.allclose(out.double().cpu(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("p,hw", [(16, 64), (2048, 256), (100, 37)])
def test_count_gumbel_injected_noise(gpu, p, hw):
    g = torch.Generator().manual_seed(p)
    logits = torch.randn(2, hw, p, generator=g)
    e = torch.empty(2, p, hw).exponential_(generator=g)
    z = logits - e.log().permute(0, 2, 1)
    idx = z.argmax(dim=2)
    proto, hist = K.count_gumbel(logits.to(gpu).view(2, hw, 1, p), 1.0, e.to(gpu).view(2, p, hw, 1), seed=0)
    proto = proto.cpu().view(2, hw, p)
    assert torch.equal(proto.argmax(dim=2), idx)
    assert torch.all((proto.sum(dim=2) - 1).abs() <= 1.2e-7)
    assert torch.count_nonzero(proto) == 2 * hw
    ref_hist = torch.stack([torch.bincount(idx[i], minlength=p) for i in range(2)])
    assert torch.equal(hist.cpu().long(), ref_hist)


def test_count_gumbel_philox_statistics(gpu):
    """In-kernel Philox noise: with all-zero logits the argmax is uniform over P."""
    p, hw, b = 16, 4096, 4
    logits = torch.zeros(b, hw, 1, p, device=gpu)
    _, hist = K.count_gumbel(logits, 1.0, None, seed=1234)
    h = hist.cpu().double().sum(0)
    expected = b * hw / p
    chi2 = float(((h - expected) ** 2 / expected).sum())
    assert chi2 < 50.0, chi2              # 15 dof: p(chi2 > 50) ~ 1e-5
    _, hist2 = K.count_gumbel(logits, 1.0, None, seed=1234)
    assert torch.equal(hist, hist2)       # counter-based: reproducible per seed
    _, hist3 = K.count_gumbel(logits, 1.0, None, seed=99)
    assert not torch.equal(hist, hist3)


def test_count_gumbel_philox_follows_softmax(gpu):
    """Gumbel-max law of the in-kernel noise (hardware log2 / exp2 path): the argmax of
    (x - log E) / tau falls on channel i with probability softmax(x)_i, for any tau."""
    p, hw, b = 8, 8192, 4
    x = torch.linspace(-1.5, 1.0, p)
    logits = x.view(1, 1, 1, p).expand(b, hw, 1, p).contiguous().to(gpu)
    probs = torch.softmax(x.double(), 0)
    for tau, seed in ((1.0, 7), (0.5, 8)):
        proto, hist = K.count_gumbel(logits, tau, None, seed=seed)
        h = hist.cpu().double().sum(0)
        expected = probs * b * hw
        chi2 = float(((h - expected) ** 2 / expected).sum())
        assert chi2 < 40.0, (tau, chi2)       # 7 dof: p(chi2 > 40) ~ 1e-6
        s = proto.sum(dim=3)
        assert torch.allclose(s, torch.ones_like(s)) and torch.equal((proto > 0).sum(dim=3), torch.ones_like(s).long())


def test_count_finish_and_encode(gpu):
    hist = torch.tensor([[0, 1, 2, 3, 4, 7]], dtype=torch.int32, device=gpu)
    raw, cl = K.count_finish(hist, None, 3, True)
    assert torch.equal(cl.cpu(), torch.tensor([[0.0, 1, 2, 3, 3, 3]]))
    sums = torch.tensor([[0.4, 0.5, 1.5, 2.5, 3.7, -0.2]], device=gpu)
    _, cl2 = K.count_finish(None, sums, 3, True)
    assert torch.equal(cl2.cpu(), torch.tensor([[0.0, 0.0, 2.0, 2.0, 3.0, 0.0]]))   # half to even
    _, cl3 = K.count_finish(None, sums, 3, False)
    assert torch.allclose(cl3.cpu(), torch.tensor([[0.4, 0.5, 1.5, 2.5, 3.0, 0.0]]))
    x = torch.tensor([[0.0, 1.0, 3.0], [0.05, 2.0, 2.9], [1.0, 0.0, 0.2], [3.0, 2.0, 1.0]], device=gpu)
    enc = K.count_encode(x, 3, kind=0, do_round=True).cpu().view(4, 3, 3)
    from count_pipnet_amd.count_pipnet_utils import create_modified_encoding
    assert torch.equal(enc, create_modified_encoding(x.cpu().round(), 3))
    w = torch.tensor([1 / 3, 2 / 3, 1.0], device=gpu)
    lin = K.count_encode(x, 3, kind=1, do_round=False, w=w).cpu()
    assert torch.allclose(lin, (x.cpu().reshape(-1, 1) * w.cpu()).view(4, 9))


@pytest.mark.parametrize("cin,cout,h,k,s,pad,epi", [
    (64, 64, 56, 3, 1, 1, _lib.EPI_BIAS_RELU), (128, 128, 56, 3, 2, 1, _lib.EPI_BIAS_RELU),
    (256, 1024, 28, 1, 1, 0, _lib.EPI_BIAS_RESID_RELU), (64, 256, 56, 1, 1, 0, _lib.EPI_BIAS),
    (256, 512, 56, 1, 2, 0, _lib.EPI_BIAS), (4, 64, 64, 7, 2, 3, _lib.EPI_BIAS_RELU),
    (12, 40, 9, 3, 1, 1, _lib.EPI_NONE), (32, 48, 7, 5, 2, 2, _lib.EPI_BIAS_RESID_RELU)])
def test_conv2d_nhwc(gpu, cin, cout, h, k, s, pad, epi):
    g = torch.Generator().manual_seed(cin * 7 + h + k)
    x = _rand(2, cin, h, h, gen=g)
    w = _rand(cout, cin, k, k, gen=g, scale=1.0 / (cin * k * k) ** 0.5)
    b = _rand(cout, gen=g)
    y = F.conv2d(x, w, b if epi != _lib.EPI_NONE else None, stride=s, padding=pad)
    r = _rand(*y.shape, gen=g)
    if epi == _lib.EPI_BIAS_RELU:
        y = torch.relu(y)
    if epi == _lib.EPI_BIAS_RESID_RELU:
        y = torch.relu(y + r)
    d = lambda t: t.float().to(gpu)  # noqa: E731
    out = K.conv2d_nhwc(d(x.permute(0, 2, 3, 1).contiguous()), d(w.permute(0, 2, 3, 1).contiguous()),
                        d(b) if epi != _lib.EPI_NONE else None, s, pad, epi,
                        d(r.permute(0, 2, 3, 1).contiguous()) if epi == _lib.EPI_BIAS_RESID_RELU else None)
    ref = y.permute(0, 2, 3, 1)
    assert torch.allclose(out.double().cpu(), ref, rtol=2e-5, atol=2e-5), (out.double().cpu() - ref).abs().max()


@pytest.mark.parametrize("c,h", [(64, 112), (8, 9)])
def test_maxpool_and_relayout(gpu, c, h):
    g = torch.Generator().manual_seed(c + h)
    x = torch.randn(2, c, h, h, generator=g)
    ref = F.max_pool2d(x, 3, 2, 1).permute(0, 2, 3, 1)
    out = K.maxpool2d_nhwc(x.permute(0, 2, 3, 1).contiguous().to(gpu), 3, 2, 1).cpu()
    assert torch.equal(out, ref)
    xin = torch.randn(2, 3, h, h, generator=g)
    y = K.nchw_to_nhwc(xin.to(gpu), 4).cpu()
    assert torch.equal(y[..., :3], xin.permute(0, 2, 3, 1)) and torch.all(y[..., 3] == 0)


@pytest.mark.parametrize("epi", [_lib.EPI_NONE, _lib.EPI_BIAS, _lib.EPI_MUL, _lib.EPI_RESID, _lib.EPI_BIAS_GELU])
def test_linear_splitk(gpu, epi):
    """Short-M products take the split-K path (workspace slabs + reducing epilogue)."""
    from count_pipnet_amd.kernels import splitk_factor
    g = torch.Generator().manual_seed(100 + epi)
    m, n, k = 37, 1536, 2048
    assert splitk_factor(m, n, k) > 1
    a, w, b = _rand(m, k, gen=g), _rand(n, k, gen=g, scale=0.03), _rand(n, gen=g)
    s, r = _rand(n, gen=g), _rand(m, n, gen=g)
    acc = a @ w.t()
    ref = {_lib.EPI_NONE: acc, _lib.EPI_BIAS: acc + b, _lib.EPI_MUL: acc * r, _lib.EPI_RESID: r + s * (acc + b),
           _lib.EPI_BIAS_GELU: F.gelu(acc + b)}[epi]
    d = lambda t: t.float().to(gpu)  # noqa: E731
    out = K.linear(d(a), d(w), d(b), epi, scale=d(s), r=d(r)).double().cpu()
    tol = 4e-6 * (1 + ref.abs()) + 4e-6 * ((a.abs() @ w.abs().t()) * (1 + s.abs() + r.abs()))
    assert torch.all((out - ref).abs() <= tol), (out - ref).abs().max()


@pytest.mark.parametrize("c,m", [(96, 1000), (96, 128), (192, 777), (192, 64), (96, 1), (192, 3), (192, 40000)])
def test_cnblock_mlp_fused(gpu, c, m):
    """The fused narrow-stage CNBlock MLP (csrc/mlp_f32.hip): x + gamma*(W2 gelu(W1 t + b1) + b2)
    against fp64 torch, ragged M (rows past the last 128-/64-pixel workgroup), asymmetric
    weights; and against the unfused Linear1+GELU / Linear2+residual kernels (different fp32
    summation order, so close, not bitwise)."""
    g = torch.Generator().manual_seed(c + m)
    t, x = _rand(m, c, gen=g), _rand(m, c, gen=g)
    w1, b1 = _rand(4 * c, c, gen=g, scale=0.1), _rand(4 * c, gen=g, scale=0.5)
    w2, b2 = _rand(c, 4 * c, gen=g, scale=0.05), _rand(c, gen=g)
    gm = _rand(c, gen=g)
    hid = F.gelu(t @ w1.t() + b1)
    ref = x + gm * (hid @ w2.t() + b2)
    d = lambda v: v.float().to(gpu).contiguous()  # noqa: E731
    xo = d(x)
    K.cnblock_mlp(d(t), d(w1), d(b1), d(w2), d(b2), d(gm), xo)
    out = xo.double().cpu()
    tol = 4e-6 * (gm.abs() * ((hid.abs() @ w2.abs().t()) + (t.abs() @ w1.abs().t()).mean())) + 1e-5
    assert torch.all((out - ref).abs() <= tol), (out - ref).abs().max()
    # the unfused kernels on the same inputs
    xu = d(x)
    u = K.linear(d(t), d(w1), d(b1), _lib.EPI_BIAS_GELU)
    K.linear(u, d(w2), d(b2), _lib.EPI_RESID, scale=d(gm), r=xu, out=xu)
    assert torch.allclose(xo, xu, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("m", [16384, 777, 3])
def test_cnblock_mlp_fused_hidden_split(gpu, m):
    """C = 192 on a <= 16 x 16 map (C5's stage 2): the hidden dimension split over two waves
    per pixel group (HS = 2, chosen by the map size) against fp64 torch, ragged M; and it does
    not depend on M (bitwise, prefixes of the batch)."""
    c, hw = 192, 256
    g = torch.Generator().manual_seed(c + m + hw)
    t, x = _rand(m, c, gen=g), _rand(m, c, gen=g)
    w1, b1 = _rand(4 * c, c, gen=g, scale=0.1), _rand(4 * c, gen=g, scale=0.5)
    w2, b2 = _rand(c, 4 * c, gen=g, scale=0.05), _rand(c, gen=g)
    gm = _rand(c, gen=g)
    hid = F.gelu(t @ w1.t() + b1)
    ref = x + gm * (hid @ w2.t() + b2)
    d = lambda v: v.float().to(gpu).contiguous()  # noqa: E731
    xo = d(x)
    K.cnblock_mlp(d(t), d(w1), d(b1), d(w2), d(b2), d(gm), xo, hw=hw)
    out = xo.double().cpu()
    tol = 4e-6 * (gm.abs() * ((hid.abs() @ w2.abs().t()) + (t.abs() @ w1.abs().t()).mean())) + 1e-5
    assert torch.all((out - ref).abs() <= tol), (out - ref).abs().max()
    for rows in {m // 2 + 1, 1}:
        part = d(x[:rows])
        K.cnblock_mlp(d(t[:rows]), d(w1), d(b1), d(w2), d(b2), d(gm), part, hw=hw)
        assert torch.equal(part, xo[:rows]), rows


def test_cnblock_mlp_rejects_unsupported(gpu):
    z = torch.zeros(4, 384, device=gpu)
    with pytest.raises(RuntimeError):
        K.cnblock_mlp(z, torch.zeros(1536, 384, device=gpu), torch.zeros(1536, device=gpu),
                      torch.zeros(384, 1536, device=gpu), torch.zeros(384, device=gpu), torch.zeros(384, device=gpu), z)


@pytest.mark.parametrize("c,m", [(96, 70000), (192, 40000)])
def test_cnblock_mlp_batch_invariant(gpu, c, m):
    """The launch configuration of the fused MLP depends on M (workgroup size), its per-pixel
    arithmetic must not: every instantiation gives the same bits for a pixel."""
    g = torch.Generator(device=gpu).manual_seed(c)
    t = torch.randn(m, c, device=gpu, generator=g)
    x = torch.randn(m, c, device=gpu, generator=g)
    w1 = torch.randn(4 * c, c, device=gpu, generator=g) * 0.1
    b1 = torch.randn(4 * c, device=gpu, generator=g)
    w2 = torch.randn(c, 4 * c, device=gpu, generator=g) * 0.05
    b2 = torch.randn(c, device=gpu, generator=g)
    gm = torch.randn(c, device=gpu, generator=g)
    full = x.clone()
    K.cnblock_mlp(t, w1, b1, w2, b2, gm, full)
    for rows in (20000, 9000, 4096, 1000, 17):
        part = x[:rows].clone()
        K.cnblock_mlp(t[:rows].contiguous(), w1, b1, w2, b2, gm, part)
        assert torch.equal(part, full[:rows]), rows


@pytest.mark.parametrize("m,n,k,epi", [
    (46656 // 2, 1536, 384, "gelu"),     # stage-3 fc1 shape (half batch)
    (20001, 3072, 768, "gelu"),          # stage-4 fc1 shape, ragged M (last tile 33 rows)
    (43264 // 4, 768, 3072, "resid"),    # stage-4 fc2: residual epilogue in place, K = 3072
    (30001, 1024, 512, "bias"),          # bias epilogue, ragged M
    (300, 256, 512, "none"),             # fewer tiles than CUs
])
def test_gemm_product_tile_vs_fp64(gpu, m, n, k, epi):
    """The product 128x128 fp32 tile on the stage-3/4 CNBlock shapes: within 1e-3 of an fp64
    reference, rows past M never written, the residual case in place (R aliases C, as the
    CNBlock residual stream does)."""
    g = torch.Generator().manual_seed(m + n + k)
    a = torch.randn(m, k, generator=g).to(gpu)
    w = (torch.randn(n, k, generator=g) * 0.05).to(gpu)
    b = torch.randn(n, generator=g).to(gpu)
    s = torch.randn(n, generator=g).to(gpu)
    r = torch.randn(m, n, generator=g).to(gpu)
    e = {"gelu": _lib.EPI_BIAS_GELU, "resid": _lib.EPI_RESID, "none": _lib.EPI_NONE, "bias": _lib.EPI_BIAS}[epi]
    if epi == "resid":
        buf = torch.empty(m + 7, n, device=gpu)
        buf[m:] = 12345.0                                   # rows past M: must stay untouched
        buf[:m] = r
        K.linear(a, w, b, e, scale=s, r=buf[:m], out=buf[:m])
    else:
        buf = torch.full((m + 7, n), 12345.0, device=gpu)
        K.linear(a, w, b, e, scale=s, out=buf[:m])
    torch.cuda.synchronize()
    assert torch.all(buf[m:] == 12345.0)
    ref = a.double() @ w.double().t()
    if epi == "gelu":
        ref = torch.nn.functional.gelu(ref + b.double())
    elif epi == "resid":
        ref = r.double() + s.double() * (ref + b.double())
    elif epi == "bias":
        ref = ref + b.double()
    assert (buf[:m].double() - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("k,epi,aload", [
    (1536, "resid", 0),                  # C2 stage-3 fc2 (in place)
    (768, "bias", 1),                    # stage-2 -> 3 downsample (2x2 stride-1 gather, 28 -> 27)
    (768, "bias", 2),                    # torchvision's stride-2 downsample (56 -> 28) at 32 images
    (1536, "none", 0),
])
def test_gemm_wide_rows_equal_64row_rows(gpu, k, epi, aload):
    """Variant 5 (the 192 x 384 tile on 12 waves) is picked by shape (N = 384, K >= 768, >= 100
    tiles), variant 2 (the 64-row tile) below that; both run the same 32 x 64 wave K order, so a
    row's bits never depend on which one the batch size selected; ragged last tiles stay in bounds."""
    n = 384
    e = {"resid": _lib.EPI_RESID, "bias": _lib.EPI_BIAS, "none": _lib.EPI_NONE}[epi]
    g = torch.Generator(device=gpu).manual_seed(k + aload)
    w = torch.randn(n, k, device=gpu, generator=g) * 0.05
    b = torch.randn(n, device=gpu, generator=g)
    s = torch.randn(n, device=gpu, generator=g)
    if aload:
        c = k // 4
        stride = aload                 # (the column is the 2x2 gather stride) 1: 28 -> 27 (C2), 2: 56 -> 28
        hin = 28 if stride == 1 else 56
        hout = (hin - 2) // stride + 1
        imgs, small = (40, 20) if stride == 1 else (32, 16)  # 29,160 / 14,580 or 25,088 / 12,544 rows
        x = torch.randn(imgs, hin, hin, c, device=gpu, generator=g)
        wk = w.view(n, 2, 2, c).contiguous()
        hw = hout * hout
        assert K.gemm_variant(imgs * hw, n, k, e, 1) == 5 and K.gemm_variant(small * hw, n, k, e, 1) == 2
        full = K.conv2x2(x, wk, b, stride)
        part = K.conv2x2(x[:small].contiguous(), wk, b, stride)
        torch.cuda.synchronize()
        assert torch.equal(part, full[:small])
        ref = torch.nn.functional.conv2d(x[:1].permute(0, 3, 1, 2).double(), wk.permute(0, 3, 1, 2).double(),
                                         b.double(), stride=stride).permute(0, 2, 3, 1)
        assert (full[:1].double() - ref).abs().max().item() < 1e-3
        return
    m, ms = 46656 - 77, 19199                              # ragged wide tiles / 64-row tiles
    assert K.gemm_variant(m, n, k, e) == 5 and K.gemm_variant(ms, n, k, e) == 2
    a = torch.randn(m, k, device=gpu, generator=g)
    r = torch.randn(m + 5, n, device=gpu, generator=g)
    r[m:] = 12345.0
    if epi == "resid":
        full, part = r.clone(), r[:ms].clone()
        K.linear(a, w, b, e, scale=s, r=full[:m], out=full[:m])
        K.linear(a[:ms].contiguous(), w, b, e, scale=s, r=part, out=part)
        torch.cuda.synchronize()
        assert torch.all(full[m:] == 12345.0)
    else:
        full = torch.full((m + 5, n), 12345.0, device=gpu)
        K.linear(a, w, b, e, scale=s, out=full[:m])
        part = K.linear(a[:ms].contiguous(), w, b, e, scale=s)
        torch.cuda.synchronize()
        assert torch.all(full[m:] == 12345.0)
    assert torch.equal(part, full[:ms])
    ref = a[-300:].double() @ w.double().t()
    if epi == "resid":
        ref = r[m - 300:m].double() + s.double() * (ref + b.double())
    elif epi == "bias":
        ref = ref + b.double()
    assert (full[m - 300:m].double() - ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("b,hw,p,k,thresh", [
    (64, 26 * 26, 768, 200, 0.1),     # C2 head (inference: 0.1 presence threshold)
    (5, 26 * 26, 768, 200, None),     # raw mode: x' = pooled
    (3, 28 * 28, 2048, 200, 0.1),     # C3 head (P = 2048)
    (4, 7 * 7, 96, 9, 0.1),           # K < 16, one pixel block per image
    (2, 33, 20, 3, 0.1),              # P % 8 != 0 (bf16 takes the lane-strided kernel), ragged pixel block
    (2, 100, 130, 37, None),          # P % 4 != 0: the scalar GEMV slices
])
def test_fused_head_bitwise_two_kernel_path(gpu, dtype, b, hw, p, k, thresh):
    """pipnet_softmax_pool_linear_{f32,bf16} (the NonNegLinear in each image's last workgroup,
    one launch) against pipnet_softmax_pool + pipnet_nonneg_linear (two launches): proto,
    pooled, x' and logits bitwise equal; logits within 1e-5 of an fp64 reference."""
    g = torch.Generator().manual_seed(b * 7 + p + k)
    feat = (torch.randn(b, hw, p, generator=g) * 3).to(gpu)
    if dtype == "bf16":
        feat = feat.to(torch.bfloat16)
    w = torch.randn(k, p, generator=g).to(gpu)          # negative entries: relu(W) matters
    bias = torch.randn(k, generator=g).to(gpu)
    h = 1
    f4 = feat.view(b, h, hw, p)
    proto, pooled, xo, out = K.softmax_pool_linear(f4, w, bias, thresh)
    if dtype == "bf16":
        proto2, pooled2 = K.softmax_pool_bf16(f4, 0)
    else:
        proto2, pooled2 = K.softmax_pool(f4, 0)
    xo2, out2 = K.nonneg_linear(pooled2, w, bias, thresh)
    torch.cuda.synchronize()
    assert torch.equal(proto, proto2)
    assert torch.equal(pooled, pooled2)
    assert torch.equal(xo, xo2)
    assert torch.equal(out, out2)
    xr = pooled.double()
    if thresh is not None:
        xr = torch.where(xr < thresh, 0.0, xr)
    ref = xr @ w.double().clamp_min(0).t() + bias.double()
    assert (out.double() - ref).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item())
    # a second call into reused (non-zero) output buffers and the same workspace, whose tickets
    # the first call must have left at zero
    proto3, pooled3, xo3, out3 = K.softmax_pool_linear(f4, w, bias, thresh, out=(proto, pooled, xo, out.clone()))
    torch.cuda.synchronize()
    assert torch.equal(out3, out2) and torch.equal(pooled3, pooled2)
    pmax, tickets = K._HEAD_WS[(f4.device.index, torch.cuda.current_stream(f4.device).cuda_stream)]
    assert int(tickets.abs().sum().item()) == 0 and float(pmax.abs().sum().item()) == 0.0   # reset by the launch


def test_fused_head_is_one_launch(gpu):
    """The PIP-Net head is a single kernel launch (no zero-fill of pooled or tickets ahead of it):
    counted with the HIP-graph node count of a captured call."""
    g = torch.Generator().manual_seed(5)
    feat = (torch.randn(8, 2, 26, 768, generator=g) * 6).to(gpu)      # peaked softmax: presence > 0.1
    w = torch.randn(200, 768, generator=g).to(gpu)
    K.softmax_pool_linear(feat, w, None, 0.1)          # workspace allocated outside the capture
    s = torch.cuda.Stream(gpu)
    s.wait_stream(torch.cuda.current_stream(gpu))
    with torch.cuda.stream(s):
        K.softmax_pool_linear(feat, w, None, 0.1)      # this stream's workspace, outside the capture
        outs = [torch.full((8, 2, 26, 768), -1.0, device=gpu), torch.full((8, 768), -1.0, device=gpu),
                torch.full((8, 768), -1.0, device=gpu), torch.full((8, 200), -1.0, device=gpu)]
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(graph, stream=s):
        K.softmax_pool_linear(feat, w, None, 0.1, out=tuple(outs))
    torch.cuda.synchronize()
    n = _graph_nodes(graph)
    graph.instantiate()
    graph.replay()
    graph.replay()
    torch.cuda.synchronize()
    ref = K.softmax_pool_linear(feat, w, None, 0.1)
    torch.cuda.synchronize()
    assert n == 1, n
    assert ref[3].abs().sum().item() > 0
    for name, a, r in zip(("proto", "pooled", "x'", "logits"), outs, ref):
        assert torch.equal(a, r), (name, (a - r).abs().max().item())


def _graph_nodes(graph) -> int:
    """Number of nodes of a captured torch CUDAGraph(keep_graph=True) (hipGraphGetNodes)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    count = ctypes.c_size_t(0)
    hip.hipGraphGetNodes.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t)]
    assert hip.hipGraphGetNodes(ctypes.c_void_p(graph.raw_cuda_graph()), None, ctypes.byref(count)) == 0
    return count.value


def test_fused_head_reads_weight_at_call_time(gpu):
    """The fused head reads W when it runs: an in-place clamp between two calls (test.py:71-73)
    changes the logits exactly as the two-kernel path does."""
    g = torch.Generator().manual_seed(3)
    feat = torch.randn(4, 1, 49, 64, generator=g).to(gpu)
    w = torch.randn(10, 64, generator=g).to(gpu)
    _, _, _, out_a = K.softmax_pool_linear(feat, w, None, 0.1)
    out_a = out_a.clone()
    w.sub_(0.5).clamp_(min=0)
    _, pooled, _, out_b = K.softmax_pool_linear(feat, w, None, 0.1)
    _, ref = K.nonneg_linear(pooled, w, None, 0.1)
    torch.cuda.synchronize()
    assert torch.equal(out_b, ref)
    assert not torch.equal(out_a, out_b)
