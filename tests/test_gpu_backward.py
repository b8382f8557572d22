"""Backward building blocks on the GPU (csrc/backward_ops.hip) against float64 torch.

* wgrad (dW = A^T B over pixel rows): ragged tiles (N not a multiple of 128), short and long
  reductions, strided row views, accumulate, the single-slab direct path; bit-identical
  across repeated runs (fixed slabs, fixed-order reduction);
* colsum: ragged N, accumulate.
"""
import pytest
import torch

from count_pipnet_amd import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("m,n1,n2", [(86528, 768, 3072), (4096, 192, 96), (37, 12, 20), (1000, 132, 260),
                                     (32, 128, 128), (5, 4, 8)])
def test_wgrad(gpu, m, n1, n2):
    g = torch.Generator().manual_seed(m + n1 + n2)
    a = torch.randn(m, n1, generator=g).to(gpu)
    b = torch.randn(m, n2, generator=g).to(gpu)
    out = K.wgrad(a, b)
    ref = (a.double().t() @ b.double())
    tol = 2e-5 * (m ** 0.5)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=tol)
    again = K.wgrad(a, b)
    assert torch.equal(out, again)


def test_wgrad_strided_and_accumulate(gpu):
    g = torch.Generator().manual_seed(1)
    big = torch.randn(3000, 520, generator=g).to(gpu)
    a, b = big[:, 8:264], big[:, 264:520]          # row stride 520
    c0 = torch.randn(256, 256, generator=g).to(gpu)
    c = c0.clone()
    K.wgrad(a, b, out=c, accumulate=True)
    torch.testing.assert_close(c.double(), c0.double() + a.double().t() @ b.double(), rtol=1e-5, atol=2e-3)


@pytest.mark.parametrize("m,n", [(86528, 768), (17, 300), (1, 4)])
def test_colsum(gpu, m, n):
    g = torch.Generator().manual_seed(m * 7 + n)
    a = torch.randn(m, n, generator=g).to(gpu)
    torch.testing.assert_close(K.colsum(a).double(), a.double().sum(0), rtol=1e-5, atol=2e-5 * m ** 0.5)
    o = torch.ones(n, device=gpu)
    K.colsum(a, out=o, accumulate=True)
    torch.testing.assert_close(o.double(), 1.0 + a.double().sum(0), rtol=1e-5, atol=2e-5 * m ** 0.5)


# ---- training-step kernels vs torch autograd (float64 on the host) --------------------------
import torch.nn.functional as F  # noqa: E402

from count_pipnet_amd import _lib  # noqa: E402
from oracle import train_ref  # noqa: E402


def _g(seed):
    return torch.Generator().manual_seed(seed)


def test_gelu_forward_and_backward_epilogue(gpu):
    g = _g(3)
    m, k, n = 300, 64, 96
    h = torch.randn(m, n, generator=g) * 3
    torch.testing.assert_close(K.gelu_fwd(h.to(gpu)).cpu().double(), F.gelu(h.double()), rtol=1e-6, atol=1e-6)
    a = torch.randn(m, k, generator=g)
    wt = torch.randn(n, k, generator=g) * 0.1
    out = K.linear(a.to(gpu), wt.to(gpu), None, _lib.EPI_GELU_BWD, r=h.to(gpu)).cpu().double()
    hd = h.double().requires_grad_(True)
    F.gelu(hd).backward(a.double() @ wt.double().t())
    torch.testing.assert_close(out, hd.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("c,rows,rps,with_rs", [(768, 2 * 676, 676, True), (192, 4 * 64, 64, False), (96, 50, 25, True)])
def test_resid_scale_and_ls_backward(gpu, c, rows, rps, with_rs):
    g = _g(c + rows)
    x, y2, dy = (torch.randn(rows, c, generator=g) for _ in range(3))
    ls = torch.randn(c, generator=g) * 0.1
    rs = (torch.rand(rows // rps, generator=g) < 0.6).float() / 0.9 if with_rs else None
    out = K.resid_scale(x.to(gpu), y2.to(gpu), ls.to(gpu), None if rs is None else rs.to(gpu), rps).cpu()
    r_rows = rs.repeat_interleave(rps).view(-1, 1) if rs is not None else torch.ones(rows, 1)
    torch.testing.assert_close(out, x + r_rows * (ls * y2), rtol=1e-6, atol=1e-6)
    d_ls, d_b2 = torch.zeros(c, device=gpu), torch.full((c,), 2.0, device=gpu)
    dy2 = K.ls_backward(dy.to(gpu), y2.to(gpu), ls.to(gpu), None if rs is None else rs.to(gpu), rps, d_ls, d_b2,
                        accumulate=False)
    ls_d = ls.double().requires_grad_(True)
    y2_d = y2.double().requires_grad_(True)
    (r_rows.double() * (ls_d * y2_d)).backward(dy.double())
    torch.testing.assert_close(dy2.cpu().double(), y2_d.grad, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(d_ls.cpu().double(), ls_d.grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(d_b2.cpu().double(), y2_d.grad.sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("c,rows,want_dz", [(768, 1000, True), (384, 729, False), (192, 33, True), (96, 7, True)])
def test_ln_backward(gpu, c, rows, want_dz):
    g = _g(c * 3 + rows)
    z = torch.randn(rows, c, generator=g) * 2 + 0.5
    dt = torch.randn(rows, c, generator=g)
    gamma, beta = 1 + 0.1 * torch.randn(c, generator=g), 0.1 * torch.randn(c, generator=g)
    dg, dbt = torch.zeros(c, device=gpu), torch.zeros(c, device=gpu)
    dz = K.ln_backward(z.to(gpu), dt.to(gpu), gamma.to(gpu), dg, dbt, want_dz)
    zd, gd, bd = (t.double().requires_grad_(True) for t in (z, gamma, beta))
    F.layer_norm(zd, (c,), gd, bd, 1e-6).backward(dt.double())
    if want_dz:
        torch.testing.assert_close(dz.cpu().double(), zd.grad, rtol=1e-4, atol=1e-5)
    else:
        assert dz is None
    torch.testing.assert_close(dg.cpu().double(), gd.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dbt.cpu().double(), bd.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("b,h,w,c", [(2, 26, 26, 768), (3, 8, 8, 192), (1, 5, 9, 96)])
def test_dwconv7_forward_input_and_weight_grads(gpu, b, h, w, c):
    g = _g(b * 100 + h + c)
    x = torch.randn(b, c, h, w, generator=g)
    wt = torch.randn(c, 1, 7, 7, generator=g) * 0.1
    bias = torch.randn(c, generator=g)
    dz = torch.randn(b, c, h, w, generator=g)
    xn = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    wp = wt.reshape(c, 49).t().contiguous().to(gpu)
    y = K.dwconv7_plain(xn, wp, bias.to(gpu)).cpu().permute(0, 3, 1, 2).double()
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, wt, bias))
    ref = F.conv2d(xd, wd, bd, padding=3, groups=c)
    torch.testing.assert_close(y, ref.detach(), rtol=1e-5, atol=1e-5)
    ref.backward(dz.double())
    # input gradient: flipped taps, accumulated onto an existing buffer
    dzn = dz.permute(0, 2, 3, 1).contiguous().to(gpu)
    wflip = wt.flip(2, 3).reshape(c, 49).t().contiguous().to(gpu)
    base = torch.randn(b, h, w, c, generator=g)
    dx = K.dwconv7_plain(dzn, wflip, None, out=base.clone().to(gpu), accumulate=True).cpu()
    torch.testing.assert_close(dx.double(), base.double() + xd.grad.permute(0, 2, 3, 1), rtol=1e-5, atol=1e-5)
    dwp, dbias = torch.zeros(49, c, device=gpu), torch.zeros(c, device=gpu)
    K.dwconv7_wgrad(dzn, xn, dwp, dbias)
    torch.testing.assert_close(dwp.cpu().double(), wd.grad.reshape(c, 49).t(), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(dbias.cpu().double(), bd.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("b,h,cin,cout,stride", [(4, 27, 384, 768, 1), (2, 16, 96, 192, 2), (1, 7, 8, 12, 1)])
def test_wgrad_conv2x2(gpu, b, h, cin, cout, stride):
    g = _g(h * cin + stride)
    x = torch.randn(b, cin, h, h, generator=g)
    wt = torch.randn(cout, cin, 2, 2, generator=g) * 0.05
    oh = (h - 2) // stride + 1
    dy = torch.randn(b, cout, oh, oh, generator=g)
    wd = wt.double().requires_grad_(True)
    F.conv2d(x.double(), wd, stride=stride).backward(dy.double())
    out = torch.zeros(cout, 4 * cin, device=gpu)
    K.wgrad_conv2x2(dy.permute(0, 2, 3, 1).contiguous().to(gpu), x.permute(0, 2, 3, 1).contiguous().to(gpu),
                    stride, out)
    want = wd.grad.permute(0, 2, 3, 1).reshape(cout, 4 * cin)
    torch.testing.assert_close(out.cpu().double(), want, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("bh,hw,p,k,mode", [(2, 26, 768, 200, "train"), (3, 64, 32, 10, "finetune"),
                                            (2, 9, 20, 5, "pretrain")])
def test_head_backward_matches_autograd(gpu, bh, hw, p, k, mode):
    g = _g(bh * 1000 + p)
    n = 2 * bh
    side = int(hw ** 0.5) if int(hw ** 0.5) ** 2 == hw else None
    hh, ww = (side, side) if side else (hw, 1)
    logits = torch.randn(n, p, hh, ww, generator=g) * 3
    w = torch.randn(k, p, generator=g)
    ys = torch.randint(0, k, (bh,), generator=g)
    mult = 2.0
    w_align, w_tanh, w_class = (5.0, 2.0, 2.0) if mode != "pretrain" else (0.7, 5.0, 0.0)
    ld = logits.double().requires_grad_(True)
    proto = torch.softmax(ld, dim=1)
    pooled = F.adaptive_max_pool2d(proto, (1, 1)).flatten(1)
    out = pooled @ torch.relu(w.double()).t()
    terms = train_ref.loss_terms(proto, pooled, out, ys, mult)
    e1, e2 = train_ref.proto_pixels(proto[:bh]), train_ref.proto_pixels(proto[bh:])
    align = (train_ref.align_loss(e1, e2.detach()) + train_ref.align_loss(e2, e1.detach())) / 2   # train.py:163
    loss = w_align * align + w_tanh * terms["tanh"]
    if mode != "pretrain":
        loss = loss + w_class * terms["cls"]
    if mode == "finetune":
        loss = w_class * terms["cls"] + 0 * loss
    loss.backward()
    d_out = None
    if mode != "pretrain":
        d_out = train_ref.d_out(out.detach().float(), ys, mult, True, w_class).to(gpu)
    wa, wt_ = (0.0, 0.0) if mode == "finetune" else (w_align, w_tanh)
    proto_n = proto.detach().float().permute(0, 2, 3, 1).contiguous().to(gpu)
    dl = K.head_backward(proto_n, pooled.detach().float().to(gpu), d_out, w.to(gpu), wa, wt_)
    torch.testing.assert_close(dl.cpu().double().permute(0, 3, 1, 2), ld.grad, rtol=2e-4, atol=1e-6)
