"""ResNet training building blocks on the GPU (csrc/bn_ops.hip, count_pipnet_amd.resnet_train)
against float64 torch autograd.

* train-mode BatchNorm2d: batch statistics, the running-statistics update (momentum,
  unbiased variance) and the normalise (+ residual) (+ ReLU) == F.batch_norm(training=True);
  its backward (ReLU mask from the saved output, the identity-path gradient) == autograd;
* the stride scatter and the zero-padded conv weight gradient (3x3 pad 1, strided 1x1);
* one Bottleneck with a stride-2 downsample (layer2.0's shape) and one without, train mode:
  every parameter gradient and the input gradient == autograd of the torch module, and the
  running statistics the forward updated == torch's.
"""
import pytest
import torch
import torch.nn.functional as F

from count_pipnet_amd import kernels as K
from count_pipnet_amd import resnet_train as R
from count_pipnet_amd.resnet_features import Bottleneck, conv1x1

pytestmark = pytest.mark.gpu


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("b,h,w,c,relu,res", [(4, 14, 14, 64, True, False), (2, 8, 8, 256, False, True),
                                              (3, 7, 5, 2048, True, True), (2, 3, 3, 16, False, False)])
def test_bn_forward_matches_torch(gpu, b, h, w, c, relu, res):
    g = torch.Generator().manual_seed(b * h + c)
    x = torch.randn(b, c, h, w, generator=g, dtype=torch.float64) * 3 + 1.5
    gamma = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(c, generator=g, dtype=torch.float64)
    r = torch.randn(b, c, h, w, generator=g, dtype=torch.float64) if res else None
    rm0 = torch.randn(c, generator=g, dtype=torch.float64)
    rv0 = torch.rand(c, generator=g, dtype=torch.float64) + 0.5
    rm, rv = rm0.clone(), rv0.clone()
    ref = F.batch_norm(x, rm, rv, gamma, beta, training=True, momentum=0.1, eps=1e-5)
    if res:
        ref = ref + r
    if relu:
        ref = torch.relu(ref)
    xd = _nhwc(x.float()).to(gpu)
    hrm, hrv = rm0.float().to(gpu), rv0.float().to(gpu)
    mean, invstd = K.bn_stats(xd, 1e-5, 0.1, hrm, hrv)
    y = K.bn_apply(xd, mean, invstd, gamma.float().to(gpu), beta.float().to(gpu),
                   _nhwc(r.float()).to(gpu) if res else None, relu)
    torch.testing.assert_close(y.cpu().double(), _nhwc(ref), rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(hrm.cpu().double(), rm, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(hrv.cpu().double(), rv, rtol=1e-5, atol=1e-6)
    m2 = xd.view(-1, c).double()
    torch.testing.assert_close(mean.cpu().double(), m2.mean(0).cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("b,h,c,relu,masked", [(4, 14, 64, True, True), (2, 8, 512, False, False),
                                               (3, 5, 2048, True, False), (2, 3, 16, False, True)])
def test_bn_backward_matches_autograd(gpu, b, h, c, relu, masked):
    g = torch.Generator().manual_seed(b * h * c)
    x = (torch.randn(b, c, h, h, generator=g, dtype=torch.float64) * 2 + 0.7).requires_grad_(True)
    gamma = (torch.rand(c, generator=g, dtype=torch.float64) + 0.5).requires_grad_(True)
    beta = torch.randn(c, generator=g, dtype=torch.float64).requires_grad_(True)
    r = torch.randn(b, c, h, h, generator=g, dtype=torch.float64)
    y = F.batch_norm(x, None, None, gamma, beta, training=True, eps=1e-5) + r
    if relu:
        y = torch.relu(y)
    dy = torch.randn(b, c, h, h, generator=g, dtype=torch.float64)
    y.backward(dy)
    xd = _nhwc(x.detach().float()).to(gpu)
    mean, invstd = K.bn_stats(xd, 1e-5, 0.1)
    out = K.bn_apply(xd, mean, invstd, gamma.detach().float().to(gpu), beta.detach().float().to(gpu),
                     _nhwc(r.float()).to(gpu), relu)
    dx, dm, dg, db = K.bn_backward(xd, _nhwc(dy.float()).to(gpu), mean, invstd, gamma.detach().float().to(gpu),
                                   relu_out=out if relu else None, want_masked=masked)
    scale = x.grad.abs().max().item()
    torch.testing.assert_close(dx.cpu().double(), _nhwc(x.grad), rtol=1e-4, atol=1e-5 * scale)
    torch.testing.assert_close(dg.cpu().double(), gamma.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(db.cpu().double(), beta.grad, rtol=1e-4, atol=1e-4)
    if masked:
        want = dy * (y.detach() > 0) if relu else dy
        torch.testing.assert_close(dm.cpu().double(), _nhwc(want), rtol=0, atol=1e-6)


@pytest.mark.parametrize("b,oh,ow,c,h,w,s,acc", [(2, 28, 28, 64, 56, 56, 2, False), (3, 4, 5, 8, 8, 10, 2, True),
                                                 (1, 3, 3, 4, 7, 7, 3, True)])
def test_stride_scatter(gpu, b, oh, ow, c, h, w, s, acc):
    g = torch.Generator().manual_seed(oh * c)
    x = torch.randn(b, oh, ow, c, generator=g)
    base = torch.randn(b, h, w, c, generator=g)
    want = base.clone() if acc else torch.zeros(b, h, w, c)
    want[:, 0:oh * s:s, 0:ow * s:s] += x
    out = base.clone().to(gpu) if acc else None
    got = K.stride_scatter(x.to(gpu), h, w, s, out=out, accumulate=acc)
    assert torch.equal(got.cpu(), want)


@pytest.mark.parametrize("b,h,cin,cout,k,s,p", [(2, 14, 64, 64, 3, 1, 1), (2, 15, 32, 48, 3, 2, 1),
                                                (3, 9, 16, 32, 1, 2, 0), (1, 8, 8, 4, 7, 2, 3)])
def test_wgrad_conv_padded(gpu, b, h, cin, cout, k, s, p):
    g = torch.Generator().manual_seed(h * cin + k)
    x = torch.randn(b, cin, h, h, generator=g, dtype=torch.float64)
    wt = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64).requires_grad_(True)
    y = F.conv2d(x, wt, stride=s, padding=p)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    out = torch.empty(cout, k * k * cin, device=gpu)
    K.wgrad_conv(_nhwc(dy.float()).to(gpu), _nhwc(x.float()).to(gpu), k, k, s, out, pad=p)
    got = out.view(cout, k, k, cin).permute(0, 3, 1, 2).cpu().double()
    torch.testing.assert_close(got, wt.grad, rtol=1e-4, atol=1e-4 * wt.grad.abs().max().item())


def _block(inplanes, planes, stride, seed, gpu):
    torch.manual_seed(seed)
    ds = None
    if stride != 1 or inplanes != planes * 4:
        ds = torch.nn.Sequential(conv1x1(inplanes, planes * 4, stride), torch.nn.BatchNorm2d(planes * 4))
    blk = Bottleneck(inplanes, planes, stride, ds)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
                m.running_mean.uniform_(-0.1, 0.1)
                m.running_var.uniform_(0.8, 1.2)
    return blk.to(gpu).train()


@pytest.mark.parametrize("inplanes,planes,stride,b,h", [(256, 128, 2, 2, 16), (512, 128, 1, 2, 8), (64, 64, 1, 3, 10)])
def test_bottleneck_train_step_matches_autograd(gpu, inplanes, planes, stride, b, h):
    """One Bottleneck in train mode: the HIP forward (BN batch statistics) and backward vs
    autograd of the same torch module in float64 (the module's own running stats updated by
    exactly one forward each)."""
    blk = _block(inplanes, planes, stride, inplanes + planes, gpu)
    ref = _block(inplanes, planes, stride, inplanes + planes, gpu).double()
    g = torch.Generator().manual_seed(stride * 100 + h)
    x = torch.randn(b, inplanes, h, h, generator=g)
    xr = x.double().to(gpu).requires_grad_(True)
    yr = ref(xr)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double().to(gpu))
    cache = {}
    xh = _nhwc(x).to(gpu)
    out, rec = R._block_forward(cache, "blk", blk, xh, True)
    torch.testing.assert_close(out.cpu().double(), _nhwc(yr.detach().cpu()), rtol=1e-4, atol=1e-4)
    dx = R._block_backward(cache, "blk", blk, rec, _nhwc(dy).to(gpu), need_dx=True)
    torch.testing.assert_close(dx.cpu().double(), _nhwc(xr.grad.cpu()), rtol=1e-3,
                               atol=2e-4 * xr.grad.abs().max().item())
    rp = dict(ref.named_parameters())
    for n, p in blk.named_parameters():
        want = rp[n].grad.cpu()
        err = (p.grad.cpu().double() - want).abs().max().item() / (want.abs().max().item() + 1e-12)
        assert err < 1e-3, f"{n}: relative error {err:.3g}"
    rb = dict(ref.named_buffers())
    for n, t in blk.named_buffers():
        if n.endswith(("running_mean", "running_var")):
            torch.testing.assert_close(t.cpu().double(), rb[n].cpu(), rtol=1e-4, atol=1e-5, msg=n)
        elif n.endswith("num_batches_tracked"):
            assert int(t) == int(rb[n]) == 1
