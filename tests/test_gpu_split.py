"""Split-bf16 ("bf16x3") kernels of the ConvNeXt path (include/pipnet_amd.h,
pipnet_conv2d_nhwc_s3, pipnet_dwconv7_ln_s3, pipnet_layernorm_s3), through the C ABI.

* the producers write split planes [hi | lo] of exactly the value the fp32 kernel computes:
  bit-exact against RNE splits of the fp32 kernel's output;
* the split GEMM computes hi.hi + lo.hi + hi.lo in fp32: within 2e-6 (relative to max |y|)
  of that sum evaluated in fp64, and within 3e-5 of the exact fp64 product (the dropped
  lo.lo term and the lo roundings, ~2^-16 relative) -- for every tile it can run on,
  ragged M, 1x1 and 2x2 / stride 1-2 convolutions, and all three epilogues.
"""
import pytest
import torch

from count_pipnet_amd import _lib
from count_pipnet_amd import kernels as K

pytestmark = pytest.mark.gpu


def _split(x):
    hi = x.to(torch.bfloat16)
    return hi, (x - hi.float()).to(torch.bfloat16)


def _emulated(x, w, kh, stride):
    """fp64 value of the split product (hi.hi + lo.hi + hi.lo) and the exact fp64 product;
    x [B,H,W,Cin] fp32, w [Cout,kh,kh,Cin] fp32 -> [B,OH,OW,Cout]."""
    xh, xl = _split(x)
    wh, wl = _split(w)

    def conv(a, b):
        y = torch.nn.functional.conv2d(a.double().permute(0, 3, 1, 2), b.double().permute(0, 3, 1, 2), stride=stride)
        return y.permute(0, 2, 3, 1)
    return conv(xh, wh) + conv(xl, wh) + conv(xh, wl), conv(x, w)


def _gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / 2 ** 0.5))


@pytest.mark.parametrize("b,h,cin,cout,kh,stride,tile", [
    (2, 13, 96, 384, 1, 1, -1), (3, 9, 96, 96, 1, 1, -1), (2, 11, 192, 192, 1, 1, 4), (2, 11, 192, 192, 1, 1, 0),
    (1, 7, 384, 1536, 1, 1, 5), (2, 7, 768, 256, 1, 1, -1), (4, 28, 96, 192, 2, 2, -1), (2, 27, 192, 384, 2, 1, -1),
    (2, 13, 384, 768, 2, 1, 5), (3, 10, 128, 136, 1, 1, -1), (2, 13, 384, 384, 1, 1, 7), (1, 11, 192, 192, 1, 1, 7),
    (2, 27, 192, 384, 2, 1, 7), (2, 9, 96, 200, 1, 1, 7)])
@pytest.mark.parametrize("epi", ["f32_bias", "f32_resid", "s3_gelu"])
def test_conv_s3_matches_split_product(gpu, b, h, cin, cout, kh, stride, tile, epi):
    g = torch.Generator().manual_seed(b * 1000 + h * 10 + kh)
    x = torch.randn(b, h, h, cin, generator=g)
    w = torch.randn(cout, kh, kh, cin, generator=g) * (kh * kh * cin) ** -0.5
    bias = torch.randn(cout, generator=g) * 0.1
    emu, exact = _emulated(x, w, kh, stride)
    emu, exact = emu + bias.double(), exact + bias.double()
    x3 = K.split_planes(x.to(gpu))
    wp = K.split_planes_weight(w.to(gpu))
    code = {"f32_bias": _lib.EPI_F32_BIAS, "f32_resid": _lib.EPI_F32_RESID, "s3_gelu": _lib.EPI_S3_GELU}[epi]
    if epi == "f32_resid":
        scale = torch.rand(cout, generator=g) + 0.5
        r = torch.randn(emu.shape, generator=g, dtype=torch.float32)
        rd = r.to(gpu)
        y = K.conv_s3(x3, wp, kh, kh, cout, bias.to(gpu), stride, 0, code, scale=scale.to(gpu), r=rd, out=rd, tile=tile)
        emu = r.double() + scale.double() * emu
        exact = r.double() + scale.double() * exact
        got = y.cpu().double()
    elif epi == "s3_gelu":
        y = K.conv_s3(x3, wp, kh, kh, cout, bias.to(gpu), stride, 0, code, tile=tile).cpu()
        hi, lo = y[..., :cout], y[..., cout:]
        got = hi.double() + lo.double()
        # the split of the kernel's fp32 value: hi = RNE(v), |lo| <= ulp_bf16(v) / 2
        assert torch.all(lo.double().abs() <= hi.double().abs() * 2.0 ** -8 + 1e-30)
        emu, exact = _gelu64(emu), _gelu64(exact)
    else:
        got = K.conv_s3(x3, wp, kh, kh, cout, bias.to(gpu), stride, 0, code, tile=tile).cpu().double()
    torch.cuda.synchronize()
    scale_ = exact.abs().max().item()
    # s3_gelu: gelu_pk16 (|error| < 1e-6 absolute) and the split storage of the output
    # itself (hi + lo carries v to half an ulp of lo: <= 2^-16 |v|)
    tol = (2e-6 + emu.abs() * 2.0 ** -16) if epi == "s3_gelu" else 0.0
    assert torch.all((got - emu).abs() <= 2e-6 * scale_ + tol)
    assert torch.all((got - exact).abs() <= 3e-5 * scale_ + tol)


@pytest.mark.parametrize("b,h,c", [(2, 9, 96), (1, 8, 192), (2, 7, 384), (1, 6, 768), (2, 24, 96), (1, 12, 192)])
def test_dwconv7_ln_s3_is_split_of_fp32_kernel(gpu, b, h, c):
    g = torch.Generator().manual_seed(c + h)
    x = torch.randn(b, h, h, c, generator=g).to(gpu)
    wdw = (torch.randn(49, c, generator=g) * 0.1).to(gpu)
    bias, lw, lb = (torch.randn(c, generator=g).to(gpu) for _ in range(3))
    y = K.dwconv7_ln(x, wdw, bias, lw, lb)
    y3 = K.dwconv7_ln_s3(x, wdw, bias, lw, lb)
    torch.cuda.synchronize()
    assert torch.equal(y3, K.split_planes(y))


@pytest.mark.parametrize("rows,c", [(37, 96), (64, 192), (5, 384), (3, 768)])
def test_layernorm_s3_is_split_of_fp32_kernel(gpu, rows, c):
    g = torch.Generator().manual_seed(rows * c)
    x = torch.randn(rows, c, generator=g).to(gpu)
    w, b = torch.randn(c, generator=g).to(gpu), torch.randn(c, generator=g).to(gpu)
    y = K.layernorm(x, w, b)
    y3 = K.layernorm_s3(x, w, b)
    torch.cuda.synchronize()
    assert torch.equal(y3, K.split_planes(y))


def test_conv_s3_rejects_bad_arguments(gpu):
    x3 = torch.zeros(1, 4, 4, 2 * 40, device=gpu, dtype=torch.bfloat16)      # Cin = 40: not % 32
    wp = K.split_planes_weight(torch.zeros(64, 1, 1, 40, device=gpu))
    with pytest.raises(RuntimeError):
        K.conv_s3(x3, wp, 1, 1, 64, None, 1, 0, _lib.EPI_F32_BIAS)
    x3 = torch.zeros(1, 4, 4, 64, device=gpu, dtype=torch.bfloat16)
    wp = K.split_planes_weight(torch.zeros(64, 1, 1, 32, device=gpu))
    with pytest.raises(RuntimeError):                                          # resid without r / scale
        K.conv_s3(x3, wp, 1, 1, 64, None, 1, 0, _lib.EPI_F32_RESID)
    with pytest.raises(RuntimeError):                                          # tile 2 has no split epilogue
        K.conv_s3(x3, wp, 1, 1, 64, None, 1, 0, _lib.EPI_F32_BIAS, tile=2)
