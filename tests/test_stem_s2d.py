"""Space-to-depth form of the ResNet stem (resnet_features.py:161-163: Conv2d(3, 64, k7, s2, p3)),
used by the bf16 HIP path (resnet_hip.py, csrc/conv_bf16.hip pipnet_nchw_to_s2d_bf16): the
relayout restated on the CPU and the regrouped weights (kernels.stem_weight_s2d) must give the
7x7 stride-2 conv exactly as a 4x4 stride-1 conv -- checked in fp64 against F.conv2d."""
import pytest
import torch
import torch.nn.functional as F

from count_pipnet_amd import kernels as K


def s2d_reference(x: torch.Tensor) -> torch.Tensor:
    """[B,3,H,W] -> [B, SH, SW, 16], q = (2 bi + bj) * 4 + c, pixel (i, j) <- x[2(i-2)+bi, 2(j-2)+bj]."""
    b, c, h, w = x.shape
    sh, sw = (h - 1) // 2 + 4, (w - 1) // 2 + 4
    xp = torch.zeros(b, c, 2 * sh + 4, 2 * sw + 4, dtype=x.dtype)
    xp[:, :, 4:4 + h, 4:4 + w] = x
    xp = xp[:, :, :2 * sh, :2 * sw]
    s = xp.reshape(b, c, sh, 2, sw, 2).permute(0, 2, 4, 3, 5, 1)           # [B, SH, SW, bi, bj, c]
    return F.pad(s, (0, 1)).reshape(b, sh, sw, 16)


@pytest.mark.parametrize("h,w", [(224, 224), (37, 30), (17, 19), (8, 9)])
def test_stem_as_4x4_conv_on_s2d(h, w):
    g = torch.Generator().manual_seed(h * 100 + w)
    x = torch.randn(2, 3, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(64, 3, 7, 7, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, wt, stride=2, padding=3)
    ws = K.stem_weight_s2d(wt.permute(0, 2, 3, 1))                         # [64, 4, 4, 16]
    out = F.conv2d(s2d_reference(x).permute(0, 3, 1, 2), ws.permute(0, 3, 1, 2))
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-12), (out - ref).abs().max()
