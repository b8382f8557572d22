"""ORACLE -- CPU restatement of the reference's evaluation input transform.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench``
baselines may import this module, and only as the checker -- never as the product path
(the product path is ``pipnet_resize_normalize_rgb8`` in ``count_pipnet_amd/csrc/input_ops.hip``).

The reference evaluates on ``transform_no_augment`` (util/data.py:264-269 pets, :314-321
shapes, :500-505 CUB-200-2011, :537-542 CARS, :568-574 grayscale):

    transforms.Compose([transforms.Resize(size=(img_size, img_size)),
                        (transforms.Grayscale(3),)            # get_grayscale only
                        transforms.ToTensor(), normalize])

applied by ``torchvision.datasets.ImageFolder`` to ``Image.open(path).convert('RGB')``.
The arithmetic is third party: torchvision (absent here, version unpinned -- README.md:14
says PyTorch 1.13, i.e. torchvision ~0.14) forwards a PIL image's Resize to
``PIL.Image.resize(size[::-1], Resampling.BILINEAR)``, so the numbers are Pillow's
(``libImaging/Resample.c``; this image ships Pillow 12.2.0).  Restated here:

* ``precompute_coeffs``: per output coordinate xx, ``center = in0 + (xx + 0.5) * scale``,
  ``support = 1.0 * max(scale, 1)``, taps ``xmin = int(center - support + 0.5)`` (clamped to
  0) .. ``xmax = int(center + support + 0.5)`` (clamped to the input size), weights
  ``triangle((x + xmin - center + 0.5) / max(scale, 1))`` normalised to sum 1, all in double;
* ``normalize_coeffs_8bpc``: weights -> int32 fixed point with 22 fractional bits
  (``PRECISION_BITS = 32 - 8 - 2``), rounding half away from zero;
* horizontal pass first (only over the input rows the vertical pass uses), then the
  vertical pass, each ``clip8((1 << 21) + sum(pixel * k) >> 22)`` to uint8 -- except for
  very tall images that shrink vertically (``h > 100 * w`` and ``out_h < h``), where Pillow 12 runs the vertical pass first (only
  over the input columns the horizontal pass uses; found by probing, see
  ``tests/test_input_oracle.py``);
* a pass is skipped when that axis keeps its size.

Then ``ToTensor`` (``img.permute(2, 0, 1).float().div(255)``) and ``Normalize``
(``(t - mean[:, None, None]) / std[:, None, None]`` in float32); ``Grayscale(3)`` is
``convert('L')`` = ``(R*19595 + G*38470 + B*7471 + 0x8000) >> 16`` replicated to 3 bands.

Pinned against Pillow itself: ``tests/golden/gen_golden_input.py`` records Pillow's
outputs for seeded images of many sizes (``tests/golden/input_resize.npz``).
"""
from __future__ import annotations

import math

import numpy as np
import torch

PRECISION_BITS = 32 - 8 - 2
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _triangle(x: float) -> float:
    x = abs(x)
    return 1.0 - x if x < 1.0 else 0.0


def precompute_coeffs(in_size: int, out_size: int):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc for the BILINEAR filter (support 1).

    Returns (bounds [out_size, 2] = (xmin, count), kk [out_size, ksize] int64 fixed point)."""
    in0, in1 = 0.0, float(in_size)
    scale = (in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = in0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = int(center - support + 0.5)      # C (int) truncation toward zero
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        xmax -= xmin
        w = [_triangle((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        for x, v in enumerate(w):
            f = v * (1 << PRECISION_BITS)
            kk[xx, x] = int(-0.5 + f) if v < 0 else int(0.5 + f)
        bounds[xx] = (xmin, xmax)
    return bounds, kk


def _clip8(ss: np.ndarray) -> np.ndarray:
    return np.clip(ss >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One resample pass over `axis` (1 = horizontal, 0 = vertical) of an HxWxC uint8 image."""
    src = np.moveaxis(img.astype(np.int64), axis, 0)           # taps along dim 0
    out = np.empty((bounds.shape[0],) + src.shape[1:], np.uint8)
    for o, (xmin, cnt) in enumerate(bounds):
        ss = np.full(src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
        for t in range(cnt):
            ss += src[xmin + t] * kk[o, t]
        out[o] = _clip8(ss)
    return np.moveaxis(out, 0, axis)


def pil_resize_bilinear(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """Pillow ImagingResample(BILINEAR) of an HxWx3 uint8 RGB image -> out_h x out_w x 3."""
    h, w = img.shape[:2]
    if (h, w) == (out_h, out_w):
        return img.copy()
    bh, kh = precompute_coeffs(w, out_w)
    bv, kv = precompute_coeffs(h, out_h)
    cur = img
    if vertical_first(h, w, out_h) and w != out_w and h != out_h:
        x0 = int(bh[0, 0])
        x1 = int(bh[-1, 0] + bh[-1, 1])
        cur = _pass(img[:, x0:x1], bv, kv, axis=0)             # only the columns the horizontal pass reads
        bh = bh.copy()
        bh[:, 0] -= x0
        return _pass(cur, bh, kh, axis=1)
    if w != out_w:
        y0 = int(bv[0, 0])
        y1 = int(bv[-1, 0] + bv[-1, 1])
        cur = _pass(img[y0:y1], bh, kh, axis=1)                # only the rows the vertical pass reads
        bv = bv.copy()
        bv[:, 0] -= y0
    if h != out_h:
        cur = _pass(cur, bv, kv, axis=0)
    return cur


def vertical_first(h: int, w: int, out_h: int) -> bool:
    """Pillow 12 resamples very tall images that shrink vertically pass-V-first (probed rule)."""
    return h > 100 * w and out_h < h


def grayscale3(img: np.ndarray) -> np.ndarray:
    """PIL convert('L') (ITU-R 601-2 luma, 16-bit fixed point) replicated to 3 bands."""
    x = img.astype(np.int64)
    l = (x[..., 0] * 19595 + x[..., 1] * 38470 + x[..., 2] * 7471 + 0x8000) >> 16
    return np.repeat(l.astype(np.uint8)[..., None], 3, axis=2)


def to_tensor_normalize(img: np.ndarray, mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    """torchvision ToTensor + Normalize on an HxWx3 uint8 image -> [3,H,W] float32."""
    t = torch.from_numpy(np.array(img, dtype=np.uint8, copy=True)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32)[:, None, None]
    s = torch.as_tensor(std, dtype=torch.float32)[:, None, None]
    return t.sub(m).div(s)


def eval_transform(img: np.ndarray, size, grayscale: bool = False, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """transform_no_augment of util/data.py on a decoded RGB image -> ([3,h,w] fp32, resized uint8)."""
    r = pil_resize_bilinear(img, size[0], size[1])
    if grayscale:
        r = grayscale3(r)
    return to_tensor_normalize(r, mean, std), r
