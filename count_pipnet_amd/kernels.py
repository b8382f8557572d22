"""Tensor-level wrappers over the C-ABI (one function per HIP entry point).

Every wrapper validates device / dtype / contiguity, allocates its outputs on the input's
device and enqueues on torch's *current* HIP stream, so the calls compose with torch
streams, events and graph capture.  Nothing here computes on the host.
"""
from __future__ import annotations

import functools

from typing import Optional, Tuple

import os

import torch

from . import _lib

Tensor = torch.Tensor


# Optional instrumentation: hook(kernel_name, algorithmic_flops, launch_fn) wraps every MFMA
# GEMM launch (bench.py brackets them with HIP events on the launching stream).
_launch_hook = None


def set_launch_hook(hook) -> None:
    global _launch_hook
    _launch_hook = hook


def _launch(kname: str, flops: float, fn) -> None:
    if _launch_hook is None:
        fn()
    else:
        _launch_hook(kname, flops, fn)


@functools.lru_cache(maxsize=4096)
def gemm_variant(m: int, n: int, k: int, epilogue: int = _lib.EPI_NONE, aload: int = 0) -> int:
    """The fp32 GEMM variant the library launches for an m x n x k product (pipnet_linear_f32_plan:
    the library's own rule, csrc/gemm_f32.hip gemm_variant -- never mirrored here)."""
    v = _lib.load().pipnet_linear_f32_plan(m, n, k, epilogue, aload)
    if v < 0:
        raise RuntimeError(f"linear: no GEMM variant for {m} x {n} x {k} (epilogue {epilogue}, aload {aload})")
    return v


def gemm_kernel_name(m: int, n: int, k: int, epilogue: int, aload: int) -> str:
    """The rocprof name of the GEMM instantiation the library picks (dense, unit-stride, 16-B
    aligned torch operands -- so ``vec_epi`` holds whenever N % 4 == 0)."""
    v = gemm_variant(m, n, k, epilogue, aload)
    if v == 1:
        return f"pipnet_gemm::gemm_f32_tn_kernel<16, 2, {epilogue}, {aload}, 2, 3, 0, false>"
    if v == 0:
        return f"pipnet_gemm::gemm_f32_tn_ktail_kernel<{epilogue}, {aload}>"
    if v == 5:
        return f"pipnet_gemm::gemm_f32_tnw_kernel<{epilogue}, {aload}, 0>"
    if v == 3:
        return f"pipnet_gemm::gemm_f32_tn_kernel<32, 2, {epilogue}, {aload}, 2, 2, 0, false>"
    npad = "true" if n % 128 else "false"      # padded-column MFMA blocks skipped
    return f"pipnet_gemm::gemm_f32_tn_kernel<32, 1, {epilogue}, {aload}, 3, 2, 0, {npad}>"


_CUS = {}


def _num_cus() -> int:
    """CUs of the current device (per device, as the library's launch rule sees it)."""
    if not torch.cuda.is_available():
        return 256
    d = torch.cuda.current_device()
    if d not in _CUS:
        _CUS[d] = torch.cuda.get_device_properties(d).multi_processor_count
    return _CUS[d]


SPLITK_WG_PER_CU = int(os.environ.get("PIPNET_SPLITK_WG_PER_CU", "2"))   # env: A/B runs (tools)
SPLITK_MIN_K = int(os.environ.get("PIPNET_SPLITK_MIN_K", "256"))          # env: A/B runs (tools)


def splitk_factor(m: int, n: int, k: int, cus: int = 256) -> int:
    """K slabs for short-M GEMMs, which stream their weights once (C5's Bilinear intermediate
    at M = batch: 48 tiles of 64 x 128 over 151 MB of W / V): enough workgroups for
    SPLITK_WG_PER_CU per CU -- about 100 KB of LDS-DMA in flight per CU, what HBM latency
    needs -- each slab >= 8 K-tiles of 32."""
    if n % 4 or k % 32 or m > 512:     # backbone GEMMs (M = pixels) stay batch-invariant
        return 1
    tiles = -(-m // 64) * -(-n // 128)
    if tiles >= cus:
        return 1
    return max(1, min(-(-SPLITK_WG_PER_CU * cus // tiles), k // SPLITK_MIN_K, 64))


def _ptr(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(t: Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def require_device(t: Tensor, what: str = "input") -> None:
    if not (t.is_cuda and t.dtype == torch.float32):
        raise RuntimeError(
            f"count_pipnet_amd: the HIP inference path needs a float32 ROCm device tensor for {what} "
            f"(got device={t.device}, dtype={t.dtype}); there is no CPU fallback. Move the model and "
            "inputs to a GPU, or run the autograd path (train mode / grad enabled).")


def _chk(t: Tensor, what: str, contiguous: bool = True) -> None:
    require_device(t, what)
    if contiguous and not t.is_contiguous():
        raise RuntimeError(f"count_pipnet_amd: {what} must be contiguous")


def linear(a: Tensor, w: Tensor, bias: Optional[Tensor] = None, epilogue: int = _lib.EPI_NONE,
           scale: Optional[Tensor] = None, r: Optional[Tensor] = None, out: Optional[Tensor] = None) -> Tensor:
    """out[M,N] = epi(a[M,K] @ w[N,K]^T).  a may be any 2-D row-major view with unit col stride."""
    require_device(a, "linear input")
    _chk(w, "weight")
    if a.dim() != 2 or w.dim() != 2 or a.stride(1) != 1:
        raise RuntimeError("linear: expects 2-D operands with unit column stride")
    m, k = a.shape
    n = w.shape[0]
    if w.shape[1] != k:
        raise RuntimeError(f"linear: K mismatch {tuple(a.shape)} x {tuple(w.shape)}")
    if out is None:
        out = torch.empty((m, n), device=a.device, dtype=torch.float32)
    ldr = r.stride(0) if r is not None else 0
    splits = splitk_factor(m, n, k)
    if splits > 1:
        ws = torch.empty((splits, m, n), device=a.device, dtype=torch.float32)
        _launch(f"pipnet_gemm::gemm_f32_tn_kernel<32, 1, 0, 0, 3, 2, 0, false>", 2.0 * m * n * k,
                lambda: _lib.call("pipnet_linear_splitk_f32", a.data_ptr(), a.stride(0), w.data_ptr(), _ptr(bias),
                                  _ptr(scale), _ptr(r), ldr, out.data_ptr(), out.stride(0), m, n, k, epilogue, splits,
                                  ws.data_ptr(), _stream(a)))
        return out
    _launch(gemm_kernel_name(m, n, k, epilogue, 0), 2.0 * m * n * k,
            lambda: _lib.call("pipnet_linear_f32", a.data_ptr(), a.stride(0), w.data_ptr(), _ptr(bias), _ptr(scale),
                              _ptr(r), ldr, out.data_ptr(), out.stride(0), m, n, k, epilogue, _stream(a)))
    return out


def linear_pair_mul(a: Tensor, w_pair: Tensor) -> Tensor:
    """(a @ w_pair[Nh:]^T) * (a @ w_pair[:Nh]^T) for a [M,K] and w_pair [2 Nh, K] (the stacked
    folded BilinearIntermediate weights) as ONE split-K GEMM + one reduction that takes the product
    (include/pipnet_amd.h pipnet_linear_pair_mul_f32)."""
    require_device(a, "linear input")
    _chk(w_pair, "paired weight")
    m, k = a.shape
    n2 = w_pair.shape[0]
    if a.stride(1) != 1 or w_pair.shape[1] != k or n2 % 2:
        raise RuntimeError(f"linear_pair_mul: shapes {tuple(a.shape)} x {tuple(w_pair.shape)}")
    nh = n2 // 2
    splits = max(1, splitk_factor(m, n2, k))
    out = torch.empty((m, nh), device=a.device, dtype=torch.float32)
    ws = torch.empty((splits, m, n2), device=a.device, dtype=torch.float32)
    _launch("pipnet_gemm::gemm_f32_tn_kernel<32, 1, 0, 0, 3, 2, 0, false>", 2.0 * m * n2 * k,
            lambda: _lib.call("pipnet_linear_pair_mul_f32", a.data_ptr(), a.stride(0), w_pair.data_ptr(),
                              out.data_ptr(), out.stride(0), m, nh, k, splits, ws.data_ptr(), _stream(a)))
    return out


def matmul_f64acc(a: Tensor, b: Tensor) -> Tensor:
    """[M,K] @ [K,N] (row-major fp32) with fp64 products and sums, rounded once to fp32
    (include/pipnet_amd.h pipnet_matmul_f64acc_f32): the inference-time weight folds."""
    _chk(a, "fold operand A")
    _chk(b, "fold operand B")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[0]:
        raise RuntimeError(f"matmul_f64acc: shapes {tuple(a.shape)} x {tuple(b.shape)}")
    m, k = a.shape
    n = b.shape[1]
    out = torch.empty((m, n), device=a.device, dtype=torch.float32)
    _lib.call("pipnet_matmul_f64acc_f32", a.data_ptr(), k, b.data_ptr(), n, out.data_ptr(), n, m, n, k, _stream(a))
    return out


def matmul2_f64acc(a0: Tensor, a1: Tensor, b: Tensor) -> Tensor:
    """torch.stack((a0 @ b, a1 @ b)) ([2, M, N]) as ``matmul_f64acc`` in ONE launch
    (pipnet_matmul2_f64acc_f32): the bilinear fold's W.E and V.E share the embedding operand."""
    for t, what in ((a0, "fold operand A0"), (a1, "fold operand A1"), (b, "fold operand B")):
        _chk(t, what)
    if a0.dim() != 2 or a0.shape != a1.shape or b.dim() != 2 or a0.shape[1] != b.shape[0]:
        raise RuntimeError(f"matmul2_f64acc: shapes {tuple(a0.shape)}, {tuple(a1.shape)} x {tuple(b.shape)}")
    m, k = a0.shape
    n = b.shape[1]
    out = torch.empty((2, m, n), device=a0.device, dtype=torch.float32)
    _lib.call("pipnet_matmul2_f64acc_f32", a0.data_ptr(), a1.data_ptr(), k, b.data_ptr(), n, out[0].data_ptr(),
              out[1].data_ptr(), n, m, n, k, _stream(a0))
    return out


def linear_rowscale(a: Tensor, w: Tensor, bias: Optional[Tensor], scale: Tensor, r: Tensor, row_scale: Tensor,
                    rows_per_scale: int) -> Tensor:
    """In place on ``r`` ([M,N]): r = r + row_scale[m // rows_per_scale] * (scale * (a w^T + bias))
    (CNBlock Linear2 under train-mode stochastic depth)."""
    require_device(a, "linear input")
    _chk(w, "weight")
    _chk(row_scale, "row scale")
    m, k = a.shape
    n = w.shape[0]
    if w.shape[1] != k or tuple(r.shape) != (m, n) or a.stride(1) != 1 or r.stride(1) != 1:
        raise RuntimeError(f"linear_rowscale: shapes a {tuple(a.shape)}, w {tuple(w.shape)}, r {tuple(r.shape)}")
    if row_scale.numel() * rows_per_scale < m:
        raise RuntimeError("linear_rowscale: row_scale does not cover every row")
    _launch(gemm_kernel_name(m, n, k, _lib.EPI_RESID_ROWSCALE, 0), 2.0 * m * n * k,
            lambda: _lib.call("pipnet_linear_rowscale_f32", a.data_ptr(), a.stride(0), w.data_ptr(), _ptr(bias),
                              _ptr(scale), r.data_ptr(), r.stride(0), r.data_ptr(), r.stride(0), m, n, k,
                              row_scale.data_ptr(), rows_per_scale, _stream(a)))
    return r


def conv2x2(x_nhwc: Tensor, w_packed: Tensor, bias: Optional[Tensor], stride: int) -> Tensor:
    _chk(x_nhwc, "conv2x2 input")
    b, h, w, cin = x_nhwc.shape
    cout = w_packed.shape[0]
    oh, ow = (h - 2) // stride + 1, (w - 2) // stride + 1
    y = torch.empty((b, oh, ow, cout), device=x_nhwc.device, dtype=torch.float32)
    epi = _lib.EPI_BIAS if bias is not None else _lib.EPI_NONE
    _launch(gemm_kernel_name(b * oh * ow, cout, 4 * cin, epi, 1), 2.0 * b * oh * ow * cout * 4 * cin,
            lambda: _lib.call("pipnet_conv2x2_f32", x_nhwc.data_ptr(), b, h, w, cin, w_packed.data_ptr(), _ptr(bias),
                              cout, stride, y.data_ptr(), _stream(x_nhwc)))
    return y


def conv2d_nhwc(x: Tensor, w_packed: Tensor, bias: Optional[Tensor], stride: int, pad: int,
                epilogue: int = _lib.EPI_BIAS, r: Optional[Tensor] = None) -> Tensor:
    """NHWC implicit-GEMM convolution; w_packed [Cout, KH, KW, Cin]; r = residual (NHWC)."""
    _chk(x, "conv input")
    _chk(w_packed, "conv weight")
    b, h, w, cin = x.shape
    cout, kh, kw, wcin = w_packed.shape
    if wcin != cin:
        raise RuntimeError(f"conv2d_nhwc: input has {cin} channels, weight {wcin}")
    oh, ow = (h + 2 * pad - kh) // stride + 1, (w + 2 * pad - kw) // stride + 1
    y = torch.empty((b, oh, ow, cout), device=x.device, dtype=torch.float32)
    m, k = b * oh * ow, kh * kw * cin
    aload = 0 if (kh == 1 and kw == 1 and stride == 1 and pad == 0) else 2
    _launch(gemm_kernel_name(m, cout, k, epilogue, aload), 2.0 * m * cout * k,
            lambda: _lib.call("pipnet_conv2d_nhwc_f32", x.data_ptr(), b, h, w, cin, w_packed.data_ptr(), _ptr(bias),
                              cout, kh, kw, stride, pad, _ptr(r), epilogue, y.data_ptr(), _stream(x)))
    return y


def maxpool2d_nhwc(x: Tensor, k: int, stride: int, pad: int) -> Tensor:
    _chk(x, "maxpool input")
    b, h, w, c = x.shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    y = torch.empty((b, oh, ow, c), device=x.device, dtype=torch.float32)
    _lib.call("pipnet_maxpool2d_nhwc_f32", x.data_ptr(), b, h, w, c, k, stride, pad, y.data_ptr(), _stream(x))
    return y


def nchw_to_nhwc(x: Tensor, cpad: int) -> Tensor:
    _chk(x, "network input (NCHW)")
    b, c, h, w = x.shape
    y = torch.empty((b, h, w, cpad), device=x.device, dtype=torch.float32)
    _lib.call("pipnet_nchw_to_nhwc_f32", x.data_ptr(), b, c, h, w, cpad, y.data_ptr(), _stream(x))
    return y


# ---- bf16 ResNet path (BASELINE C3) ---------------------------------------------------

BF16_KTILE = 64


def _chk_bf(t: Tensor, what: str) -> None:
    if not (t.is_cuda and t.dtype == torch.bfloat16):
        raise RuntimeError(f"count_pipnet_amd: {what} must be a bfloat16 ROCm device tensor "
                           f"(got device={t.device}, dtype={t.dtype}); there is no CPU fallback")
    if not t.is_contiguous():
        raise RuntimeError(f"count_pipnet_amd: {what} must be contiguous")


@functools.lru_cache(maxsize=4096)
def bf16_conv_plan(b: int, h: int, w: int, cin: int, cout: int, kh: int, kw: int, stride: int, pad: int,
                   epilogue: int, tile: int = -1) -> int:
    """The workgroup tile the library takes for this bf16 conv (pipnet_conv2d_nhwc_bf16_plan: the
    library's own rule, csrc/conv_bf16.hip plan_conv -- never mirrored here):
    9 = the persistent ping-pong tile (1x1 stride-1 convs with N % 256 == 0, plain epilogues),
    11 = 3x3 stride-1 pad-1 Cin = N = 64 (W <= 63) / 128 (W <= 31) convs on an LDS input halo,
    8 = the ping-pong tile with an LDS input halo (3x3 stride-1 pad-1, Cin % 64 == 0, W <= 31, N >= 256),
    5 = 256x256 ping-pong on 16x16x32 MFMAs, 6 = 256x64 (N <= 64), 0 = 64x128, 3 = 256x256,
    4 = 128x128.  ``tile`` >= 0 is validated instead of chosen."""
    v = _lib.load().pipnet_conv2d_nhwc_bf16_plan(b, h, w, cin, cout, kh, kw, stride, pad, epilogue, tile)
    if v < 0:
        raise RuntimeError(f"conv2d_nhwc_bf16: no tile {tile} for {b}x{h}x{w}x{cin} -> {cout} k{kh}x{kw} s{stride} "
                           f"p{pad} epilogue {epilogue}")
    return v


def s3_conv_tile(m: int, n: int, pp_ok: bool = True, kv: int = 0) -> int:
    """Tile of a split-bf16 GEMM (csrc/conv_bf16.hip conv_variant's s3 branch; tiles 0 / 4 / 5 / 7).
    The split path's labels only -- the ResNet bf16 convs ask the library (bf16_conv_plan)."""
    m128 = 4 if -(-m // 128) * -(-n // 128) >= 512 else 0
    if not pp_ok:
        return m128
    if n == 192:
        return 7
    if n == 384:
        return 7 if kv >= 3 * 1024 else m128
    return 5 if n >= 256 else m128


_BF16_CFG = {0: ("pipnet_bf16::Cfg<2, 2, 1, 2, 32, 4>", 3), 1: ("pipnet_bf16::Cfg<2, 2, 2, 2, 64, 2>", 2),
             2: ("pipnet_bf16::Cfg<2, 4, 4, 2, 64, 2>", 1), 3: ("pipnet_bf16::Cfg<2, 4, 4, 2, 32, 4>", 1),
             4: ("pipnet_bf16::Cfg<2, 2, 2, 2, 32, 4>", 2), 6: ("pipnet_bf16::Cfg<4, 1, 2, 2, 32, 4>", 2)}


PP_RB = 8     # row blocks of the 256-wide ping-pong tiles (csrc/conv_bf16.hip PP_RB): 256-row tiles


def bf16_conv_kernel_name(m: int, n: int, epilogue: int, aload: int, tile: int, s3: bool = False,
                          kv: int = 0) -> str:
    """rocprof name of the bf16 conv instantiation of ``tile`` (bf16_conv_plan / s3_conv_tile)."""
    t = tile
    if t == 11:
        return f"pipnet_bf16::conv3x3_bf16_hsmall_kernel<{kv // 9}, {epilogue}>"
    if t == 9:
        return f"pipnet_bf16::conv_bf16_ppp_kernel<{epilogue}, {PP_RB}>"
    if t == 8:
        nb = 4 if n >= 256 else (2 if n >= 128 else 1)
        return f"pipnet_bf16::conv3x3_bf16_halo_kernel<{epilogue}, {nb}, {PP_RB}>"
    if t == 5:
        return f"pipnet_bf16::conv_bf16_pp_kernel<{epilogue}, {aload}, 4, 0, 2>"
    if t == 7:
        return f"pipnet_bf16::conv_bf16_pp_kernel<{epilogue}, {aload}, 3, 0, 2>"
    cfg, minb = _BF16_CFG[t]
    npad = "true" if s3 and t == 4 and n % 128 else "false"     # padded-column MFMA blocks skipped
    return f"pipnet_bf16::conv_bf16_kernel<{cfg}, {epilogue}, {aload}, {minb}, {npad}>"


def pack_conv_weight_bf16(w_ohwi: Tensor) -> Tensor:
    """[Cout, KH, KW, Cin] (fp32) -> [Cout, Kp] bf16, Kp = KH*KW*Cin rounded up to 64 (zeros)."""
    cout = w_ohwi.shape[0]
    k = w_ohwi[0].numel()
    kp = -(-k // BF16_KTILE) * BF16_KTILE
    out = torch.zeros((cout, kp), device=w_ohwi.device, dtype=torch.bfloat16)
    out[:, :k] = w_ohwi.reshape(cout, k).to(torch.bfloat16)
    return out


# Tile 11 (3x3 Cin = N = 64 / 128 on the LDS input halo) for automatic launches; False = the generic
# tile (6 / 4 / 0: bitwise the same outputs) (in-process A/B: tools/ab_toggle.py count_pipnet_amd.kernels.CONV3X3_N64_HALO c3)
CONV3X3_N64_HALO = True


def conv2d_nhwc_bf16(x: Tensor, w_packed: Tensor, kh: int, kw: int, bias: Optional[Tensor], stride: int,
                     pad: int, epilogue: int = _lib.EPI_BIAS, r: Optional[Tensor] = None, tile: int = -1) -> Tensor:
    """NHWC bf16 implicit-GEMM convolution; w_packed from pack_conv_weight_bf16; bias fp32;
    tile -1 = automatic, 0 = 64x128 (32-deep K, 4 stages), 1/2 = 128x128 / 256x256 (64-deep K,
    2 stages), 3/4 = 256x256 / 128x128 (32-deep K, 4 stages), 5 = 256x256 ping-pong, 6 = 256x64,
    8 = ping-pong with the LDS input halo (3x3 stride-1 pad-1 only), 9 = persistent ping-pong
    (1x1 stride-1, N % 256 == 0), 11 = 3x3 stride-1 pad-1 N = 64 on an LDS input halo."""
    _chk_bf(x, "conv input")
    _chk_bf(w_packed, "conv weight")
    if r is not None:
        _chk_bf(r, "residual")
    if bias is not None:
        _chk(bias, "conv bias")
    b, h, w, cin = x.shape
    cout, kp = w_packed.shape
    k = kh * kw * cin
    if kp != -(-k // BF16_KTILE) * BF16_KTILE:
        raise RuntimeError(f"conv2d_nhwc_bf16: packed weight K {kp} does not match {kh}x{kw}x{cin}")
    oh, ow = (h + 2 * pad - kh) // stride + 1, (w + 2 * pad - kw) // stride + 1
    y = torch.empty((b, oh, ow, cout), device=x.device, dtype=torch.bfloat16)
    m = b * oh * ow
    aload = 0 if (kh == 1 and kw == 1 and stride == 1 and pad == 0) else 2
    if tile < 0 and not CONV3X3_N64_HALO and bf16_conv_plan(b, h, w, cin, cout, kh, kw, stride, pad, epilogue) == 11:
        tile = 6 if cout == 64 else 4       # the same arithmetic on the generic tile (A/B arm)
    t = bf16_conv_plan(b, h, w, cin, cout, kh, kw, stride, pad, epilogue, tile)
    _launch(bf16_conv_kernel_name(m, cout, epilogue, aload, t, kv=k),
            2.0 * m * cout * k,
            lambda: _lib.call("pipnet_conv2d_nhwc_bf16_tile", x.data_ptr(), b, h, w, cin, w_packed.data_ptr(),
                              _ptr(bias), cout, kh, kw, stride, pad, _ptr(r), epilogue, y.data_ptr(), tile,
                              _stream(x)))
    return y


def stem_pool_bf16(s2d: Tensor, w_packed: Tensor, bias: Tensor) -> Tensor:
    """ResNet stem over the space-to-depth image (4x4 stride 1, 16 -> 64, + bias + ReLU) fused
    with MaxPool2d(3, 2, 1) (pipnet_stem_pool_bf16): bitwise conv2d_nhwc_bf16 + maxpool2d_nhwc_bf16."""
    _chk_bf(s2d, "stem s2d input")
    _chk_bf(w_packed, "stem weight")
    _chk(bias, "stem bias")
    b, sh, sw, c = s2d.shape
    if c != 16 or tuple(w_packed.shape) != (64, 256):
        raise RuntimeError(f"stem_pool_bf16: expects a 16-channel s2d image and a [64, 256] weight, got "
                           f"{tuple(s2d.shape)} / {tuple(w_packed.shape)}")
    ph, pw = (sh - 4) // 2 + 1, (sw - 4) // 2 + 1
    y = torch.empty((b, ph, pw, 64), device=s2d.device, dtype=torch.bfloat16)
    _launch("pipnet_bf16::stem_pool_bf16_kernel", 2.0 * b * (sh - 3) * (sw - 3) * 64 * 256,
            lambda: _lib.call("pipnet_stem_pool_bf16", s2d.data_ptr(), b, sh, sw, w_packed.data_ptr(),
                              bias.data_ptr(), y.data_ptr(), _stream(s2d)))
    return y


def maxpool2d_nhwc_bf16(x: Tensor, k: int, stride: int, pad: int) -> Tensor:
    _chk_bf(x, "maxpool input")
    b, h, w, c = x.shape
    oh, ow = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
    y = torch.empty((b, oh, ow, c), device=x.device, dtype=torch.bfloat16)
    _lib.call("pipnet_maxpool2d_nhwc_bf16", x.data_ptr(), b, h, w, c, k, stride, pad, y.data_ptr(), _stream(x))
    return y


def nchw_to_nhwc_bf16(x: Tensor, cpad: int) -> Tensor:
    _chk(x, "network input (NCHW)")
    b, c, h, w = x.shape
    y = torch.empty((b, h, w, cpad), device=x.device, dtype=torch.bfloat16)
    _lib.call("pipnet_nchw_to_nhwc_bf16", x.data_ptr(), b, c, h, w, cpad, y.data_ptr(), _stream(x))
    return y


def conv1x1_bf16_dual(x: Tensor, w_packed: Tensor, bias: Tensor, n1: int, n2: int) -> Tuple[Tensor, Tensor]:
    """Two 1x1 stride-1 bf16 convs over one NHWC input in one launch (pipnet_conv1x1_bf16_dual):
    w_packed = the two packed weights stacked [n1 + n2, Kp], bias [n1 + n2] fp32 ->
    (x W1^T + b1, relu(x W2^T + b2)), each bit-equal to its own pipnet_conv2d_nhwc_bf16."""
    _chk_bf(x, "conv input")
    b, h, w, cin = x.shape
    if tuple(w_packed.shape[:1]) != (n1 + n2,) or bias.numel() != n1 + n2 or n1 % 256 or n2 % 256:
        raise RuntimeError(f"conv1x1_bf16_dual: weights {tuple(w_packed.shape)}, n1 {n1}, n2 {n2}")
    y1 = torch.empty((b, h, w, n1), device=x.device, dtype=torch.bfloat16)
    y2 = torch.empty((b, h, w, n2), device=x.device, dtype=torch.bfloat16)
    m = b * h * w
    _launch(f"pipnet_bf16::conv_bf16_ppp_kernel<12, {PP_RB}>",
            2.0 * m * (n1 + n2) * cin,
            lambda: _lib.call("pipnet_conv1x1_bf16_dual", x.data_ptr(), m, cin, w_packed.data_ptr(), bias.data_ptr(),
                              n1, y1.data_ptr(), n2, y2.data_ptr(), _stream(x)))
    return y1, y2


def nchw_to_s2d_bf16(x: Tensor) -> Tensor:
    """[B,3,H,W] fp32 -> [B, (H-1)//2 + 4, (W-1)//2 + 4, 16] bf16 space-to-depth stem input
    (pipnet_nchw_to_s2d_bf16): the k7 s2 p3 ResNet stem becomes a 4x4 stride-1 conv over it."""
    _chk(x, "network input (NCHW)")
    b, c, h, w = x.shape
    if c != 3:
        raise RuntimeError(f"nchw_to_s2d_bf16: expects 3 channels, got {c}")
    y = torch.empty((b, (h - 1) // 2 + 4, (w - 1) // 2 + 4, 16), device=x.device, dtype=torch.bfloat16)
    _lib.call("pipnet_nchw_to_s2d_bf16", x.data_ptr(), b, h, w, y.data_ptr(), _stream(x))
    return y


def stem_weight_s2d(w_ohwi: Tensor) -> Tensor:
    """[Cout, 7, 7, 3] (fp32, BatchNorm folded) -> [Cout, 4, 4, 16]: the taps of the k7 s2 conv
    regrouped for the 4x4 conv over the space-to-depth image, W'[o][a][a'][(2 bi + bj) * 4 + c] =
    w[o][2a+bi-1][2a'+bj-1][c], zero for the tap index -1 and the c = 3 slot."""
    co = w_ohwi.shape[0]
    w8 = torch.nn.functional.pad(w_ohwi, (0, 1, 1, 0, 1, 0))            # [Cout, 8 (ky+1), 8 (kx+1), 4]
    return w8.view(co, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(co, 4, 4, 16).contiguous()


def _head_out(out, b, h, w, p, dev):
    """Caller-provided (proto [B,h,w,P], pooled [B,P]) fp32 contiguous outputs, or new ones."""
    if out is None:
        return (torch.empty((b, h, w, p), device=dev, dtype=torch.float32),
                torch.empty((b, p), device=dev, dtype=torch.float32))
    proto, pooled = out
    if tuple(proto.shape) != (b, h, w, p) or tuple(pooled.shape) != (b, p):
        raise RuntimeError(f"softmax_pool: out shapes {tuple(proto.shape)}, {tuple(pooled.shape)} do not match "
                           f"{(b, h, w, p)}, {(b, p)}")
    _chk(proto, "proto out")
    _chk(pooled, "pooled out")
    return proto, pooled


def softmax_pool_bf16(feat_nhwc: Tensor, pool_mode: int, out=None) -> Tuple[Tensor, Tensor]:
    """bf16 logits [B,h,w,P] -> fp32 (proto [B,h,w,P], pooled [B,P])."""
    _chk_bf(feat_nhwc, "prototype logits")
    b, h, w, p = feat_nhwc.shape
    proto, pooled = _head_out(out, b, h, w, p, feat_nhwc.device)
    _lib.call("pipnet_softmax_pool_bf16", feat_nhwc.data_ptr(), b, h * w, p, pool_mode, proto.data_ptr(),
              pooled.data_ptr(), _stream(feat_nhwc))
    return proto, pooled


def convnext_stem(x_nchw: Tensor, w: Tensor, b: Tensor, ln_w: Tensor, ln_b: Tensor) -> Tensor:
    _chk(x_nchw, "network input (NCHW)")
    n, c, h, wd = x_nchw.shape
    if c != 3:
        raise RuntimeError(f"convnext stem expects 3 input channels, got {c}")
    y = torch.empty((n, h // 4, wd // 4, 96), device=x_nchw.device, dtype=torch.float32)
    _lib.call("pipnet_convnext_stem_f32", x_nchw.data_ptr(), n, h, wd, w.data_ptr(), b.data_ptr(), ln_w.data_ptr(),
              ln_b.data_ptr(), y.data_ptr(), _stream(x_nchw))
    return y


MLP_FUSED_CHANNELS = (96, 192)


@functools.lru_cache(maxsize=1024)
def cnblock_mlp_kernel_name(c: int, m: int = 1 << 20, hw: int = 0) -> str:
    """rocprof name of the fused MLP instantiation the library launches (pipnet_cnblock_mlp_plan:
    the library's own rule, csrc/mlp_f32.hip mlp_plan -- never mirrored here)."""
    code = _lib.load().pipnet_cnblock_mlp_plan(m, c, hw)
    if code < 0:
        raise RuntimeError(f"cnblock_mlp: no plan for M = {m}, C = {c}, hw = {hw}")
    hc, nw, hs = code // 100, code // 10 % 10, code % 10
    return f"cnblock_mlp_kernel<{c}, {hc}, {nw}, 1, {hs}>"


def cnblock_mlp(t: Tensor, w1: Tensor, b1: Tensor, w2: Tensor, b2: Tensor, gamma: Tensor, x: Tensor,
                hw: int = 0) -> Tensor:
    """In place on ``x`` [M, C]: x += gamma * (W2 gelu(W1 t + b1) + b2) -- the whole CNBlock MLP
    of a narrow stage (C = 96 / 192) in one kernel, the hidden activation kept in registers
    (csrc/mlp_f32.hip).  ``hw`` = the layer's pixels per image (0 = unknown): picks the
    instantiation by map size, never by M."""
    for v, what in ((t, "mlp input"), (w1, "fc1 weight"), (b1, "fc1 bias"), (w2, "fc2 weight"), (b2, "fc2 bias"),
                    (gamma, "layer scale"), (x, "residual")):
        _chk(v, what)
    m, c = t.shape
    if c not in MLP_FUSED_CHANNELS or tuple(x.shape) != (m, c) or tuple(w1.shape) != (4 * c, c) \
            or tuple(w2.shape) != (c, 4 * c) or b1.numel() != 4 * c or b2.numel() != c or gamma.numel() != c:
        raise RuntimeError(f"cnblock_mlp: shapes t {tuple(t.shape)} w1 {tuple(w1.shape)} w2 {tuple(w2.shape)}")
    _launch(cnblock_mlp_kernel_name(c, m, hw), 2.0 * 2 * m * 4 * c * c,
            lambda: _lib.call("pipnet_cnblock_mlp_hw_f32", t.data_ptr(), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                              b2.data_ptr(), gamma.data_ptr(), x.data_ptr(), m, c, hw, _stream(t)))
    return x


def dwconv7_ln(x_nhwc: Tensor, w_packed: Tensor, bias: Tensor, ln_w: Tensor, ln_b: Tensor,
               out: Optional[Tensor] = None) -> Tensor:
    _chk(x_nhwc, "dwconv input")
    b, h, w, c = x_nhwc.shape
    y = torch.empty_like(x_nhwc) if out is None else out
    _lib.call("pipnet_dwconv7_ln_f32", x_nhwc.data_ptr(), b, h, w, c, w_packed.data_ptr(), bias.data_ptr(),
              ln_w.data_ptr(), ln_b.data_ptr(), y.data_ptr(), _stream(x_nhwc))
    return y


# ---- split-bf16 ("bf16x3") ConvNeXt path (include/pipnet_amd.h, pipnet_conv2d_nhwc_s3) ----
S3_KTILE = 32          # split weights: K padded to the 32-deep K tiles of the split kernels
def split_planes_weight(w_ohwi: Tensor) -> Tensor:
    """fp32 weight [Cout, KH, KW, Cin] -> packed split-bf16 B operand [Cout, Kp] bf16: per tap
    [hi | hi | lo] over 3 Cin (hi = RNE(w), lo = RNE(w - hi)), Kp = KH*KW*3Cin rounded up to 32."""
    hi = w_ohwi.to(torch.bfloat16)
    lo = (w_ohwi - hi.float()).to(torch.bfloat16)
    cout, kh, kw, cin = w_ohwi.shape
    k = kh * kw * 3 * cin
    kp = -(-k // S3_KTILE) * S3_KTILE
    out = torch.zeros((cout, kp), device=w_ohwi.device, dtype=torch.bfloat16)
    out[:, :k] = torch.cat([hi, hi, lo], dim=-1).reshape(cout, k)
    return out


def split_planes(x: Tensor) -> Tensor:
    """fp32 [..., C] -> split planes [..., 2C] bf16 [hi | lo] (what the producer kernels
    write; for tests and for inputs that do not come from a split-writing kernel)."""
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, lo], dim=-1).contiguous()


def conv_s3(x2: Tensor, w_packed: Tensor, kh: int, kw: int, cout: int, bias: Optional[Tensor], stride: int, pad: int,
            epilogue: int, scale: Optional[Tensor] = None, r: Optional[Tensor] = None, out: Optional[Tensor] = None,
            tile: int = -1) -> Tensor:
    """Split-bf16 conv / linear: x2 [B,H,W,2Cin] split planes, w_packed from split_planes_weight.
    EPI_S3_GELU -> split planes [B,OH,OW,2Cout] of gelu(conv + b); EPI_F32_BIAS -> fp32
    [B,OH,OW,Cout]; EPI_F32_RESID -> fp32 r + scale * (conv + b) (``out`` may be ``r``)."""
    _chk_bf(x2, "split-plane input")
    _chk_bf(w_packed, "split-plane weight")
    if bias is not None:
        _chk(bias, "bias")
    b, h, w, cin2 = x2.shape
    cin = cin2 // 2
    k = kh * kw * 3 * cin
    if cin2 % 2 or w_packed.shape[0] != cout or w_packed.shape[1] != -(-k // S3_KTILE) * S3_KTILE:
        raise RuntimeError(f"conv_s3: packed weight {tuple(w_packed.shape)} does not match {kh}x{kw}x3*{cin} -> {cout}")
    oh, ow = (h + 2 * pad - kh) // stride + 1, (w + 2 * pad - kw) // stride + 1
    if epilogue == _lib.EPI_S3_GELU:
        shape, dt = (b, oh, ow, 2 * cout), torch.bfloat16
    else:
        shape, dt = (b, oh, ow, cout), torch.float32
    if epilogue == _lib.EPI_F32_RESID:
        if r is None or scale is None:
            raise RuntimeError("conv_s3: EPI_F32_RESID needs r and scale")
        _chk(r, "residual")
        _chk(scale, "layer scale")
        if r.numel() != b * oh * ow * cout:
            raise RuntimeError(f"conv_s3: residual {tuple(r.shape)} does not match {(b, oh, ow, cout)}")
    if out is None:
        out = torch.empty(shape, device=x2.device, dtype=dt)
    elif out.dtype != dt or out.numel() != b * oh * ow * shape[-1] or not out.is_contiguous():
        raise RuntimeError(f"conv_s3: out {tuple(out.shape)} {out.dtype} does not match {shape} {dt}")
    m = b * oh * ow
    aload = 0 if (kh == 1 and kw == 1 and stride == 1 and pad == 0) else 2
    t = tile if tile >= 0 else s3_conv_tile(m, cout, kv=k)
    _launch(bf16_conv_kernel_name(m, cout, epilogue, aload, t, s3=True, kv=k), 2.0 * m * cout * k / 3.0,
            lambda: _lib.call("pipnet_conv2d_nhwc_s3", x2.data_ptr(), b, h, w, cin, w_packed.data_ptr(), _ptr(bias),
                              _ptr(scale), _ptr(r), cout, kh, kw, stride, pad, epilogue, out.data_ptr(), tile,
                              _stream(x2)))
    return out


def dwconv7_ln_s3(x_nhwc: Tensor, w_packed: Tensor, bias: Tensor, ln_w: Tensor, ln_b: Tensor) -> Tensor:
    """pipnet_dwconv7_ln_f32 writing split planes [B,H,W,2C] bf16."""
    _chk(x_nhwc, "dwconv input")
    b, h, w, c = x_nhwc.shape
    y = torch.empty((b, h, w, 2 * c), device=x_nhwc.device, dtype=torch.bfloat16)
    _lib.call("pipnet_dwconv7_ln_s3", x_nhwc.data_ptr(), b, h, w, c, w_packed.data_ptr(), bias.data_ptr(),
              ln_w.data_ptr(), ln_b.data_ptr(), y.data_ptr(), _stream(x_nhwc))
    return y


def layernorm_s3(x: Tensor, w: Tensor, b: Tensor) -> Tensor:
    """Row LayerNorm writing split planes [..., 2C] bf16."""
    _chk(x, "layernorm input")
    c = x.shape[-1]
    y = torch.empty(tuple(x.shape[:-1]) + (2 * c,), device=x.device, dtype=torch.bfloat16)
    _lib.call("pipnet_layernorm_s3", x.data_ptr(), x.numel() // c, c, w.data_ptr(), b.data_ptr(), y.data_ptr(),
              _stream(x))
    return y


def layernorm(x: Tensor, w: Tensor, b: Tensor, out: Optional[Tensor] = None) -> Tensor:
    _chk(x, "layernorm input")
    c = x.shape[-1]
    y = torch.empty_like(x) if out is None else out
    _lib.call("pipnet_layernorm_f32", x.data_ptr(), x.numel() // c, c, w.data_ptr(), b.data_ptr(), y.data_ptr(),
              _stream(x))
    return y


def softmax_pool(feat_nhwc: Tensor, pool_mode: int, out=None) -> Tuple[Tensor, Tensor]:
    """feat [B,h,w,P] -> (proto [B,h,w,P], pooled [B,P]); pool 0 = max, 1 = sum.
    ``out`` = (proto, pooled) to write into (e.g. batch slices of a larger output)."""
    _chk(feat_nhwc, "prototype logits")
    b, h, w, p = feat_nhwc.shape
    proto, pooled = _head_out(out, b, h, w, p, feat_nhwc.device)
    _lib.call("pipnet_softmax_pool_f32", feat_nhwc.data_ptr(), b, h * w, p, pool_mode, proto.data_ptr(),
              pooled.data_ptr(), _stream(feat_nhwc))
    return proto, pooled


def softmax_pool_linear(feat_nhwc: Tensor, w: Tensor, bias: Optional[Tensor], thresh: Optional[float],
                        out=None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """The PIP-Net head in one launch (pipnet.py:33-37): fp32 or bf16 logits [B,h,w,P] ->
    (proto [B,h,w,P], pooled [B,P], x' [B,P], logits [B,K]) with x' = where(pooled < thresh, 0,
    pooled) (or pooled when ``thresh`` is None) and logits = x' relu(w)^T + bias, w read at call
    time.  ``out`` = (proto, pooled, x', logits) to write into (batch slices of a larger output).
    Bitwise equal to softmax_pool(..., 0) + nonneg_linear.  Under HIP-graph capture the call keeps
    using the capture stream's cached scratch (one graph node): serialise replays with eager calls
    on that stream."""
    bf = feat_nhwc.dtype == torch.bfloat16
    if bf:
        _chk_bf(feat_nhwc, "prototype logits")
    else:
        _chk(feat_nhwc, "prototype logits")
    _chk(w, "classifier weight")
    b, h, wd, p = feat_nhwc.shape
    k = w.shape[0]
    if w.dim() != 2 or w.shape[1] != p:
        raise RuntimeError(f"softmax_pool_linear: weight {tuple(w.shape)} vs {p} prototypes")
    dev = feat_nhwc.device
    if out is None:
        proto, pooled = _head_out(None, b, h, wd, p, dev)
        x_out = torch.empty((b, p), device=dev, dtype=torch.float32)
        logits = torch.empty((b, k), device=dev, dtype=torch.float32)
    else:
        proto, pooled = _head_out((out[0], out[1]), b, h, wd, p, dev)
        x_out, logits = out[2], out[3]
        if tuple(x_out.shape) != (b, p) or tuple(logits.shape) != (b, k):
            raise RuntimeError("softmax_pool_linear: out shapes do not match")
        _chk(x_out, "classifier input out")
        _chk(logits, "logits out")
    part, tickets = _head_workspace(dev, _stream(feat_nhwc), int(_lib.load().pipnet_softmax_pool_linear_part_floats(
        b, h * wd, p)), b)
    _lib.call("pipnet_softmax_pool_linear_bf16" if bf else "pipnet_softmax_pool_linear_f32", feat_nhwc.data_ptr(), b,
              h * wd, p, proto.data_ptr(), pooled.data_ptr(), w.data_ptr(), _ptr(bias), k,
              0 if thresh is None else 1, 0.0 if thresh is None else float(thresh), x_out.data_ptr(),
              logits.data_ptr(), part.data_ptr(), tickets.data_ptr(), _stream(feat_nhwc))
    return proto, pooled, x_out, logits


# Fused-head scratch, one (running maxima, tickets) pair per (device, stream): both are zeroed once
# here and left zero by every completed launch (include/pipnet_amd.h), so
# the head needs no memset per call; per stream because two concurrent heads (the split forward's
# sub-batch streams) must not share them.  Buffers only grow; a grown one is allocated (zeroed) on
# the stream that uses it.
_HEAD_WS = {}


def _head_workspace(dev: torch.device, stream: int, nfloats: int, b: int) -> Tuple[Tensor, Tensor]:
    key = (dev.index, stream)
    # A capture reuses this stream's cached scratch when it is large enough (so the captured head
    # stays ONE graph node: a graph-owned buffer would add its zero-fill nodes).  The graph then
    # shares the scratch -- and its self-resetting tickets -- with eager calls on the capture
    # stream: replays must be serialised with such calls (replay on the capture stream, or
    # synchronise first); a replay on another stream racing an eager call would corrupt both.
    part, tickets = _HEAD_WS.get(key, (None, None))
    capturing = torch.cuda.is_current_stream_capturing()
    if part is None or part.numel() < nfloats:
        part = torch.zeros(max(nfloats, 4), device=dev, dtype=torch.float32)
    if tickets is None or tickets.numel() < b:
        tickets = torch.zeros(max(b, 64), device=dev, dtype=torch.int32)
    if not capturing:          # graph-owned buffers (their zero-fill replays with them) are never cached
        _HEAD_WS[key] = (part, tickets)
    return part, tickets


def nonneg_linear(x: Tensor, w: Tensor, bias: Optional[Tensor], thresh: Optional[float],
                  out=None) -> Tuple[Tensor, Tensor]:
    """(x', out) with x' = where(x < thresh, 0, x) (or x) and out = x' relu(w)^T + bias.
    ``out`` = (x', logits) to write into."""
    _chk(x, "classifier input")
    _chk(w, "classifier weight")
    b, d = x.shape
    k = w.shape[0]
    if out is None:
        x_out = torch.empty_like(x)
        out = torch.empty((b, k), device=x.device, dtype=torch.float32)
    else:
        x_out, out = out
        if tuple(x_out.shape) != (b, d) or tuple(out.shape) != (b, k):
            raise RuntimeError("nonneg_linear: out shapes do not match")
        _chk(x_out, "classifier input out")
        _chk(out, "logits out")
    _lib.call("pipnet_nonneg_linear_f32", x.data_ptr(), b, d, w.data_ptr(), _ptr(bias), k,
              0 if thresh is None else 1, 0.0 if thresh is None else float(thresh), x_out.data_ptr(),
              out.data_ptr(), _stream(x))
    return x_out, out


def count_gumbel(logits_nhwc: Tensor, tau: float, exp_noise_nchw: Optional[Tensor], seed: int,
                 offset: int = 0, out=None) -> Tuple[Tensor, Tensor]:
    """Hard Gumbel-softmax one-hot map [B,h,w,P] + int32 histogram [B,P].  ``offset`` (Philox
    blocks) shifts the noise stream: image b0 of a batch starts at b0*h*w*P/4.  ``out`` =
    (proto, hist) to write into (batch slices of a larger output)."""
    _chk(logits_nhwc, "prototype logits")
    b, h, w, p = logits_nhwc.shape
    if exp_noise_nchw is not None:
        _chk(exp_noise_nchw, "exp noise")
        if tuple(exp_noise_nchw.shape) != (b, p, h, w):
            raise RuntimeError(f"exp noise shape {tuple(exp_noise_nchw.shape)} != {(b, p, h, w)}")
    if out is None:
        proto = torch.empty_like(logits_nhwc)
        hist = torch.empty((b, p), device=logits_nhwc.device, dtype=torch.int32)
    else:
        proto, hist = out
        if tuple(proto.shape) != (b, h, w, p) or tuple(hist.shape) != (b, p) or hist.dtype != torch.int32:
            raise RuntimeError(f"count_gumbel: out {tuple(proto.shape)}, {tuple(hist.shape)} {hist.dtype} do not "
                               f"match {(b, h, w, p)}, {(b, p)} int32")
        _chk(proto, "proto out")
        if not (hist.is_cuda and hist.is_contiguous()):
            raise RuntimeError("count_gumbel: hist out must be a contiguous device tensor")
    _lib.call("pipnet_count_gumbel_f32", logits_nhwc.data_ptr(), b, h * w, p, float(tau), _ptr(exp_noise_nchw),
              int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), proto.data_ptr(), hist.data_ptr(),
              _stream(logits_nhwc))
    return proto, hist


def count_gumbel_soft(logits_nhwc: Tensor, tau: float, exp_noise_nchw: Optional[Tensor], seed: int,
                      offset: int = 0) -> Tuple[Tensor, Tensor]:
    """Train-mode (soft) Gumbel-softmax map [B,h,w,P] + fp32 spatial sums (raw counts) [B,P]."""
    _chk(logits_nhwc, "prototype logits")
    b, h, w, p = logits_nhwc.shape
    if exp_noise_nchw is not None:
        _chk(exp_noise_nchw, "exp noise")
        if tuple(exp_noise_nchw.shape) != (b, p, h, w):
            raise RuntimeError(f"exp noise shape {tuple(exp_noise_nchw.shape)} != {(b, p, h, w)}")
    proto = torch.empty_like(logits_nhwc)
    sums = torch.empty((b, p), device=logits_nhwc.device, dtype=torch.float32)
    _lib.call("pipnet_count_gumbel_soft_f32", logits_nhwc.data_ptr(), b, h * w, p, float(tau), _ptr(exp_noise_nchw),
              int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), proto.data_ptr(), sums.data_ptr(),
              _stream(logits_nhwc))
    return proto, sums


def nonneg_linear_dx(d_out: Tensor, w: Tensor) -> Tensor:
    """d_out [N,K] relu(w [K,D]) -> [N,D] (NonNegLinear input gradient)."""
    _chk(d_out, "d_out")
    _chk(w, "classifier weight")
    n, k = d_out.shape
    if w.shape[0] != k:
        raise RuntimeError(f"nonneg_linear_dx: d_out {tuple(d_out.shape)} vs W {tuple(w.shape)}")
    dx = torch.empty((n, w.shape[1]), device=d_out.device, dtype=torch.float32)
    _lib.call("pipnet_nonneg_linear_dx_f32", d_out.data_ptr(), w.data_ptr(), n, w.shape[1], k, dx.data_ptr(),
              _stream(d_out))
    return dx


def bilinear_bwd_prep(g: Tensor, u: Tensor, v: Tensor) -> Tuple[Tensor, Tensor]:
    """(g * v, g * u) for out = u * v."""
    for t, what in ((g, "grad"), (u, "W(e)"), (v, "V(e)")):
        _chk(t, what)
    if not (g.shape == u.shape == v.shape):
        raise RuntimeError("bilinear_bwd_prep: shape mismatch")
    du, dv = torch.empty_like(g), torch.empty_like(g)
    _lib.call("pipnet_bilinear_bwd_prep_f32", g.data_ptr(), u.data_ptr(), v.data_ptr(), g.numel(), du.data_ptr(),
              dv.data_ptr(), _stream(g))
    return du, dv


ONEHOT_STRATEGY = {None: 0, "none": 0, "current_grad": 1, "max_grad": 2}


def count_ste_backward(counts: Tensor, d_clamped: Tensor, max_count: int, use_ste: bool, gated: bool) -> Tensor:
    """d raw counts from d clamped counts through STE_Round / ClampSTE (count_pipnet.py:90-97)."""
    _chk(counts, "counts")
    _chk(d_clamped, "d clamped counts")
    if counts.shape != d_clamped.shape:
        raise RuntimeError(f"count_ste_backward: counts {tuple(counts.shape)} vs grad {tuple(d_clamped.shape)}")
    d = torch.empty_like(counts)
    _lib.call("pipnet_count_ste_bwd_f32", counts.data_ptr(), counts.numel(), int(max_count), int(bool(use_ste)),
              int(bool(gated)), d_clamped.data_ptr(), d.data_ptr(), _stream(counts))
    return d


def onehot_ste_backward(x: Tensor, g: Tensor, strategy: Optional[str] = None, respect_active: bool = False) -> Tensor:
    """ModifiedSTEFunction.backward (count_pipnet_utils.py:226-321): x [B,P] encoder input,
    g [B,P*M] (or [B,P,M]) encoding gradient -> d x [B,P]."""
    _chk(x, "one-hot encoder input")
    _chk(g, "encoding gradient")
    b, p = x.shape
    if g.numel() % max(x.numel(), 1) or g.shape[0] != b:
        raise RuntimeError(f"onehot_ste_backward: x {tuple(x.shape)} vs grad {tuple(g.shape)}")
    if strategy not in ONEHOT_STRATEGY:
        raise ValueError(f"Unknown positive_grad_strategy {strategy!r}")
    m = g.numel() // max(x.numel(), 1)
    dx = torch.empty_like(x)
    flag = torch.empty(1, device=x.device, dtype=torch.int32)
    _lib.call("pipnet_onehot_ste_bwd_f32", x.data_ptr(), x.numel(), m, g.data_ptr(), ONEHOT_STRATEGY[strategy],
              int(bool(respect_active)), flag.data_ptr(), dx.data_ptr(), _stream(x))
    return dx


def linear_intermediate_backward(x: Tensor, g: Tensor, w: Tensor, want_dx: bool = True,
                                 dw_out: Optional[Tensor] = None) -> Tuple[Optional[Tensor], Tensor]:
    """LinearIntermediate backward (count_pipnet_utils.py:471-519): x [B,P] counts, g [B,P*E]
    output gradient, w [E,1] -> (d x [B,P] or None, d w [E,1])."""
    _chk(x, "intermediate input")
    _chk(g, "intermediate output gradient")
    e = w.numel()
    if g.numel() != x.numel() * e or g.shape[0] != x.shape[0]:
        raise RuntimeError(f"linear_intermediate_backward: x {tuple(x.shape)}, grad {tuple(g.shape)}, E={e}")
    wv = w.detach().reshape(-1).contiguous()
    dx = torch.empty_like(x) if want_dx else None
    dw = torch.empty(e, 1, device=x.device, dtype=torch.float32) if dw_out is None else dw_out
    part = torch.empty(int(_lib.load().pipnet_linear_inter_partials_floats(e)), device=x.device,
                       dtype=torch.float32)
    _lib.call("pipnet_linear_inter_bwd_f32", x.data_ptr(), x.numel(), e, g.data_ptr(), wv.data_ptr(),
              dx.data_ptr() if dx is not None else None, dw.data_ptr(), 0, part.data_ptr(), _stream(x))
    return dx, dw


def count_head_backward(proto_nhwc: Tensor, counts: Tensor, d_counts: Optional[Tensor], w_align: float,
                        w_tanh: float, tanh_coeff: float, tau: float) -> Tensor:
    """d loss / d logits of the CountPIPNet head (soft Gumbel-softmax / softmax, spatial sum)
    for the align / tanh terms of calculate_loss plus the classifier chain's d counts."""
    _chk(proto_nhwc, "proto features")
    _chk(counts, "counts")
    n, h, ww, p = proto_nhwc.shape
    if tuple(counts.shape) != (n, p) or n % 2:
        raise RuntimeError(f"count_head_backward: proto {tuple(proto_nhwc.shape)} vs counts {tuple(counts.shape)}")
    if d_counts is not None:
        _chk(d_counts, "d counts")
        if d_counts.shape != counts.shape:
            raise RuntimeError("count_head_backward: d counts shape")
    d_logits = torch.empty_like(proto_nhwc)
    dcnt = torch.empty((n, p), device=proto_nhwc.device, dtype=torch.float32)
    _lib.call("pipnet_count_head_bwd_f32", proto_nhwc.data_ptr(), counts.data_ptr(), n // 2, h * ww, p,
              _ptr(d_counts), float(w_align), float(w_tanh), float(tanh_coeff), 1.0 / float(tau), dcnt.data_ptr(),
              d_logits.data_ptr(), _stream(proto_nhwc))
    return d_logits


def philox_exp1(seed: int, offset: int, n: int, device, log_e: bool = False) -> Tensor:
    """The Gumbel heads' Exp(1) draw on its own (pipnet_philox_exp1_f32): element i = the value
    count_gumbel uses for element i of its NHWC [B, HW, P] stream under (seed, offset) -- E, or
    log E on the hard head's hardware-log form.  For parity tests (oracle/philox_ref.py)."""
    if n % 4:
        raise RuntimeError(f"philox_exp1: n = {n} must be a multiple of 4")
    out = torch.empty(n, device=device, dtype=torch.float32)
    _chk(out, "philox output")
    _lib.call("pipnet_philox_exp1_f32", int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), n, int(log_e),
              out.data_ptr(), _stream(out))
    return out


def count_gumbel_devseed(logits_nhwc: Tensor, tau: float, seed_state: Tensor) -> Tuple[Tensor, Tensor]:
    """count_gumbel with the Philox key in device memory (seed_state: int64[2] on the device),
    advanced on the stream per call -- the form a captured HIP graph replays."""
    _chk(logits_nhwc, "prototype logits")
    if not (seed_state.is_cuda and seed_state.dtype == torch.int64 and seed_state.numel() == 2):
        raise RuntimeError("count_gumbel_devseed: seed_state must be a 2-element int64 device tensor")
    b, h, w, p = logits_nhwc.shape
    proto = torch.empty_like(logits_nhwc)
    hist = torch.empty((b, p), device=logits_nhwc.device, dtype=torch.int32)
    _lib.call("pipnet_count_gumbel_devseed_f32", logits_nhwc.data_ptr(), b, h * w, p, float(tau),
              seed_state.data_ptr(), proto.data_ptr(), hist.data_ptr(), _stream(logits_nhwc))
    return proto, hist


def count_finish(hist: Optional[Tensor], sums: Optional[Tensor], max_count: int, do_round: bool) -> Tuple[Tensor, Tensor]:
    ref = hist if hist is not None else sums
    b, p = ref.shape
    raw = torch.empty((b, p), device=ref.device, dtype=torch.float32)
    clamped = torch.empty_like(raw)
    _lib.call("pipnet_count_finish_f32", _ptr(hist), _ptr(sums), b, p, int(max_count), int(do_round),
              raw.data_ptr(), clamped.data_ptr(), _stream(ref))
    return raw, clamped


def count_encode(x: Tensor, c: int, kind: int, do_round: bool, w: Optional[Tensor] = None) -> Tensor:
    _chk(x, "counts")
    b, p = x.shape
    out = torch.empty((b, p * c), device=x.device, dtype=torch.float32)
    _lib.call("pipnet_count_encode_f32", x.data_ptr(), b, p, c, kind, int(do_round), _ptr(w), out.data_ptr(),
              _stream(x))
    return out


# ---- eval_pipnet metric loop ------------------------------------------------------------

def _mutated(*ts: Tensor) -> None:
    """A kernel wrote these tensors through raw pointers: bump their in-place version
    counters, as a torch in-place op would, so version-keyed caches (packed weights) and
    autograd's saved-tensor checks see the change."""
    for t in ts:
        torch.autograd.graph.increment_version(t)


def weight_sparsify_(w: Tensor, delta: float = 1e-3) -> Tensor:
    """In place: w = max(w - delta, 0) (pipnet/test.py:73)."""
    _chk(w, "classification weight")
    _lib.call("pipnet_weight_sparsify_f32", w.data_ptr(), w.numel(), delta, _stream(w))
    _mutated(w)
    return w


def eval_batch(pooled: Tensor, out: Tensor, w: Tensor, ys: Tensor, multiplier: Optional[Tensor], thr: float,
               cm: Tensor, acc: Tensor, abstained: Tensor) -> Tuple[Tensor, Tensor]:
    """One eval_pipnet batch on the device; accumulates into cm [K,K] int64, acc [5] fp64,
    abstained [1] int64.  Returns (ys_pred [B] int32, score [B] fp32)."""
    _chk(pooled, "pooled")
    _chk(out, "logits")
    _chk(w, "prototype-class weights")
    b, p = pooled.shape
    k = out.shape[1]
    if tuple(w.shape) != (k, p) or out.shape[0] != b or ys.shape != (b,):
        raise RuntimeError(f"eval_batch: shapes pooled {tuple(pooled.shape)}, out {tuple(out.shape)}, "
                           f"w {tuple(w.shape)}, ys {tuple(ys.shape)} disagree")
    if not (ys.is_cuda and ys.dtype == torch.int64 and ys.is_contiguous()):
        raise RuntimeError("eval_batch: labels must be a contiguous int64 device tensor")
    if cm.dtype != torch.int64 or acc.dtype != torch.float64 or abstained.dtype != torch.int64:
        raise RuntimeError("eval_batch: accumulator dtypes are int64 / float64 / int64")
    if multiplier is not None:
        _chk(multiplier, "normalization multiplier")
    ys_pred = torch.empty(b, device=out.device, dtype=torch.int32)
    score = torch.empty(b, device=out.device, dtype=torch.float32)
    ws = torch.empty(5 * b + k, device=out.device, dtype=torch.int32)
    _lib.call("pipnet_eval_batch_f32", pooled.data_ptr(), out.data_ptr(), w.data_ptr(), b, p, k, ys.data_ptr(),
              _ptr(multiplier), thr, ys_pred.data_ptr(), score.data_ptr(), cm.data_ptr(), acc.data_ptr(),
              abstained.data_ptr(), ws.data_ptr(), _stream(out))
    return ys_pred, score


# ---- evaluation input transform (util/data.py transform_no_augment) ----------------------

def resize_normalize_rgb8(pixels: Tensor, offsets: Tensor, sizes: Tensor, sizes_host, out_hw: Tuple[int, int],
                          mean, std, grayscale: bool = False, want_u8: bool = False):
    """Resize(out_hw, BILINEAR) [+ Grayscale(3)] + ToTensor + Normalize of a ragged batch of
    decoded RGB images packed HWC uint8 on the device (image b at byte offsets[b], shape
    sizes[b] = (h, w)); ``sizes_host`` is the same [B,2] int32 table on the host.
    Returns [B,3,oh,ow] fp32 (and the [B,oh,ow,3] uint8 resized image when ``want_u8``)."""
    import ctypes

    import numpy as np
    if not (pixels.is_cuda and pixels.dtype == torch.uint8 and pixels.is_contiguous()):
        raise RuntimeError("resize_normalize_rgb8: pixels must be a contiguous uint8 ROCm device tensor "
                           "(there is no CPU fallback)")
    if not (offsets.is_cuda and offsets.dtype == torch.int64 and sizes.is_cuda and sizes.dtype == torch.int32):
        raise RuntimeError("resize_normalize_rgb8: offsets (int64) / sizes (int32) must be device tensors")
    sizes_np = np.ascontiguousarray(np.asarray(sizes_host, dtype=np.int32).reshape(-1, 2))
    b = sizes_np.shape[0]
    if offsets.shape != (b,) or tuple(sizes.shape) != (b, 2):
        raise RuntimeError(f"resize_normalize_rgb8: {b} images but offsets {tuple(offsets.shape)}, "
                           f"sizes {tuple(sizes.shape)}")
    oh, ow = int(out_hw[0]), int(out_hw[1])
    kmax, wsb = ctypes.c_int(0), ctypes.c_int64(0)
    _lib.call("pipnet_resize_plan", sizes_np.ctypes.data, b, oh, ow, ctypes.byref(kmax), ctypes.byref(wsb))
    dev = pixels.device
    out = torch.empty((b, 3, oh, ow), device=dev, dtype=torch.float32)
    out_u8 = torch.empty((b, oh, ow, 3), device=dev, dtype=torch.uint8) if want_u8 else None
    ws = torch.empty(max(1, wsb.value // 4), device=dev, dtype=torch.int32)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    _lib.call("pipnet_resize_normalize_rgb8", pixels.data_ptr(), offsets.data_ptr(), sizes.data_ptr(), b, oh, ow,
              kmax.value, int(bool(grayscale)), m, s, ws.data_ptr(), out.data_ptr(), _ptr(out_u8),
              torch.cuda.current_stream(dev).cuda_stream)
    return (out, out_u8) if want_u8 else out


# ---- training step, finetune phase (csrc/train_ops.hip) -------------------------------------
TRAIN_MODE = {"train": 0, "pretrain": 1, "finetune": 2}


def train_loss(proto_nhwc: Tensor, pooled: Tensor, out: Tensor, ys: Tensor, mult: Optional[Tensor],
               enforce: bool, tanh_coeff: float, w_align: float, w_tanh: float, w_class: float,
               mode: str) -> Tuple[Tensor, Optional[Tensor]]:
    """calculate_loss (pipnet/train.py:154-250) on the device: returns (stats [8] fp32 =
    align, tanh, class, loss, correct, w_align, w_tanh, w_class; d_out [N,K] or None)."""
    _chk(proto_nhwc, "proto features (NHWC)")
    _chk(pooled, "pooled")
    _chk(out, "classifier output")
    n, h, w, p = proto_nhwc.shape
    if n % 2 or tuple(pooled.shape) != (n, p) or out.shape[0] != n:
        raise RuntimeError(f"train_loss: proto {tuple(proto_nhwc.shape)}, pooled {tuple(pooled.shape)}, "
                           f"out {tuple(out.shape)} must share an even batch = cat([xs1, xs2])")
    bh, k = n // 2, out.shape[1]
    if not (ys.is_cuda and ys.dtype == torch.int64 and ys.is_contiguous() and ys.shape == (bh,)):
        raise RuntimeError("train_loss: labels must be a contiguous int64 device tensor of the half batch")
    if mult is not None:
        _chk(mult, "normalization_multiplier")
    partial = torch.empty(_lib.load().pipnet_train_align_partials(), device=out.device, dtype=torch.float64)
    s = _stream(out)
    _lib.call("pipnet_train_align_partial_f32", proto_nhwc.data_ptr(), bh, h * w, p, partial.data_ptr(), s)
    stats = torch.empty(8, device=out.device, dtype=torch.float32)
    m = TRAIN_MODE[mode]
    d_out = None if m == 1 else torch.empty_like(out)
    _lib.call("pipnet_train_loss_f32", partial.data_ptr(), bh, h * w, pooled.data_ptr(), out.data_ptr(),
              ys.data_ptr(), p, k, _ptr(mult), int(bool(enforce)), float(tanh_coeff), float(w_align),
              float(w_tanh), float(w_class), m, _ptr(d_out), stats.data_ptr(), s)
    return stats, d_out


def nonneg_linear_backward(d_out: Tensor, x: Tensor, w: Tensor, want_bias: bool) -> Tuple[Tensor, Optional[Tensor]]:
    """Gradients of F.linear(x, relu(w), b) (pipnet.py:54-71): (dW, db or None)."""
    _chk(d_out, "d_out")
    _chk(x, "classifier input")
    _chk(w, "classifier weight")
    n, d = x.shape
    k = w.shape[0]
    if tuple(w.shape) != (k, d) or tuple(d_out.shape) != (n, k):
        raise RuntimeError("nonneg_linear_backward: shapes disagree")
    dw = torch.empty_like(w)
    db = torch.empty(k, device=w.device, dtype=torch.float32) if want_bias else None
    _lib.call("pipnet_nonneg_linear_bwd_f32", d_out.data_ptr(), x.data_ptr(), n, d, w.data_ptr(), k,
              dw.data_ptr(), _ptr(db), _stream(w))
    return dw, db


def adamw_step_(param: Tensor, grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, lr: float, beta1: float,
                beta2: float, eps: float, weight_decay: float, step: int,
                post: Optional[Tuple[float, float]] = None) -> None:
    """torch.optim.AdamW's update of one tensor in place at optimizer step ``step`` (1-based;
    bias corrections from the double hyper-parameters, as torch computes them for a
    non-capturable optimizer); ``post`` = (delta, floor) applies p = max(p - delta, floor)
    afterwards (pipnet/train.py:134-140)."""
    for t, what in ((param, "parameter"), (grad, "gradient"), (exp_avg, "exp_avg"), (exp_avg_sq, "exp_avg_sq")):
        _chk(t, what)
        if t.shape != param.shape:
            raise RuntimeError(f"adamw_step_: {what} shape {tuple(t.shape)} != {tuple(param.shape)}")
    delta, floor = post if post is not None else (0.0, 0.0)
    _lib.call("pipnet_adamw_step_f32", param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(),
              exp_avg_sq.data_ptr(), param.numel(), lr, beta1, beta2, eps, weight_decay, int(step),
              int(post is not None), delta, floor, _stream(param))
    _mutated(param, exp_avg, exp_avg_sq)


def clamp_min_(x: Tensor, lo: float) -> Tensor:
    _chk(x, "tensor")
    _lib.call("pipnet_clamp_min_f32", x.data_ptr(), x.numel(), lo, _stream(x))
    _mutated(x)
    return x


# ---- backward building blocks (csrc/backward_ops.hip) ----------------------------------------
def wgrad(a: Tensor, b: Tensor, out: Optional[Tensor] = None, accumulate: bool = False) -> Tensor:
    """out[N1,N2] (+)= a[M,N1]^T @ b[M,N2] (weight gradient dY^T X), deterministic."""
    for t, what in ((a, "wgrad A"), (b, "wgrad B")):
        require_device(t, what)
        if t.dim() != 2 or t.stride(1) != 1:
            raise RuntimeError(f"{what}: expects a 2-D row-major view")
    m, n1 = a.shape
    if b.shape[0] != m:
        raise RuntimeError(f"wgrad: row counts differ {tuple(a.shape)} vs {tuple(b.shape)}")
    n2 = b.shape[1]
    if out is None:
        if accumulate:
            raise RuntimeError("wgrad: accumulate needs out")
        out = torch.empty((n1, n2), device=a.device, dtype=torch.float32)
    elif tuple(out.shape) != (n1, n2) or out.stride(1) != 1:
        raise RuntimeError("wgrad: out shape")
    nbytes = _lib.load().pipnet_wgrad_workspace_bytes(m, n1, n2)
    ws = torch.empty(max(nbytes // 4, 1), device=a.device, dtype=torch.float32)
    _lib.call("pipnet_wgrad_f32", a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), m, n1, n2, out.data_ptr(),
              out.stride(0), int(accumulate), ws.data_ptr(), _stream(a))
    return out


def colsum(a: Tensor, out: Optional[Tensor] = None, accumulate: bool = False) -> Tensor:
    """out[N] (+)= a[M,N].sum(0), deterministic."""
    require_device(a, "colsum input")
    m, n = a.shape
    if out is None:
        out = torch.empty(n, device=a.device, dtype=torch.float32)
    ws = torch.empty(_lib.load().pipnet_colsum_workspace_bytes(n) // 4, device=a.device, dtype=torch.float32)
    _lib.call("pipnet_colsum_f32", a.data_ptr(), a.stride(0), m, n, out.data_ptr(), int(accumulate), ws.data_ptr(),
              _stream(a))
    return out


def _partials(c: int, device) -> Tensor:
    return torch.empty(int(_lib.load().pipnet_train_partials_floats(c)), device=device, dtype=torch.float32)


def gelu_fwd(h: Tensor) -> Tensor:
    _chk(h, "gelu input")
    g = torch.empty_like(h)
    _lib.call("pipnet_gelu_fwd_f32", h.data_ptr(), g.data_ptr(), h.numel(), _stream(h))
    return g


def resid_scale(x: Tensor, y2: Tensor, ls: Tensor, row_scale: Optional[Tensor], rows_per_scale: int,
                out: Optional[Tensor] = None) -> Tensor:
    """out = x + row_scale[m // rows_per_scale] * (ls * y2) on [M, C] rows."""
    for t, what in ((x, "residual"), (y2, "branch"), (ls, "layer scale")):
        _chk(t, what)
    m, c = x.shape
    out = torch.empty_like(x) if out is None else out
    _lib.call("pipnet_resid_scale_f32", x.data_ptr(), y2.data_ptr(), ls.data_ptr(), _ptr(row_scale), rows_per_scale,
              m, c, out.data_ptr(), _stream(x))
    return out


def ls_backward(dy: Tensor, y2: Tensor, ls: Tensor, row_scale: Optional[Tensor], rows_per_scale: int,
                d_ls: Tensor, d_b2: Tensor, accumulate: bool = False) -> Tensor:
    """Backward of resid_scale w.r.t. y2 (returned), ls and the Linear2 bias (into d_ls / d_b2)."""
    _chk(dy, "dy")
    _chk(y2, "y2")
    m, c = dy.shape
    dy2 = torch.empty_like(dy)
    _lib.call("pipnet_ls_bwd_f32", dy.data_ptr(), y2.data_ptr(), ls.data_ptr(), _ptr(row_scale), rows_per_scale, m, c,
              dy2.data_ptr(), d_ls.data_ptr(), d_b2.data_ptr(), int(accumulate), _partials(c, dy.device).data_ptr(),
              _stream(dy))
    return dy2


def ln_backward(z: Tensor, dt: Tensor, gamma: Tensor, d_gamma: Tensor, d_beta: Tensor, want_dz: bool = True,
                accumulate: bool = False) -> Optional[Tensor]:
    """LayerNorm(C, eps 1e-6) backward from the pre-norm rows z [M, C]."""
    _chk(z, "LN input")
    _chk(dt, "LN output gradient")
    m, c = z.shape
    dz = torch.empty_like(z) if want_dz else None
    _lib.call("pipnet_ln_bwd_f32", z.data_ptr(), dt.data_ptr(), gamma.data_ptr(), m, c, _ptr(dz), d_gamma.data_ptr(),
              d_beta.data_ptr(), int(accumulate), _partials(c, z.device).data_ptr(), _stream(z))
    return dz


def dwconv7_plain(x_nhwc: Tensor, w_packed: Tensor, bias: Optional[Tensor], out: Optional[Tensor] = None,
                  accumulate: bool = False) -> Tensor:
    """(out +)= [bias] + depthwise 7x7 pad 3 of x (w_packed [49, C])."""
    _chk(x_nhwc, "dwconv input")
    b, h, w, c = x_nhwc.shape
    out = torch.empty_like(x_nhwc) if out is None else out
    _lib.call("pipnet_dwconv7_plain_f32", x_nhwc.data_ptr(), b, h, w, c, w_packed.data_ptr(), _ptr(bias),
              int(accumulate), out.data_ptr(), _stream(x_nhwc))
    return out


def dwconv7_wgrad(dz_nhwc: Tensor, x_nhwc: Tensor, dw_packed: Tensor, db: Tensor, accumulate: bool = False) -> None:
    b, h, w, c = x_nhwc.shape
    _lib.call("pipnet_dwconv7_wgrad_f32", dz_nhwc.data_ptr(), x_nhwc.data_ptr(), b, h, w, c, dw_packed.data_ptr(),
              db.data_ptr(), int(accumulate), _partials(c, x_nhwc.device).data_ptr(), _stream(x_nhwc))


def wgrad_conv(dy_nhwc: Tensor, x_nhwc: Tensor, kh: int, kw: int, stride: int, out: Tensor,
               accumulate: bool = False, pad: int = 0) -> Tensor:
    """Packed [Cout, KH*KW*Cin] weight gradient of a KHxKW conv (stride, zero padding)."""
    _chk(dy_nhwc, "d conv output")
    _chk(x_nhwc, "conv input")
    b, h, w, cin = x_nhwc.shape
    cout = dy_nhwc.shape[-1]
    oh, ow = (h + 2 * pad - kh) // stride + 1, (w + 2 * pad - kw) // stride + 1
    if tuple(dy_nhwc.shape) != (b, oh, ow, cout) or out.numel() != cout * kh * kw * cin:
        raise RuntimeError(f"wgrad_conv: dY {tuple(dy_nhwc.shape)}, x {tuple(x_nhwc.shape)}, k{kh}x{kw}/{stride}")
    nbytes = _lib.load().pipnet_wgrad_workspace_bytes(b * oh * ow, cout, kh * kw * cin)
    ws = torch.empty(max(nbytes // 4, 1), device=x_nhwc.device, dtype=torch.float32)
    _lib.call("pipnet_wgrad_conv_f32", dy_nhwc.data_ptr(), x_nhwc.data_ptr(), b, h, w, cin, kh, kw, stride, pad, cout,
              out.data_ptr(), int(accumulate), ws.data_ptr(), _stream(x_nhwc))
    return out


def wgrad_conv2x2(dy_nhwc: Tensor, x_nhwc: Tensor, stride: int, out: Tensor, accumulate: bool = False) -> Tensor:
    """Packed [Cout, 4*Cin] weight gradient of the 2x2 downsample conv."""
    b, h, w, cin = x_nhwc.shape
    cout = dy_nhwc.shape[-1]
    nbytes = _lib.load().pipnet_wgrad_workspace_bytes(dy_nhwc.numel() // cout, cout, 4 * cin)
    ws = torch.empty(max(nbytes // 4, 1), device=x_nhwc.device, dtype=torch.float32)
    _lib.call("pipnet_wgrad_conv2x2_f32", dy_nhwc.data_ptr(), x_nhwc.data_ptr(), b, h, w, cin, stride, cout,
              out.data_ptr(), int(accumulate), ws.data_ptr(), _stream(x_nhwc))
    return out


def head_backward(proto_nhwc: Tensor, pooled: Tensor, d_out: Optional[Tensor], w: Optional[Tensor],
                  w_align: float, w_tanh: float, tanh_coeff: float = 1.0) -> Tensor:
    """d loss / d logits of the PIP-Net head (softmax + max-pool) for the align / tanh /
    classifier terms of calculate_loss (pipnet/train.py:154-265)."""
    _chk(proto_nhwc, "proto features")
    n, h, ww, p = proto_nhwc.shape
    d_logits = torch.empty_like(proto_nhwc)
    amax = torch.empty((n, p), device=proto_nhwc.device, dtype=torch.int32)
    dpool = torch.empty((n, p), device=proto_nhwc.device, dtype=torch.float32)
    k = 0 if w is None else w.shape[0]
    _lib.call("pipnet_head_bwd_f32", proto_nhwc.data_ptr(), pooled.data_ptr(), n // 2, h * ww, p, _ptr(d_out), _ptr(w),
              k, w_align, w_tanh, tanh_coeff, amax.data_ptr(), dpool.data_ptr(), d_logits.data_ptr(),
              _stream(proto_nhwc))
    return d_logits


# ---- ResNet training: BatchNorm2d in train mode (csrc/bn_ops.hip) ----------------------------
def _bn_ws(c: int, device) -> Tensor:
    return torch.empty(int(_lib.load().pipnet_bn_workspace_floats(c)), device=device, dtype=torch.float32)


def bn_stats(x: Tensor, eps: float, momentum: float, running_mean: Optional[Tensor] = None,
             running_var: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """Batch mean / invstd over the rows of NHWC ``x`` (train-mode BatchNorm2d); updates the
    running statistics in place when given (momentum, unbiased variance)."""
    _chk(x, "BN input")
    c = x.shape[-1]
    m = x.numel() // c
    mean = torch.empty(c, device=x.device, dtype=torch.float32)
    invstd = torch.empty_like(mean)
    for t, what in ((running_mean, "running_mean"), (running_var, "running_var")):
        if t is not None:
            _chk(t, what)
    _lib.call("pipnet_bn_stats_f32", x.data_ptr(), m, c, eps, momentum, mean.data_ptr(), invstd.data_ptr(),
              _ptr(running_mean), _ptr(running_var), _bn_ws(c, x.device).data_ptr(), _stream(x))
    if running_mean is not None:
        _mutated(running_mean, running_var)
    return mean, invstd


def bn_apply(x: Tensor, mean: Tensor, invstd: Tensor, gamma: Tensor, beta: Tensor, residual: Optional[Tensor] = None,
             relu: bool = False, out: Optional[Tensor] = None) -> Tensor:
    """gamma * (x - mean) * invstd + beta [+ residual] [ReLU] on NHWC rows."""
    _chk(x, "BN input")
    for t, what in ((gamma, "BN weight"), (beta, "BN bias")):
        _chk(t, what)
    if residual is not None:
        _chk(residual, "residual")
        if residual.shape != x.shape:
            raise RuntimeError(f"bn_apply: residual {tuple(residual.shape)} vs {tuple(x.shape)}")
    c = x.shape[-1]
    y = torch.empty_like(x) if out is None else out
    _lib.call("pipnet_bn_apply_f32", x.data_ptr(), x.numel() // c, c, mean.data_ptr(), invstd.data_ptr(),
              gamma.data_ptr(), beta.data_ptr(), _ptr(residual), int(relu), y.data_ptr(), _stream(x))
    return y


def bn_backward(x: Tensor, dy: Tensor, mean: Tensor, invstd: Tensor, gamma: Tensor, relu_out: Optional[Tensor] = None,
                want_dx: bool = True, want_masked: bool = False
                ) -> Tuple[Optional[Tensor], Optional[Tensor], Tensor, Tensor]:
    """Train-mode BatchNorm2d backward from the pre-norm rows ``x``; ``relu_out`` (the output of
    the ReLU that follows, when there is one) masks dy.  Returns (dx, masked dy, d_gamma, d_beta)."""
    _chk(x, "BN input")
    _chk(dy, "BN output gradient")
    if relu_out is not None:
        _chk(relu_out, "ReLU output")
    c = x.shape[-1]
    dx = torch.empty_like(x) if want_dx else None
    dm = torch.empty_like(x) if want_masked else None
    dg = torch.empty(c, device=x.device, dtype=torch.float32)
    db = torch.empty_like(dg)
    _lib.call("pipnet_bn_backward_f32", x.data_ptr(), dy.data_ptr(), _ptr(relu_out), x.numel() // c, c, mean.data_ptr(),
              invstd.data_ptr(), gamma.data_ptr(), _ptr(dx), _ptr(dm), dg.data_ptr(), db.data_ptr(),
              _bn_ws(c, x.device).data_ptr(), _stream(x))
    return dx, dm, dg, db


def stride_scatter(x: Tensor, h: int, w: int, stride: int, out: Optional[Tensor] = None,
                   accumulate: bool = False) -> Tensor:
    """NHWC [B, OH, OW, C] -> [B, h, w, C] with x on the stride lattice, zeros elsewhere
    (added into ``out`` when accumulate)."""
    _chk(x, "scatter input")
    b, oh, ow, c = x.shape
    if out is None:
        if accumulate:
            raise RuntimeError("stride_scatter: accumulate needs out")
        out = torch.empty((b, h, w, c), device=x.device, dtype=torch.float32)
    elif tuple(out.shape) != (b, h, w, c):
        raise RuntimeError(f"stride_scatter: out {tuple(out.shape)}")
    _lib.call("pipnet_stride_scatter_f32", x.data_ptr(), b, oh, ow, c, h, w, stride, int(accumulate), out.data_ptr(),
              _stream(x))
    return out
