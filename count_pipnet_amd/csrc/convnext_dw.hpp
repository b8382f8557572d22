// depthwise 7x7 + LayerNorm(C) kernel template (shared by convnext_ops.hip and tools/dw_lab.hip)
#pragma once
#include "common.hpp"

namespace pipnet_dw {

constexpr float LN_EPS = 1e-6f;
constexpr int DW_THREADS = 192;

// LayerNorm + store of npix buffered pixels (LDS, C floats each, row-major NP per output
// row): C/12 lanes per pixel, each owning 3 float4 channel chunks (sl, sl + C/12, sl + C/6),
// so one store instruction writes C/12 * 16 B contiguous of a pixel (a full 128 B line at
// C = 96); gamma / beta stay in registers; two-pass mean / variance as torch.
template <int C, bool S3, int ABL = 0>
__device__ __forceinline__ void ln_rows_vec(const float* tile, int npix, int NP, int b, int H, int W, int oy0,
                                            int xblk, const float* __restrict__ lnw, const float* __restrict__ lnb,
                                            void* __restrict__ yv) {
  constexpr int LPP = C / 12, PPW = 64 / LPP;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int sub = lane / LPP, sl = lane % LPP;
  f32x4 g[3], be[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    g[j] = ld4(lnw + 4 * (sl + LPP * j));
    be[j] = ld4(lnb + 4 * (sl + LPP * j));
  }
  for (int base = wv * PPW; base < npix; base += nw * PPW) {
    const int pp = base + sub;
    const int t = pp / NP, pix = pp - t * NP;
    const int ox = xblk + pix, oy = oy0 + t;
    const bool ok = pp < npix && ox < W && oy < H;
    f32x4 v[3];
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      v[j] = ok ? ld4(tile + pp * C + 4 * (sl + LPP * j)) : f32x4{0.f, 0.f, 0.f, 0.f};
      sm += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    }
#pragma unroll
    for (int o = LPP / 2; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
    float rstd = 1.0f;
    if constexpr ((ABL & 1) == 0) {        // ABL 1 (lab): no LayerNorm statistics / shuffles
      const float mean = sm * (1.0f / C);
      float qq = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        v[j] -= mean;
#pragma unroll
        for (int e = 0; e < 4; ++e) qq = fmaf(v[j][e], v[j][e], qq);
      }
#pragma unroll
      for (int o = LPP / 2; o > 0; o >>= 1) qq += __shfl_xor(qq, o, 64);
      rstd = 1.0f / sqrtf(qq * (1.0f / C) + LN_EPS);
    }
    if (!ok) continue;
    const int64_t opix = ((int64_t)b * H + oy) * W + ox;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const f32x4 r = v[j] * rstd * g[j] + be[j];
      const int c = 4 * (sl + LPP * j);
      if constexpr ((ABL & 8) != 0) {       // ABL 8 (lab): no output stores (one that never fires)
        if (!(r[0] + r[1] + r[2] + r[3] == -1234.5f)) continue;
      }
      if constexpr (S3) {
        __bf16* dst = reinterpret_cast<__bf16*>(yv) + opix * 2 * C + c;
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split_bf16(r[e], hi[e], lo[e]);
        *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(hi);
        *reinterpret_cast<uint2*>(dst + C) = *reinterpret_cast<const uint2*>(lo);
      } else {
        st4(reinterpret_cast<float*>(yv) + opix * C + c, r);
      }
    }
  }
}

// 192 threads = G groups x (C/4) channel quads; group g computes a TY x TX tile of output
// pixels (TY rows, TX consecutive columns).  Each input row of the 7-row halo is loaded
// once into registers (TX+6 float4) and feeds every output row it touches; the raw tile
// then goes through LDS for the per-pixel LayerNorm (one wave per pixel, two-pass
// mean / variance, coalesced NHWC stores).  1-D grid, XCD-contiguous, so the halo rows of
// neighbouring workgroups are served from one L2.  S3: the output is written as split-bf16
// planes [hi | lo] (2C bf16 per pixel, the A operand of the split-bf16 Linear1).
// ABL (tuning lab only, tools/dw_lab.hip variants 60+; 0 in the product): 1 = no LayerNorm statistics,
// 2 = one stencil FMA per input row instead of 7 x TX, 4 = no input loads (a lane-dependent constant),
// 8 = no output stores, 16 = no weight loads, 32 = no LDS tile round trip (stale LDS): timing only.
// (The body is a device function so that the product kernel's name carries no lab parameter.)
template <int C, int TX, int TY, bool S3, int LPP, int ABL>
__device__ __forceinline__ void dwconv7_ln_body(const float* __restrict__ x, int H, int W,
                                                const float* __restrict__ wp, const float* __restrict__ bias,
                                                const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                void* __restrict__ yv) {
  constexpr int QC = C / 4;
  constexpr int G = DW_THREADS / QC;
  constexpr int NP = G * TX;
  __shared__ __attribute__((aligned(16))) float tile[TY * NP * C];

  const int tid = threadIdx.x;
  const int q = tid % QC, g = tid / QC;
  const int nxb = (W + NP - 1) / NP;
  const int nyb = (H + TY - 1) / TY;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int xb = lin % nxb;
  const int oy0 = ((lin / nxb) % nyb) * TY;
  const int b = lin / (nxb * nyb);
  const int xblk = xb * NP;
  const int px0 = xblk + g * TX;

  const f32x4 bq = ld4(bias + 4 * q);
  f32x4 acc[TY][TX];
#pragma unroll
  for (int t = 0; t < TY; ++t)
#pragma unroll
    for (int i = 0; i < TX; ++i) acc[t][i] = bq;

  // Input rows through a buffer resource spanning exactly one image row (W*C floats): the
  // hardware range check returns zeros for the columns left / right of the image (a negative
  // offset wraps past num_records), so the 7x7 halo needs no per-load branch or select -- a
  // per-element "load or zero" made hipcc branch around every load (exec-masked blocks) and
  // spend more issue slots on 64-bit address arithmetic than on the FMAs.
  const int voff0 = ((px0 - 3) * C + 4 * q) * 4;
  // Weight row ky is loaded once, at input row ir = ky, and stays in registers for the TY
  // output rows that use it (input rows ir = ky .. ky + TY - 1): with TY > 1 a per-use load
  // re-read every weight TY times through the vector L1 -- the loads, not the FMAs, fill the
  // L1 / TA path of this kernel.  Same FMA order: bitwise the per-use form's result.
  f32x4 wrow[7][7];
#pragma unroll
  for (int ir = 0; ir < TY + 6; ++ir) {
    if (ir < 7) {
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        if constexpr ((ABL & 16) != 0) wrow[ir][kx] = f32x4{0.5f, 0.25f, 0.125f, 1.0f} * (float)(kx + 1);
        else wrow[ir][kx] = ld4(wp + (ir * 7 + kx) * C + 4 * q);
      }
    }
    const int iy = oy0 + ir - 3;
    if (iy < 0 || iy >= H) continue;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + (((int64_t)b * H + iy) * W) * C), (short)0, W * C * 4, 0x00020000);
    f32x4 v[TX + 6];
#pragma unroll
    for (int r = 0; r < TX + 6; ++r) {
      if constexpr ((ABL & 4) != 0) v[r] = f32x4{1.f, 2.f, 3.f, 4.f} * (float)(voff0 + r + iy);
      else v[r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff0 + r * C * 4, 0, 0));
    }
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      const int ky = ir - t;
      if (ky < 0 || ky >= 7) continue;
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        if constexpr ((ABL & 2) != 0) {
          if (kx > 0) continue;
        }
        const f32x4 wk = wrow[ky][kx];
#pragma unroll
        for (int px = 0; px < TX; ++px) acc[t][px] += v[px + kx] * wk;
      }
      if constexpr ((ABL & 2) != 0) {                  // keep every loaded column live
#pragma unroll
        for (int px = 0; px < TX; ++px) acc[t][px] += v[px + 6];
      }
    }
  }
  if constexpr ((ABL & 32) == 0) {
#pragma unroll
    for (int t = 0; t < TY; ++t)
#pragma unroll
      for (int i = 0; i < TX; ++i) st4(tile + (t * NP + g * TX + i) * C + 4 * q, acc[t][i]);
    __syncthreads();
  } else {                                           // keep every accumulator live; no round trip
    f32x4 keep = acc[0][0];
#pragma unroll
    for (int t = 0; t < TY; ++t)
#pragma unroll
      for (int i = 0; i < TX; ++i) keep += acc[t][i];
    if (keep[0] + keep[1] + keep[2] + keep[3] == -1234.5f) tile[tid] = 0.f;
  }

  if constexpr (LPP * 12 == C) {
    ln_rows_vec<C, S3, ABL>(tile, TY * NP, NP, b, H, W, oy0, xblk, lnw, lnb, yv);
    return;
  }
  // LayerNorm: LPP lanes per pixel (64 / LPP pixels per wave at once, log2(LPP)-step
  // shuffle reductions -- one pixel per wave (LPP = 64) serialised two 6-step reductions
  // per pixel); two-pass mean / variance as torch
  constexpr int PPW = 64 / LPP;                 // pixels per wave per pass
  constexpr int CJ = (C + LPP - 1) / LPP;       // channels per lane
  const int lane = tid & 63, wv = tid >> 6;
  const int sub = lane / LPP, sl = lane % LPP;
  for (int base = wv * PPW; base < TY * NP; base += (DW_THREADS / 64) * PPW) {
    const int pp = base + sub;
    const int t = pp / NP, pix = pp - t * NP;
    const int ox = xblk + pix, oy = oy0 + t;
    const bool ok = pp < TY * NP && ox < W && oy < H;   // lane-group uniform; every lane shuffles
    float vv[CJ];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < CJ; ++j) {
      const int c = sl + LPP * j;
      vv[j] = (ok && c < C) ? tile[pp * C + c] : 0.f;
      s += vv[j];
    }
#pragma unroll
    for (int o = LPP / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.0f / C);
    float qq = 0.f;
#pragma unroll
    for (int j = 0; j < CJ; ++j) {
      const int c = sl + LPP * j;
      const float d = (c < C) ? vv[j] - mean : 0.f;
      qq = fmaf(d, d, qq);
    }
#pragma unroll
    for (int o = LPP / 2; o > 0; o >>= 1) qq += __shfl_xor(qq, o, 64);
    const float rstd = 1.0f / sqrtf(qq * (1.0f / C) + LN_EPS);
    if (!ok) continue;
    const int64_t opix = ((int64_t)b * H + oy) * W + ox;
    if constexpr (S3) {
      __bf16* dst = reinterpret_cast<__bf16*>(yv) + opix * 2 * C;
#pragma unroll
      for (int j = 0; j < CJ; ++j) {
        const int c = sl + LPP * j;
        if (c < C) {
          __bf16 hi, lo;
          split_bf16((vv[j] - mean) * rstd * lnw[c] + lnb[c], hi, lo);
          dst[c] = hi;
          dst[C + c] = lo;
        }
      }
    } else {
      float* dst = reinterpret_cast<float*>(yv) + opix * C;
#pragma unroll
      for (int j = 0; j < CJ; ++j) {
        const int c = sl + LPP * j;
        if (c < C) dst[c] = (vv[j] - mean) * rstd * lnw[c] + lnb[c];
      }
    }
  }
}

template <int C, int TX, int TY, int MINB, bool S3 = false, int LPP = 64>
__global__ __launch_bounds__(DW_THREADS, MINB) void dwconv7_ln_kernel(const float* __restrict__ x, int H, int W,
                                                                      const float* __restrict__ wp,
                                                                      const float* __restrict__ bias,
                                                                      const float* __restrict__ lnw,
                                                                      const float* __restrict__ lnb,
                                                                      void* __restrict__ yv) {
  dwconv7_ln_body<C, TX, TY, S3, LPP, 0>(x, H, W, wp, bias, lnw, lnb, yv);
}

template <int C, int TX, int TY, int MINB, int LPP, int ABL>   // tuning lab only (tools/dw_lab.hip)
__global__ __launch_bounds__(DW_THREADS, MINB) void dwconv7_ln_abl_kernel(const float* __restrict__ x, int H, int W,
                                                                          const float* __restrict__ wp,
                                                                          const float* __restrict__ bias,
                                                                          const float* __restrict__ lnw,
                                                                          const float* __restrict__ lnb,
                                                                          void* __restrict__ yv) {
  dwconv7_ln_body<C, TX, TY, false, LPP, ABL>(x, H, W, wp, bias, lnw, lnb, yv);
}

template <int C, int TX, int TY, int MINB, int LPP, int ABL>
inline int launch_dw_abl(const float* x, int B, int H, int W, const float* wp, const float* bias, const float* lnw,
                         const float* lnb, void* y, hipStream_t s) {
  constexpr int NP = (DW_THREADS / (C / 4)) * TX;
  const dim3 grid(((W + NP - 1) / NP) * ((H + TY - 1) / TY) * B);
  hipLaunchKernelGGL((dwconv7_ln_abl_kernel<C, TX, TY, MINB, LPP, ABL>), grid, dim3(DW_THREADS), 0, s, x, H, W, wp,
                     bias, lnw, lnb, y);
  return hipGetLastError() == hipSuccess ? PIPNET_OK : PIPNET_ERR_LAUNCH;
}

template <int C, int TX, int TY, int MINB, bool S3 = false, int LPP = 64>
inline int launch_dw(const float* x, int B, int H, int W, const float* wp, const float* bias, const float* lnw,
                     const float* lnb, void* y, hipStream_t s) {
  constexpr int NP = (DW_THREADS / (C / 4)) * TX;
  const dim3 grid(((W + NP - 1) / NP) * ((H + TY - 1) / TY) * B);
  hipLaunchKernelGGL((dwconv7_ln_kernel<C, TX, TY, MINB, S3, LPP>), grid, dim3(DW_THREADS), 0, s, x, H, W, wp, bias, lnw,
                     lnb, y);
  return hipGetLastError() == hipSuccess ? PIPNET_OK : PIPNET_ERR_LAUNCH;
}

}  // namespace pipnet_dw
