// Lab (round 4): depthwise 7x7 + LayerNorm with the LayerNorm applied in registers.  The conv part
// is the product tile's (convnext_dw.hpp, weight rows loaded once per workgroup); instead of
// re-laying the raw tile through LDS for a per-pixel LayerNorm pass, every thread reduces its
// own 4 channels per pixel, the per-pixel partials (one per channel quad) are summed through a
// small padded LDS array (two passes: mean, then sum of squared deviations, as torch), and each
// thread normalises and stores its channel quad straight from registers (lanes = consecutive
// channel quads: 16-B stores, whole lines).
#pragma once
#include "../count_pipnet_amd/csrc/convnext_dw.hpp"

namespace pipnet_dw {

template <int C, int TX, int TY, int MINB>
__global__ __launch_bounds__(DW_THREADS, MINB) void dwconv7_lnr_kernel(const float* __restrict__ x, int H, int W,
                                                                       const float* __restrict__ wp,
                                                                       const float* __restrict__ bias,
                                                                       const float* __restrict__ lnw,
                                                                       const float* __restrict__ lnb,
                                                                       float* __restrict__ y) {
  constexpr int QC = C / 4;
  constexpr int G = DW_THREADS / QC;
  constexpr int NP = G * TX;
  constexpr int NPIX = TY * NP;
  constexpr int QP = QC + 4;                          // padded partial row (bank spread)
  __shared__ __attribute__((aligned(16))) float part[NPIX * QP];
  __shared__ float stat[NPIX];

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
  const int voff0 = ((px0 - 3) * C + 4 * q) * 4;
  f32x4 wrow[7][7];
#pragma unroll
  for (int ir = 0; ir < TY + 6; ++ir) {
    if (ir < 7) {
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) wrow[ir][kx] = ld4(wp + (ir * 7 + kx) * C + 4 * q);
    }
    const int iy = oy0 + ir - 3;
    if (iy < 0 || iy >= H) continue;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + (((int64_t)b * H + iy) * W) * C), (short)0, W * C * 4, 0x00020000);
    f32x4 v[TX + 6];
#pragma unroll
    for (int r = 0; r < TX + 6; ++r)
      v[r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff0 + r * C * 4, 0, 0));
#pragma unroll
    for (int t = 0; t < TY; ++t) {
      const int ky = ir - t;
      if (ky < 0 || ky >= 7) continue;
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        const f32x4 wk = wrow[ky][kx];
#pragma unroll
        for (int px = 0; px < TX; ++px) acc[t][px] += v[px + kx] * wk;
      }
    }
  }
  // ---- pass 1: per-pixel sums of the channel quads -> mean ----
#pragma unroll
  for (int t = 0; t < TY; ++t)
#pragma unroll
    for (int i = 0; i < TX; ++i) {
      const f32x4 a = acc[t][i];
      part[(t * NP + g * TX + i) * QP + q] = (a[0] + a[1]) + (a[2] + a[3]);
    }
  __syncthreads();
  for (int p = tid; p < NPIX; p += DW_THREADS) {
    const float* r = part + p * QP;
    float s = 0.f;
#pragma unroll 4
    for (int j = 0; j < QC; j += 4) {
      const f32x4 u = ld4(r + j);
      s += (u[0] + u[1]) + (u[2] + u[3]);
    }
    stat[p] = s * (1.0f / C);
  }
  __syncthreads();
  // ---- pass 2: sums of squared deviations -> rstd ----
  float mean[TY][TX];
#pragma unroll
  for (int t = 0; t < TY; ++t)
#pragma unroll
    for (int i = 0; i < TX; ++i) {
      mean[t][i] = stat[t * NP + g * TX + i];
      const f32x4 d = acc[t][i] - mean[t][i];
      acc[t][i] = d;
      part[(t * NP + g * TX + i) * QP + q] = fmaf(d[0], d[0], fmaf(d[1], d[1], fmaf(d[2], d[2], d[3] * d[3])));
    }
  __syncthreads();
  for (int p = tid; p < NPIX; p += DW_THREADS) {
    const float* r = part + p * QP;
    float s = 0.f;
#pragma unroll 4
    for (int j = 0; j < QC; j += 4) {
      const f32x4 u = ld4(r + j);
      s += (u[0] + u[1]) + (u[2] + u[3]);
    }
    stat[p] = 1.0f / sqrtf(s * (1.0f / C) + LN_EPS);
  }
  __syncthreads();
  const f32x4 gq = ld4(lnw + 4 * q), beq = ld4(lnb + 4 * q);
#pragma unroll
  for (int t = 0; t < TY; ++t) {
    const int oy = oy0 + t;
#pragma unroll
    for (int i = 0; i < TX; ++i) {
      const int ox = px0 + i;
      if (oy < H && ox < W) {
        const float rstd = stat[t * NP + g * TX + i];
        st4(y + (((int64_t)b * H + oy) * W + ox) * C + 4 * q, acc[t][i] * rstd * gq + beq);
      }
    }
  }
}

template <int C, int TX, int TY, int MINB>
inline int launch_dw_lnr(const float* x, int B, int H, int W, const float* wp, const float* bias, const float* lnw,
                         const float* lnb, float* y, hipStream_t s) {
  constexpr int NP = (DW_THREADS / (C / 4)) * TX;
  const dim3 grid(((W + NP - 1) / NP) * ((H + TY - 1) / TY) * B);
  hipLaunchKernelGGL((dwconv7_lnr_kernel<C, TX, TY, MINB>), grid, dim3(DW_THREADS), 0, s, x, H, W, wp, bias, lnw, lnb, y);
  return hipGetLastError() == hipSuccess ? PIPNET_OK : PIPNET_ERR_LAUNCH;
}

}  // namespace pipnet_dw
