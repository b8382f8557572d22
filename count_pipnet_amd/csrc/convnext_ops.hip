// ConvNeXt-tiny non-GEMM stages on gfx950, NHWC fp32 (HBM/VALU-bound, no MFMA shape):
//   * stem      Conv2d(3,96,k4,s4)+LayerNorm2d  -- reads the NCHW input directly
//   * dwconv7   depthwise 7x7 (+bias) fused with the CNBlock LayerNorm
//   * layernorm LayerNorm2d in front of each downsample conv
// torchvision semantics restated in SURVEY.md 2.3; the reference builds the net in
// features/convnext_features.py:38-94.
#include <algorithm>

#include "common.hpp"
#include "convnext_dw.hpp"

namespace {

constexpr float LN_EPS = 1e-6f;

// ---------------------------------------------------------------------------------------
// stem: the 4x4/s4 conv is a [96 x 48] x [48 x pixels] product -> fp32 MFMA 32x32x2 with the
// weights as the A operand, held in 72 VGPRs per lane for the wave's lifetime, and 32 pixels
// per tile as B.  D[channel][pixel] leaves each lane with 48 channels of ONE pixel (lanes l and
// l+32 share it), so LayerNorm2d is a per-lane sum plus one xor-32 shuffle.  (Replaced two
// VALU kernels -- weights broadcast from LDS, then from SGPRs -- whose operand latency left
// the C2 stem at 93-115 us; this one is MFMA/HBM-bound.)
// ---------------------------------------------------------------------------------------
constexpr int STEM_C = 96, STEM_K = 48, STEM_T = 256, STEM_TILE = 32;

// K order: MFMA step s = (ci*2 + u)*4 + kx sums kernel row ky = u (lanes 0-31) and ky = 2 + u
// (lanes 32-63), so each lane fetches whole 4-pixel input rows (6 float4 per tile) and its
// weights as 8 contiguous floats per (block, ci) (18 float4 per wave lifetime).
__global__ __launch_bounds__(STEM_T) __attribute__((amdgpu_waves_per_eu(2, 2))) void stem_kernel(const float* __restrict__ x, int B, int H, int W,
                                                      const float* __restrict__ w, const float* __restrict__ bias,
                                                      const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                      float* __restrict__ y, int64_t ntiles) {
  const int lane = threadIdx.x & 63, h = lane >> 5, n = lane & 31;
  const int OH = H / 4, OW = W / 4;
  const int64_t npx = (int64_t)B * OH * OW;
  float wa[3][24];                                   // A operand: w[32*blk + n][ci*16 + (2h+u)*4 + kx]
#pragma unroll
  for (int blk = 0; blk < 3; ++blk)
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const f32x4 v = ld4(w + (32 * blk + n) * STEM_K + ci * 16 + (2 * h + u) * 4);
#pragma unroll
        for (int kx = 0; kx < 4; ++kx) wa[blk][(ci * 2 + u) * 4 + kx] = v[kx];
      }
  // bias / LayerNorm affine in LDS: their per-tile reads must not sit in the vmcnt queue behind
  // the next tile's prefetch (vmcnt retires in order), nor be hoisted into 144 VGPRs
  __shared__ __attribute__((aligned(16))) float vec_sm[3 * STEM_C];
  for (int i = threadIdx.x; i < 3 * STEM_C; i += STEM_T)
    vec_sm[i] = i < STEM_C ? bias[i] : i < 2 * STEM_C ? lnw[i - STEM_C] : lnb[i - 2 * STEM_C];
  __syncthreads();
  const int64_t nwaves = (int64_t)gridDim.x * (STEM_T / 64);
  // B operand: x[pixel n][ci][2h + u][kx] as xv[ci*2 + u][kx].  Lanes past the last pixel load
  // the last pixel instead (branch-free, so the prefetch stays where it is issued); a D column
  // only ever feeds its own pixel's LayerNorm and store, so those lanes' results are dropped.
  auto load_tile = [&](int64_t tile, f32x4 (&xv)[6]) {
    const int64_t p = std::min<int64_t>(tile * STEM_TILE + n, npx - 1);
    const int b = (int)(p / ((int64_t)OH * OW));
    const int rem = (int)(p - (int64_t)b * OH * OW);
    const int oy = rem / OW, ox = rem - oy * OW;
    const float* src = x + (((int64_t)b * 3) * H + 4 * oy + 2 * h) * W + 4 * ox;
#pragma unroll
    for (int ci = 0; ci < 3; ++ci)
#pragma unroll
      for (int u = 0; u < 2; ++u) xv[ci * 2 + u] = ld4(src + ((int64_t)ci * H + u) * W);
  };
  int64_t tile = (int64_t)blockIdx.x * (STEM_T / 64) + (threadIdx.x >> 6);
  f32x4 xv[6];
  load_tile(tile, xv);
  for (; tile < ntiles; tile += nwaves) {
    const int64_t p = tile * STEM_TILE + n;
    const bool ok = p < npx;
    int z = 0;                                       // opaque 0: keeps the LDS reads per tile
    asm volatile("" : "+v"(z));
    const float* bias_t = vec_sm + z;
    const float* lnw_t = vec_sm + STEM_C + z;
    const float* lnb_t = vec_sm + 2 * STEM_C + z;
    float xb[24];
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) xb[q * 4 + kx] = xv[q][kx];
    load_tile(tile + nwaves, xv);                    // next tile's loads fly under this one's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    f32x16 acc[3];
#pragma unroll
    for (int blk = 0; blk < 3; ++blk)
#pragma unroll
      for (int j = 0; j < 4; ++j) {                  // D row (channel) 32*blk + 8j + 4h + i
        const f32x4 bv = ld4(bias_t + 32 * blk + 8 * j + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[blk][4 * j + i] = bv[i];
      }
#pragma unroll
    for (int k = 0; k < 24; ++k)
#pragma unroll
      for (int blk = 0; blk < 3; ++blk)
        acc[blk] = __builtin_amdgcn_mfma_f32_32x32x2f32(wa[blk][k], xb[k], acc[blk], 0, 0, 0);
    float s = 0.f;
#pragma unroll
    for (int blk = 0; blk < 3; ++blk)
#pragma unroll
      for (int i = 0; i < 16; ++i) s += acc[blk][i];
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.0f / STEM_C);
    float qq = 0.f;
#pragma unroll
    for (int blk = 0; blk < 3; ++blk)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float d = acc[blk][i] - mean;
        qq = fmaf(d, d, qq);
      }
    qq += __shfl_xor(qq, 32, 64);
    const float rstd = 1.0f / sqrtf(qq * (1.0f / STEM_C) + LN_EPS);
    if (ok) {
      float* dst = y + p * STEM_C;
#pragma unroll
      for (int blk = 0; blk < 3; ++blk)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 32 * blk + 8 * j + 4 * h;
          const f32x4 gw = ld4(lnw_t + c), gb = ld4(lnb_t + c);
          f32x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (acc[blk][4 * j + i] - mean) * rstd * gw[i] + gb[i];
          st4(dst + c, o);
        }
    }
  }
}

// ---------------------------------------------------------------------------------------
// row LayerNorm: one wave per row of C channels.
// ---------------------------------------------------------------------------------------
template <int NJ, bool S3 = false>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t rows, int C,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        void* __restrict__ yv) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* src = x + row * C;
  float v[NJ];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < C ? src[c] : 0.f;
    s += v[j];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    const float d = c < C ? v[j] - mean : 0.f;
    q = fmaf(d, d, q);
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)C + LN_EPS);
  if constexpr (S3) {                      // split-bf16 planes [hi | lo]
    __bf16* dst = reinterpret_cast<__bf16*>(yv) + row * 2 * C;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < C) {
        __bf16 hi, lo;
        split_bf16((v[j] - mean) * rstd * w[c] + b[c], hi, lo);
        dst[c] = hi;
        dst[C + c] = lo;
      }
    }
  } else {
    float* dst = reinterpret_cast<float*>(yv) + row * C;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < C) dst[c] = (v[j] - mean) * rstd * w[c] + b[c];
    }
  }
}

}  // namespace

extern "C" int pipnet_convnext_stem_f32(const float* x, int B, int H, int W, const float* w, const float* b,
                                        const float* ln_w, const float* ln_b, float* y, void* stream) {
  if (B < 0 || H < 4 || W < 4 || (H & 3) || (W & 3)) return PIPNET_ERR_ARG;
  if (!x || !w || !b || !ln_w || !ln_b || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w) || !aligned16(y) || !aligned16(b) || !aligned16(ln_w) || !aligned16(ln_b))
    return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int64_t npx = (int64_t)B * (H / 4) * (W / 4);
  const int64_t ntiles = (npx + STEM_TILE - 1) / STEM_TILE;
  // at most 2 waves per SIMD (its occupancy), each looping over tiles with the weights in registers
  const int64_t grid = std::min<int64_t>((ntiles + STEM_T / 64 - 1) / (STEM_T / 64), 256 * 2);
  hipLaunchKernelGGL(stem_kernel, dim3((unsigned)grid), dim3(STEM_T), 0, (hipStream_t)stream,
                     x, B, H, W, w, b, ln_w, ln_b, y, ntiles);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// LayerNorm lanes per pixel = C / 12: each lane owns 3 float4 channel chunks, gamma / beta in
// registers, full-line stores (tools/dw_lab.hip, profiles/r02/dw_lab.txt: 64 -> 63 / 37 -> 35 /
// 59 -> 56 / 90 -> 85 us at the C2 stages).  Small maps take narrower column tiles (a row tile of
// G * 7 pixels left 43 % of the lanes idle at W = 32 / 16): C5 stage 1 36.7 -> 26.2 us, stage 2
// 18.2 -> 16.9 us; at C1's 16^2 / 8^2 maps (batch 16) the wide tile stays 2 % faster, hence the
// lower bounds.  Round 4: with each weight row loaded once per workgroup (convnext_dw.hpp),
// taller tiles (TY = 2-4 output rows) cut the vector-L1 traffic of the weights and the 7-row
// input halo: C2 stages 68 -> 49 (96 @ 56^2), 34 -> 29 (192 @ 28^2), 56 -> 47 us (384 @ 27^2),
// C5 stages 25 -> 17.5 (96 @ 32^2), 17 -> 12.4 us (192 @ 16^2); 768 @ 26^2 keeps TY = 1
// (profiles/r04/dw_window_lab.txt).  Every tile sums the same 49 products in the same order:
// bitwise equal outputs.  The choice depends on W only (per-pixel results stay batch-invariant).
extern "C" int pipnet_dwconv7_ln_f32(const float* x, int B, int H, int W, int C, const float* w_packed,
                                     const float* bias, const float* ln_w, const float* ln_b, float* y,
                                     void* stream) {
  if (B < 0 || H <= 0 || W <= 0) return PIPNET_ERR_ARG;
  if (!x || !w_packed || !bias || !ln_w || !ln_b || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(bias) || !aligned16(ln_w) || !aligned16(ln_b) ||
      !aligned16(y))
    return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (C) {
    case 96:
      if (W > 16 && W <= 32) return pipnet_dw::launch_dw<96, 4, 4, 1, false, 8>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      if (W > 32) return pipnet_dw::launch_dw<96, 7, 2, 1, false, 8>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      return pipnet_dw::launch_dw<96, 7, 1, 1, false, 8>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 192:
      if (W > 8 && W <= 16) return pipnet_dw::launch_dw<192, 4, 2, 1, false, 16>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      if (W > 16) return pipnet_dw::launch_dw<192, 7, 2, 1, false, 16>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      return pipnet_dw::launch_dw<192, 7, 1, 1, false, 16>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 384: return pipnet_dw::launch_dw<384, 7, 3, 1, false, 32>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 768: return pipnet_dw::launch_dw<768, 13, 1, 1>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    default: return PIPNET_ERR_ARG;
  }
}

extern "C" int pipnet_dwconv7_ln_s3(const float* x, int B, int H, int W, int C, const float* w_packed,
                                    const float* bias, const float* ln_w, const float* ln_b, void* y, void* stream) {
  if (B < 0 || H <= 0 || W <= 0) return PIPNET_ERR_ARG;
  if (!x || !w_packed || !bias || !ln_w || !ln_b || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(bias) || !aligned16(ln_w) || !aligned16(ln_b) ||
      !aligned16(y))
    return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (C) {
    case 96:
      if (W > 16 && W <= 32) return pipnet_dw::launch_dw<96, 4, 4, 1, true, 8>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      if (W > 32) return pipnet_dw::launch_dw<96, 7, 2, 1, true, 8>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      return pipnet_dw::launch_dw<96, 7, 1, 1, true, 8>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 192:
      if (W > 8 && W <= 16) return pipnet_dw::launch_dw<192, 4, 2, 1, true, 16>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      if (W > 16) return pipnet_dw::launch_dw<192, 7, 2, 1, true, 16>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
      return pipnet_dw::launch_dw<192, 7, 1, 1, true, 16>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 384: return pipnet_dw::launch_dw<384, 7, 3, 1, true, 32>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 768: return pipnet_dw::launch_dw<768, 13, 1, 1, true>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    default: return PIPNET_ERR_ARG;
  }
}

extern "C" int pipnet_layernorm_s3(const float* x, int64_t rows, int C, const float* w, const float* b, void* y,
                                   void* stream) {
  if (rows < 0 || C <= 0 || C > 2048 || !x || !w || !b || !y) return PIPNET_ERR_ARG;
  if (rows == 0) return PIPNET_OK;
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const int nj = (C + 63) / 64;
  if (nj <= 2) hipLaunchKernelGGL((layernorm_kernel<2, true>), grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else if (nj <= 3) hipLaunchKernelGGL((layernorm_kernel<3, true>), grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else if (nj <= 6) hipLaunchKernelGGL((layernorm_kernel<6, true>), grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else if (nj <= 12) hipLaunchKernelGGL((layernorm_kernel<12, true>), grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else hipLaunchKernelGGL((layernorm_kernel<32, true>), grid, dim3(256), 0, s, x, rows, C, w, b, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_layernorm_f32(const float* x, int64_t rows, int C, const float* w, const float* b, float* y,
                                    void* stream) {
  if (rows < 0 || C <= 0 || C > 2048 || !x || !w || !b || !y) return PIPNET_ERR_ARG;
  if (rows == 0) return PIPNET_OK;
  const dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  const int nj = (C + 63) / 64;
  if (nj <= 2) hipLaunchKernelGGL(layernorm_kernel<2>, grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else if (nj <= 3) hipLaunchKernelGGL(layernorm_kernel<3>, grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else if (nj <= 6) hipLaunchKernelGGL(layernorm_kernel<6>, grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else if (nj <= 12) hipLaunchKernelGGL(layernorm_kernel<12>, grid, dim3(256), 0, s, x, rows, C, w, b, y);
  else hipLaunchKernelGGL(layernorm_kernel<32>, grid, dim3(256), 0, s, x, rows, C, w, b, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
