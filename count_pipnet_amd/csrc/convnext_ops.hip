// ConvNeXt-tiny non-GEMM stages on gfx950, NHWC fp32 (HBM/VALU-bound, no MFMA shape):
//   * stem      Conv2d(3,96,k4,s4)+LayerNorm2d  -- reads the NCHW input directly
//   * dwconv7   depthwise 7x7 (+bias) fused with the CNBlock LayerNorm
//   * layernorm LayerNorm2d in front of each downsample conv
// torchvision semantics restated in SURVEY.md 2.3; the reference builds the net in
// features/convnext_features.py:38-94.
#include "common.hpp"
#include "convnext_dw.hpp"

namespace {

constexpr float LN_EPS = 1e-6f;

// ---------------------------------------------------------------------------------------
// stem: one workgroup per (image, output row).  Input rows and transposed weights in LDS;
// thread = (4-channel quad, pixel group), float4 accumulators; the raw row goes back through
// LDS for the LayerNorm (one wave per pixel) so the NHWC row is written fully coalesced.
// ---------------------------------------------------------------------------------------
constexpr int STEM_C = 96, STEM_K = 48, STEM_Q = STEM_C / 4, STEM_G = 10, STEM_NPX = 6;
constexpr int STEM_OLD = STEM_C + 4;       // padded LDS row of the raw output tile

__global__ __launch_bounds__(256) void stem_kernel(const float* __restrict__ x, int H, int W,
                                                   const float* __restrict__ w, const float* __restrict__ bias,
                                                   const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                   float* __restrict__ y) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int OH = H / 4, OW = W / 4;
  float* wsm = sm;                                 // [48][96]  (k-major: float4 over channels)
  float* otile = wsm + STEM_K * STEM_C;            // [OW][100]
  float* xin = otile + OW * STEM_OLD;              // [3][4][W]
  const int b = blockIdx.x / OH, oy = blockIdx.x - (blockIdx.x / OH) * OH;
  const int tid = threadIdx.x;
  for (int i = tid; i < STEM_C * STEM_K; i += 256) {
    const int c = i / STEM_K, k = i - c * STEM_K;
    wsm[k * STEM_C + c] = w[i];
  }
  const int w4 = W / 4;
  for (int i = tid; i < 12 * w4; i += 256) {
    const int r = i / w4, xx = i - r * w4;          // r = c*4 + ky
    const int c = r >> 2, ky = r & 3;
    st4(xin + r * W + 4 * xx, ld4(x + (((int64_t)b * 3 + c) * H + 4 * oy + ky) * W + 4 * xx));
  }
  __syncthreads();
  const int q = tid % STEM_Q, g = tid / STEM_Q;
  if (g < STEM_G) {
    const f32x4 bq = ld4(bias + 4 * q);
    for (int px0 = g; px0 < OW; px0 += STEM_G * STEM_NPX) {
      f32x4 acc[STEM_NPX];
#pragma unroll
      for (int p = 0; p < STEM_NPX; ++p) acc[p] = bq;
#pragma unroll 4
      for (int k = 0; k < STEM_K; ++k) {
        const f32x4 wk = ld4(wsm + k * STEM_C + 4 * q);
        const float* xr = xin + (k >> 2) * W + (k & 3);   // (c*4+ky) row, kx column offset
#pragma unroll
        for (int p = 0; p < STEM_NPX; ++p) {
          const int px = px0 + p * STEM_G;
          const float v = px < OW ? xr[4 * px] : 0.f;
          acc[p] += v * wk;
        }
      }
#pragma unroll
      for (int p = 0; p < STEM_NPX; ++p) {
        const int px = px0 + p * STEM_G;
        if (px < OW) st4(otile + px * STEM_OLD + 4 * q, acc[p]);
      }
    }
  }
  __syncthreads();
  const int lane = tid & 63, wv = tid >> 6;
  for (int px = wv; px < OW; px += 4) {
    const float v0 = otile[px * STEM_OLD + lane];
    const float v1 = lane < 32 ? otile[px * STEM_OLD + 64 + lane] : 0.f;
    const float mean = wave_sum(v0 + v1) * (1.0f / STEM_C);
    const float d0 = v0 - mean, d1 = lane < 32 ? v1 - mean : 0.f;
    const float rstd = 1.0f / sqrtf(wave_sum(d0 * d0 + d1 * d1) * (1.0f / STEM_C) + LN_EPS);
    float* dst = y + (((int64_t)b * OH + oy) * OW + px) * STEM_C;
    dst[lane] = d0 * rstd * lnw[lane] + lnb[lane];
    if (lane < 32) dst[64 + lane] = d1 * rstd * lnw[64 + lane] + lnb[64 + lane];
  }
}

// ---------------------------------------------------------------------------------------
// row LayerNorm: one wave per row of C channels.
// ---------------------------------------------------------------------------------------
template <int NJ>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int64_t rows, int C,
                                                        const float* __restrict__ w, const float* __restrict__ b,
                                                        float* __restrict__ y) {
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
  float* dst = y + row * C;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < C) dst[c] = (v[j] - mean) * rstd * w[c] + b[c];
  }
}

}  // namespace

extern "C" int pipnet_convnext_stem_f32(const float* x, int B, int H, int W, const float* w, const float* b,
                                        const float* ln_w, const float* ln_b, float* y, void* stream) {
  if (B < 0 || H < 4 || W < 4 || (H & 3) || (W & 3) || W > 960) return PIPNET_ERR_ARG;
  if (!x || !w || !b || !ln_w || !ln_b || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(y) || !aligned16(b)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const size_t shmem = (STEM_K * STEM_C + (W / 4) * STEM_OLD + 12 * W) * sizeof(float);
  hipLaunchKernelGGL(stem_kernel, dim3(B * (H / 4)), dim3(256), shmem, (hipStream_t)stream, x, H, W, w, b, ln_w,
                     ln_b, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_dwconv7_ln_f32(const float* x, int B, int H, int W, int C, const float* w_packed,
                                     const float* bias, const float* ln_w, const float* ln_b, float* y,
                                     void* stream) {
  if (B < 0 || H <= 0 || W <= 0) return PIPNET_ERR_ARG;
  if (!x || !w_packed || !bias || !ln_w || !ln_b || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(bias)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  switch (C) {
    case 96: return pipnet_dw::launch_dw<96, 7, 1, 1>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 192: return pipnet_dw::launch_dw<192, 7, 1, 1>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 384: return pipnet_dw::launch_dw<384, 7, 1, 2>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    case 768: return pipnet_dw::launch_dw<768, 13, 1, 1>(x, B, H, W, w_packed, bias, ln_w, ln_b, y, s);
    default: return PIPNET_ERR_ARG;
  }
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
