// ResNet backbone helpers on gfx950 (HBM-bound, NHWC fp32): input relayout and max-pool.
// The convolutions themselves are the implicit-GEMM MFMA kernels of gemm_f32_impl.hpp
// (pipnet_conv2d_nhwc_f32); reference: features/resnet_features.py:126-229.
#include "common.hpp"

namespace {

// [B,C,H,W] -> [B,H,W,Cpad] (channels >= C zero).  One thread per output pixel-row chunk.
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x, int B, int C, int H, int W,
                                                           int Cpad, float* __restrict__ y) {
  const int64_t n = (int64_t)B * H * W;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / ((int64_t)H * W);
    const int64_t hw = i - b * H * W;
    float* dst = y + i * Cpad;
    for (int c = 0; c < Cpad; ++c) dst[c] = c < C ? x[(b * C + c) * H * W + hw] : 0.f;
  }
}

// MaxPool2d on NHWC: one thread per (output pixel, 4-channel quad); padding never wins
// (torch pads max-pool with -inf).
__global__ __launch_bounds__(256) void maxpool_nhwc_kernel(const float* __restrict__ x, int B, int H, int W, int C,
                                                           int k, int stride, int pad, int OH, int OW,
                                                           float* __restrict__ y) {
  const int QC = C / 4;
  const int64_t n = (int64_t)B * OH * OW * QC;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int q = (int)(i % QC);
    const int64_t pix = i / QC;
    const int ox = (int)(pix % OW);
    const int oy = (int)((pix / OW) % OH);
    const int64_t b = pix / ((int64_t)OW * OH);
    f32x4 m = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * stride - pad + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * stride - pad + kx;
        if (ix < 0 || ix >= W) continue;
        const f32x4 v = ld4(x + (((b * H + iy) * W + ix) * C) + 4 * q);
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], v[e]);
      }
    }
    st4(y + pix * C + 4 * q, m);
  }
}

int grid_for(int64_t n) { return (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192); }

}  // namespace

extern "C" int pipnet_nchw_to_nhwc_f32(const float* x, int B, int C, int H, int W, int Cpad, float* y,
                                       void* stream) {
  if (B < 0 || C <= 0 || H <= 0 || W <= 0 || Cpad < C || !x || !y) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for((int64_t)B * H * W)), dim3(256), 0, (hipStream_t)stream, x,
                     B, C, H, W, Cpad, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_maxpool2d_nhwc_f32(const float* x, int B, int H, int W, int C, int k, int stride, int pad,
                                         float* y, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || (C & 3) || k <= 0 || stride <= 0 || pad < 0 || 2 * pad > k) return PIPNET_ERR_ARG;
  if (!x || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(y)) return PIPNET_ERR_ALIGN;
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (B == 0) return PIPNET_OK;
  hipLaunchKernelGGL(maxpool_nhwc_kernel, dim3(grid_for((int64_t)B * OH * OW * (C / 4))), dim3(256), 0,
                     (hipStream_t)stream, x, B, H, W, C, k, stride, pad, OH, OW, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
