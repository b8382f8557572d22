// Evaluation input transform on the GPU: the reference's
// transform_no_augment = Resize((h, w)) [+ Grayscale(3)] + ToTensor + Normalize
// (util/data.py:264-269, :314-321, :500-505, :537-542, :568-574) applied to a ragged batch of
// decoded RGB images (ImageFolder's pil_loader output), written straight into the NCHW fp32
// batch the backbone reads.
//
// Resize of a PIL image is Pillow's ImagingResample(BILINEAR) (torchvision forwards it), so
// this restates Pillow's integer arithmetic exactly (oracle/input_ref.py, pinned against
// Pillow 12.2.0 outputs):
//   * per output coordinate: taps [xmin, xmin + n) and weights computed in double exactly as
//     precompute_coeffs (triangle filter, support max(scale, 1)), normalised, then 22-bit
//     fixed point rounded half away from zero (normalize_coeffs_8bpc) -- resize_coeffs_kernel;
//   * two separable passes, each clip8((1 << 21) + sum(u8 * k) >> 22) to uint8: horizontal
//     first, vertical first for very tall images that shrink vertically (h > 100 w, oh < h),
//     a pass skipped when its axis keeps its size -- resize_normalize_kernel recomputes the
//     first pass per output pixel (ksize_v x ksize_h integer MACs, L1/L2 resident), so there is
//     no intermediate image in HBM and one launch covers images of any size;
//   * Grayscale(3): PIL convert('L') = (19595 R + 38470 G + 7471 B + 0x8000) >> 16;
//   * ToTensor + Normalize in fp32 with IEEE division: (u8 / 255 - mean) / std.
// HBM traffic per image: the decoded pixels (read ~once, taps hit L1/L2) + 12 B per output
// pixel (+3 B with the optional uint8 HWC copy).
#include "common.hpp"

namespace {

constexpr int PREC = 22;   // PRECISION_BITS = 32 - 8 - 2

__host__ __device__ inline int ksize_for(int in_size, int out_size) {
  const double scale = (double)((float)in_size - 0.0f) / out_size;
  const double support = scale < 1.0 ? 1.0 : scale;
  return (int)ceil(support) * 2 + 1;
}

__device__ inline double triangle(double x) {
  if (x < 0.0) x = -x;
  return x < 1.0 ? 1.0 - x : 0.0;
}

// Table row = (xmin, n, k[0..kmax)) for one output coordinate of one image axis.
// Layout: [B][out_h + out_w][2 + kmax] int32, vertical rows first.
__global__ __launch_bounds__(256) void resize_coeffs_kernel(const int32_t* __restrict__ sizes, int B, int out_h,
                                                            int out_w, int kmax, int32_t* __restrict__ table) {
#pragma clang fp contract(off)
  const int per = out_h + out_w;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * per) return;
  const int b = i / per;
  const int r = i - b * per;
  const bool vert = r < out_h;
  const int xx = vert ? r : r - out_h;
  const int in_size = sizes[2 * b + (vert ? 0 : 1)];
  const int out_size = vert ? out_h : out_w;
  int32_t* row = table + (int64_t)i * (2 + kmax);
  const double scale = (double)((float)in_size - 0.0f) / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double center = 0.0 + (xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > kmax) xmax = kmax;    // cannot happen (kmax >= ksize); keeps the row in bounds
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += triangle(((double)(x + xmin) - center + 0.5) * ss);
  for (int x = 0; x < kmax; ++x) {
    int32_t q = 0;
    if (x < xmax) {
      double w = triangle(((double)(x + xmin) - center + 0.5) * ss);
      if (ww != 0.0) w /= ww;
      const double f = w * (double)(1 << PREC);
      q = w < 0 ? (int32_t)(-0.5 + f) : (int32_t)(0.5 + f);
    }
    row[2 + x] = q;
  }
  row[0] = xmin;
  row[1] = xmax;
}

__device__ inline int clip8(int ss) {
  const int v = ss >> PREC;            // arithmetic shift, as Pillow's clip8 lookup
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// One thread per output pixel (b, y, x), x fastest: coalesced plane stores.
__global__ __launch_bounds__(256) void resize_normalize_kernel(
    const uint8_t* __restrict__ pix, const int64_t* __restrict__ offsets, const int32_t* __restrict__ sizes, int B,
    int out_h, int out_w, int kmax, const int32_t* __restrict__ table, int gray, float m0, float m1, float m2,
    float s0, float s1, float s2, float* __restrict__ out, uint8_t* __restrict__ out_u8) {
  const int64_t plane = (int64_t)out_h * out_w;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)B * plane) return;
  const int b = (int)(i / plane);
  const int rem = (int)(i - (int64_t)b * plane);
  const int y = rem / out_w;
  const int x = rem - y * out_w;
  const int h = sizes[2 * b], w = sizes[2 * b + 1];
  const uint8_t* img = pix + offsets[b];
  const int rs = 2 + kmax;
  const int32_t* tv = table + ((int64_t)b * (out_h + out_w) + y) * rs;           // vertical row y
  const int32_t* th = table + ((int64_t)b * (out_h + out_w) + out_h + x) * rs;   // horizontal row x
  const bool need_h = w != out_w, need_v = h != out_h;
  int c3[3];
  if (!need_h && !need_v) {
    const uint8_t* p = img + ((int64_t)y * w + x) * 3;
    c3[0] = p[0], c3[1] = p[1], c3[2] = p[2];
  } else if (!need_v) {                  // horizontal pass only
    const int xmin = th[0], n = th[1];
    const uint8_t* p = img + ((int64_t)y * w + xmin) * 3;
    int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
    for (int t = 0; t < n; ++t) {
      const int k = th[2 + t];
      a0 += p[3 * t] * k, a1 += p[3 * t + 1] * k, a2 += p[3 * t + 2] * k;
    }
    c3[0] = clip8(a0), c3[1] = clip8(a1), c3[2] = clip8(a2);
  } else if (!need_h) {                  // vertical pass only
    const int ymin = tv[0], n = tv[1];
    int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
    for (int s = 0; s < n; ++s) {
      const uint8_t* p = img + ((int64_t)(ymin + s) * w + x) * 3;
      const int k = tv[2 + s];
      a0 += p[0] * k, a1 += p[1] * k, a2 += p[2] * k;
    }
    c3[0] = clip8(a0), c3[1] = clip8(a1), c3[2] = clip8(a2);
  } else if (h > 100 * w && out_h < h) {   // Pillow: vertical pass first for very tall images
    const int ymin = tv[0], nv = tv[1], xmin = th[0], nh = th[1];
    int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
    for (int t = 0; t < nh; ++t) {
      int v0 = 1 << (PREC - 1), v1 = v0, v2 = v0;
      for (int s = 0; s < nv; ++s) {
        const uint8_t* p = img + ((int64_t)(ymin + s) * w + xmin + t) * 3;
        const int k = tv[2 + s];
        v0 += p[0] * k, v1 += p[1] * k, v2 += p[2] * k;
      }
      const int k = th[2 + t];
      a0 += clip8(v0) * k, a1 += clip8(v1) * k, a2 += clip8(v2) * k;
    }
    c3[0] = clip8(a0), c3[1] = clip8(a1), c3[2] = clip8(a2);
  } else {                                // horizontal pass first (the common case)
    const int ymin = tv[0], nv = tv[1], xmin = th[0], nh = th[1];
    int a0 = 1 << (PREC - 1), a1 = a0, a2 = a0;
    for (int s = 0; s < nv; ++s) {
      const uint8_t* p = img + ((int64_t)(ymin + s) * w + xmin) * 3;
      int v0 = 1 << (PREC - 1), v1 = v0, v2 = v0;
      for (int t = 0; t < nh; ++t) {
        const int k = th[2 + t];
        v0 += p[3 * t] * k, v1 += p[3 * t + 1] * k, v2 += p[3 * t + 2] * k;
      }
      const int k = tv[2 + s];
      a0 += clip8(v0) * k, a1 += clip8(v1) * k, a2 += clip8(v2) * k;
    }
    c3[0] = clip8(a0), c3[1] = clip8(a1), c3[2] = clip8(a2);
  }
  if (gray) {
    const int l = (c3[0] * 19595 + c3[1] * 38470 + c3[2] * 7471 + 0x8000) >> 16;
    c3[0] = c3[1] = c3[2] = l;
  }
  if (out_u8) {
    uint8_t* q = out_u8 + i * 3;
    q[0] = (uint8_t)c3[0], q[1] = (uint8_t)c3[1], q[2] = (uint8_t)c3[2];
  }
  float* o = out + (int64_t)b * 3 * plane + rem;
  o[0] = ((float)c3[0] / 255.0f - m0) / s0;
  o[plane] = ((float)c3[1] / 255.0f - m1) / s1;
  o[2 * plane] = ((float)c3[2] / 255.0f - m2) / s2;
}

}  // namespace

extern "C" int pipnet_resize_plan(const int32_t* sizes_host, int B, int out_h, int out_w, int* kmax,
                                  int64_t* workspace_bytes) {
  if (B < 0 || out_h <= 0 || out_w <= 0 || !kmax || !workspace_bytes || (B > 0 && !sizes_host))
    return PIPNET_ERR_ARG;
  int k = 3;
  for (int b = 0; b < B; ++b) {
    const int h = sizes_host[2 * b], w = sizes_host[2 * b + 1];
    if (h <= 0 || w <= 0) return PIPNET_ERR_ARG;
    const int kv = ksize_for(h, out_h), kh = ksize_for(w, out_w);
    k = kv > k ? kv : k;
    k = kh > k ? kh : k;
  }
  *kmax = k;
  *workspace_bytes = (int64_t)B * (out_h + out_w) * (2 + k) * (int64_t)sizeof(int32_t);
  return PIPNET_OK;
}

extern "C" int pipnet_resize_normalize_rgb8(const uint8_t* pixels, const int64_t* offsets, const int32_t* sizes,
                                            int B, int out_h, int out_w, int kmax, int grayscale,
                                            const float* mean3, const float* std3, int32_t* workspace,
                                            float* out, uint8_t* out_u8, void* stream) {
  if (B < 0 || out_h <= 0 || out_w <= 0 || kmax < 3 || !mean3 || !std3) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  if (!pixels || !offsets || !sizes || !workspace || !out) return PIPNET_ERR_ARG;
  if ((int64_t)out_h * out_w >= ((int64_t)1 << 31) / 4) return PIPNET_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int rows = B * (out_h + out_w);
  hipLaunchKernelGGL(resize_coeffs_kernel, dim3((rows + 255) / 256), dim3(256), 0, s, sizes, B, out_h, out_w, kmax,
                     workspace);
  PIPNET_CHECK_LAUNCH();
  const int64_t n = (int64_t)B * out_h * out_w;
  hipLaunchKernelGGL(resize_normalize_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, pixels, offsets,
                     sizes, B, out_h, out_w, kmax, workspace, grayscale ? 1 : 0, mean3[0], mean3[1], mean3[2],
                     std3[0], std3[1], std3[2], out, out_u8);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
