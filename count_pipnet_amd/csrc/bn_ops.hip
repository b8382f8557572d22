// BatchNorm2d in training mode, and the stride-s gradient scatter, for the ResNet training
// step (features/resnet_features.py:77-119 Bottleneck, 126-222 ResNet_features; every
// BatchNorm2d of the backbone runs in train mode under net.train(), pipnet/train.py:14).
//
// torch.nn.BatchNorm2d train-mode semantics on NHWC rows x[M][C] (M = B*H*W):
//   mean = sum_m x / M, var = sum_m (x - mean)^2 / M (two passes), invstd = 1/sqrt(var + eps),
//   y = gamma * (x - mean) * invstd + beta  [+ residual] [ReLU],
//   running_mean = (1 - mom) running_mean + mom mean,
//   running_var  = (1 - mom) running_var  + mom var * M / (M - 1);
// backward with g = dy [* (out > 0) when a ReLU follows]:
//   d_beta = sum g, d_gamma = sum g xhat, dx = gamma invstd (g - d_beta/M - xhat d_gamma/M).
// Column reductions: each workgroup reduces a fixed strided slab of rows into partial[g][..][C]
// (lanes own channel quads, row lanes combined in a fixed order), a finishing kernel sums the
// slabs in order -- deterministic, no atomics.
#include "common.hpp"

namespace {

constexpr int BN_T = 256;
constexpr int BN_G = 256;          // row slabs of the column reductions

// MODE 0: sum x.  MODE 1: sum (x - mean)^2.  MODE 2: sum g and sum g * xhat (backward).
template <int MODE>
__global__ __launch_bounds__(BN_T) void bn_partial_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                          const float* __restrict__ relu_out, int64_t M, int C,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          float* __restrict__ partial) {
  __shared__ f32x4 red[2][BN_T];
  const int Q = C >> 2;
  const int QB = Q < 64 ? Q : 64;            // channel quads per row pass (host: 256 % QB == 0)
  const int RL = BN_T / QB;                   // row lanes
  const int tid = threadIdx.x;
  const int qi = tid % QB, rl = tid / QB;
  const int q = blockIdx.x * QB + qi;
  const int c = 4 * q;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
  if (q < Q) {
    const f32x4 mu = MODE >= 1 ? ld4(mean + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 is = MODE == 2 ? ld4(invstd + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int64_t m = (int64_t)blockIdx.y * RL + rl; m < M; m += (int64_t)gridDim.y * RL) {
      const f32x4 v = ld4(x + m * C + c);
      if constexpr (MODE == 0) {
        s0 += v;
      } else if constexpr (MODE == 1) {
        const f32x4 d = v - mu;
        s0 += d * d;
      } else {
        f32x4 g = ld4(dy + m * C + c);
        if (relu_out) {
          const f32x4 y = ld4(relu_out + m * C + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) g[e] = y[e] > 0.f ? g[e] : 0.f;
        }
        s0 += g;
        s1 += g * ((v - mu) * is);
      }
    }
  }
  red[0][tid] = s0;
  red[1][tid] = s1;
  __syncthreads();
  if (rl == 0 && q < Q) {
    f32x4 t0 = red[0][qi], t1 = red[1][qi];
    for (int r = 1; r < RL; ++r) {
      t0 += red[0][r * QB + qi];
      t1 += red[1][r * QB + qi];
    }
    st4(partial + ((int64_t)blockIdx.y * 2) * C + c, t0);
    if (MODE == 2) st4(partial + ((int64_t)blockIdx.y * 2 + 1) * C + c, t1);
  }
}

// MODE 0: mean.  MODE 1: invstd + running stats.  MODE 2: d_gamma / d_beta + the two
// per-channel coefficients of the backward apply (coef[0][c] = sum g / M, coef[1][c] =
// sum g xhat / M).
template <int MODE>
__global__ __launch_bounds__(256) void bn_finish_kernel(const float* __restrict__ partial, int G, int C, int64_t M,
                                                        float eps, float momentum, float* __restrict__ mean,
                                                        float* __restrict__ invstd, float* __restrict__ rmean,
                                                        float* __restrict__ rvar, float* __restrict__ d_gamma,
                                                        float* __restrict__ d_beta, float* __restrict__ coef) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s0 = 0.f, s1 = 0.f;
  for (int g = 0; g < G; ++g) {
    s0 += partial[((int64_t)g * 2) * C + c];
    if (MODE == 2) s1 += partial[((int64_t)g * 2 + 1) * C + c];
  }
  const float inv_m = 1.0f / (float)M;
  if constexpr (MODE == 0) {
    mean[c] = s0 * inv_m;
  } else if constexpr (MODE == 1) {
    const float var = s0 * inv_m;
    invstd[c] = 1.0f / sqrtf(var + eps);
    if (rmean) {
      const float unbiased = (float)((double)s0 / (double)(M - 1));
      rmean[c] = (1.0f - momentum) * rmean[c] + momentum * mean[c];
      rvar[c] = (1.0f - momentum) * rvar[c] + momentum * unbiased;
    }
  } else {
    d_beta[c] = s0;
    d_gamma[c] = s1;
    coef[c] = s0 * inv_m;
    coef[C + c] = s1 * inv_m;
  }
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ x, int64_t n4, int C,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const float* __restrict__ r,
                                                       float* __restrict__ y) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int c = (int)((4 * i) % C);
    const f32x4 v = ld4(x + 4 * i);
    const f32x4 mu = ld4(mean + c), is = ld4(invstd + c), g = ld4(gamma + c), b = ld4(beta + c);
    f32x4 o = g * (v - mu) * is + b;
    if constexpr (RES) o += ld4(r + 4 * i);
    if constexpr (RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaxf(o[e], 0.f);
    }
    st4(y + 4 * i, o);
  }
}

__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                           const float* __restrict__ relu_out, int64_t n4, int C,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ coef, float* __restrict__ dx,
                                                           float* __restrict__ d_masked) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int c = (int)((4 * i) % C);
    f32x4 g = ld4(dy + 4 * i);
    if (relu_out) {
      const f32x4 yo = ld4(relu_out + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) g[e] = yo[e] > 0.f ? g[e] : 0.f;
    }
    if (d_masked) st4(d_masked + 4 * i, g);
    if (dx) {
      const f32x4 is = ld4(invstd + c);
      const f32x4 xh = (ld4(x + 4 * i) - ld4(mean + c)) * is;
      st4(dx + 4 * i, (g - ld4(coef + c) - xh * ld4(coef + C + c)) * is * ld4(gamma + c));
    }
  }
}

// out[b][y][x][c] (+)= (y, x on the stride-s lattice inside OH x OW) ? in[b][y/s][x/s][c] : 0
// -- the input gradient of a stride-s 1x1 conv, and the zero-inserted output gradient a
// stride-s 3x3 conv's input gradient is computed from (as a stride-1 conv).
__global__ __launch_bounds__(256) void stride_scatter_kernel(const float* __restrict__ in, int B, int OH, int OW,
                                                             int C, int H, int W, int s, int accumulate,
                                                             float* __restrict__ out) {
  const int64_t n4 = (int64_t)B * H * W * (C / 4);
  const int Q = C / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int q = (int)(i % Q);
    const int64_t p = i / Q;
    const int xx = (int)(p % W);
    const int64_t t = p / W;
    const int yy = (int)(t % H);
    const int b = (int)(t / H);
    const int oy = yy / s, ox = xx / s;
    const bool on = yy - oy * s == 0 && xx - ox * s == 0 && oy < OH && ox < OW;
    f32x4 v = on ? ld4(in + (((int64_t)b * OH + oy) * OW + ox) * C + 4 * q) : f32x4{0.f, 0.f, 0.f, 0.f};
    if (accumulate) v += ld4(out + 4 * i);
    st4(out + 4 * i, v);
  }
}

int elem_grid(int64_t n4) {
  const int64_t g = (n4 + 255) / 256;
  return (int)(g < 256 * 16 ? g : 256 * 16);
}

bool bn_shape_ok(int64_t M, int C) {
  if (M < 1 || C < 4 || (C & 3)) return false;
  const int Q = C / 4;
  return Q >= 64 || (BN_T % Q) == 0;
}

}  // namespace

extern "C" int64_t pipnet_bn_workspace_floats(int C) { return C > 0 ? ((int64_t)BN_G * 2 + 2) * C : 0; }

extern "C" int pipnet_bn_stats_f32(const float* x, int64_t M, int C, float eps, float momentum, float* mean,
                                   float* invstd, float* running_mean, float* running_var, float* workspace,
                                   void* stream) {
  if (!bn_shape_ok(M, C) || M < 2 || !x || !mean || !invstd || !workspace) return PIPNET_ERR_ARG;
  if ((running_mean == nullptr) != (running_var == nullptr)) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(mean) || !aligned16(workspace)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int Q = C / 4, QB = Q < 64 ? Q : 64;
  const dim3 grid((unsigned)((Q + QB - 1) / QB), BN_G);
  const unsigned gf = (unsigned)((C + 255) / 256);
  hipLaunchKernelGGL(bn_partial_kernel<0>, grid, dim3(BN_T), 0, s, x, nullptr, nullptr, M, C, nullptr, nullptr,
                     workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_finish_kernel<0>, dim3(gf), dim3(256), 0, s, workspace, BN_G, C, M, eps, momentum, mean,
                     nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_partial_kernel<1>, grid, dim3(BN_T), 0, s, x, nullptr, nullptr, M, C, mean, nullptr,
                     workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_finish_kernel<1>, dim3(gf), dim3(256), 0, s, workspace, BN_G, C, M, eps, momentum, mean,
                     invstd, running_mean, running_var, nullptr, nullptr, nullptr);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_bn_apply_f32(const float* x, int64_t M, int C, const float* mean, const float* invstd,
                                   const float* gamma, const float* beta, const float* residual, int relu, float* y,
                                   void* stream) {
  if (!bn_shape_ok(M, C) || !x || !mean || !invstd || !gamma || !beta || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(y) || !aligned16(mean) || !aligned16(invstd) || !aligned16(gamma) ||
      !aligned16(beta) || (residual && !aligned16(residual)))
    return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int64_t n4 = M * C / 4;
  const dim3 g(elem_grid(n4));
  if (residual && relu)
    hipLaunchKernelGGL((bn_apply_kernel<true, true>), g, dim3(256), 0, s, x, n4, C, mean, invstd, gamma, beta, residual,
                       y);
  else if (residual)
    hipLaunchKernelGGL((bn_apply_kernel<true, false>), g, dim3(256), 0, s, x, n4, C, mean, invstd, gamma, beta,
                       residual, y);
  else if (relu)
    hipLaunchKernelGGL((bn_apply_kernel<false, true>), g, dim3(256), 0, s, x, n4, C, mean, invstd, gamma, beta,
                       residual, y);
  else
    hipLaunchKernelGGL((bn_apply_kernel<false, false>), g, dim3(256), 0, s, x, n4, C, mean, invstd, gamma, beta,
                       residual, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_bn_backward_f32(const float* x, const float* dy, const float* relu_out, int64_t M, int C,
                                      const float* mean, const float* invstd, const float* gamma, float* dx,
                                      float* d_masked, float* d_gamma, float* d_beta, float* workspace,
                                      void* stream) {
  if (!bn_shape_ok(M, C) || !x || !dy || !mean || !invstd || !gamma || !d_gamma || !d_beta || !workspace)
    return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(dy) || (relu_out && !aligned16(relu_out)) || (dx && !aligned16(dx)) ||
      (d_masked && !aligned16(d_masked)) || !aligned16(workspace) || !aligned16(mean) || !aligned16(invstd) ||
      !aligned16(gamma))
    return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int Q = C / 4, QB = Q < 64 ? Q : 64;
  float* coef = workspace + (int64_t)BN_G * 2 * C;
  hipLaunchKernelGGL(bn_partial_kernel<2>, dim3((unsigned)((Q + QB - 1) / QB), BN_G), dim3(BN_T), 0, s, x, dy,
                     relu_out, M, C, mean, invstd, workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_finish_kernel<2>, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, s, workspace, BN_G, C, M,
                     0.f, 0.f, nullptr, nullptr, nullptr, nullptr, d_gamma, d_beta, coef);
  PIPNET_CHECK_LAUNCH();
  if (dx || d_masked) {
    const int64_t n4 = M * C / 4;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(elem_grid(n4)), dim3(256), 0, s, x, dy, relu_out, n4, C, mean,
                       invstd, gamma, coef, dx, d_masked);
    PIPNET_CHECK_LAUNCH();
  }
  return PIPNET_OK;
}

extern "C" int pipnet_stride_scatter_f32(const float* in, int B, int OH, int OW, int C, int H, int W, int stride,
                                         int accumulate, float* out, void* stream) {
  if (B < 0 || OH <= 0 || OW <= 0 || C < 4 || (C & 3) || H <= 0 || W <= 0 || stride <= 0 || !in || !out)
    return PIPNET_ERR_ARG;
  if ((int64_t)(OH - 1) * stride >= H || (int64_t)(OW - 1) * stride >= W) return PIPNET_ERR_ARG;
  if (!aligned16(in) || !aligned16(out)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int64_t n4 = (int64_t)B * H * W * (C / 4);
  hipLaunchKernelGGL(stride_scatter_kernel, dim3(elem_grid(n4)), dim3(256), 0, (hipStream_t)stream, in, B, OH, OW, C,
                     H, W, stride, accumulate, out);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
