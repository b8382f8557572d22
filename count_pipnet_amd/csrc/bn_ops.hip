// BatchNorm2d in training mode, and the stride-s gradient scatter, for the ResNet training
// step (features/resnet_features.py:77-119 Bottleneck, 126-222 ResNet_features; every
// BatchNorm2d of the backbone runs in train mode under net.train(), pipnet/train.py:14).
//
// torch.nn.BatchNorm2d train-mode semantics on NHWC rows x[M][C] (M = B*H*W):
//   mean = sum_m x / M, var = sum_m (x - mean)^2 / M, invstd = 1/sqrt(var + eps) (one pass:
//   Welford per thread, Chan et al. pairwise combination of the partial (count, mean, M2)),
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
constexpr int BN_GMAX = 1024;      // max row slabs of the column reductions
constexpr int BN_UNROLL = 4;       // rows in flight per thread

// Row slabs: each thread of slab g walks rows g*RL + rl + k*G*RL; enough slabs to fill the
// chip, each thread keeping >= 16 rows.
int bn_slabs(int64_t M, int C) {
  const int Q = C / 4, QB = Q < 64 ? Q : 64, RL = BN_T / QB;
  const int64_t want = M / ((int64_t)RL * 16);
  return (int)(want < 1 ? 1 : (want > BN_GMAX ? BN_GMAX : want));
}

// Chan et al. pairwise combination of (count, mean, M2) -- fixed order everywhere.
PIPNET_DEV void chan_combine(float& n, f32x4& mean, f32x4& m2, float nb, f32x4 meanb, f32x4 m2b) {
  const float nt = n + nb;
  if (nb == 0.f) return;
  if (n == 0.f) {
    n = nb;
    mean = meanb;
    m2 = m2b;
    return;
  }
  const f32x4 d = meanb - mean;
  const float fb = nb / nt;
  mean += d * fb;
  m2 += m2b + d * d * (n * fb);
  n = nt;
}

// Forward statistics in one pass: per thread Welford over its rows (channel quad), the row
// lanes of the workgroup combined in LDS, partial[g][0..2][C] = (count, mean, M2) per slab.
__global__ __launch_bounds__(BN_T) void bn_welford_kernel(const float* __restrict__ x, int64_t M, int C,
                                                          float* __restrict__ partial) {
  __shared__ f32x4 sm[BN_T], s2[BN_T];
  __shared__ float sn[BN_T];
  const int Q = C >> 2;
  const int QB = Q < 64 ? Q : 64;
  const int RL = BN_T / QB;
  const int tid = threadIdx.x;
  const int qi = tid % QB, rl = tid / QB;
  const int q = blockIdx.x * QB + qi;
  const int c = 4 * q;
  float n = 0.f;
  f32x4 mean = {0.f, 0.f, 0.f, 0.f}, m2 = {0.f, 0.f, 0.f, 0.f};
  if (q < Q) {
    const int64_t step = (int64_t)gridDim.y * RL;
    int64_t m = (int64_t)blockIdx.y * RL + rl;
    for (; m + (BN_UNROLL - 1) * step < M; m += BN_UNROLL * step) {
      f32x4 v[BN_UNROLL];
#pragma unroll
      for (int u = 0; u < BN_UNROLL; ++u) v[u] = ld4(x + (m + u * step) * C + c);
#pragma unroll
      for (int u = 0; u < BN_UNROLL; ++u) {
        n += 1.f;
        const f32x4 d = v[u] - mean;
        mean += d * (1.0f / n);
        m2 += d * (v[u] - mean);
      }
    }
    for (; m < M; m += step) {
      const f32x4 v = ld4(x + m * C + c);
      n += 1.f;
      const f32x4 d = v - mean;
      mean += d * (1.0f / n);
      m2 += d * (v - mean);
    }
  }
  sm[tid] = mean;
  s2[tid] = m2;
  sn[tid] = n;
  __syncthreads();
  if (rl == 0 && q < Q) {
    for (int r = 1; r < RL; ++r) chan_combine(n, mean, m2, sn[r * QB + qi], sm[r * QB + qi], s2[r * QB + qi]);
    float* pp = partial + (int64_t)blockIdx.y * 3 * C;
    st4(pp + c, f32x4{n, n, n, n});
    st4(pp + C + c, mean);
    st4(pp + 2 * C + c, m2);
  }
}

// Backward sums: partial[g][0][C] = sum g, [1][C] = sum g * xhat (g = dy [* (relu_out > 0)]).
__global__ __launch_bounds__(BN_T) void bn_bwd_partial_kernel(const float* __restrict__ x,
                                                              const float* __restrict__ dy,
                                                              const float* __restrict__ relu_out, int64_t M, int C,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              float* __restrict__ partial) {
  __shared__ f32x4 red[2][BN_T];
  const int Q = C >> 2;
  const int QB = Q < 64 ? Q : 64;
  const int RL = BN_T / QB;
  const int tid = threadIdx.x;
  const int qi = tid % QB, rl = tid / QB;
  const int q = blockIdx.x * QB + qi;
  const int c = 4 * q;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
  if (q < Q) {
    const f32x4 mu = ld4(mean + c), is = ld4(invstd + c);
    const int64_t step = (int64_t)gridDim.y * RL;
    for (int64_t m0 = (int64_t)blockIdx.y * RL + rl; m0 < M; m0 += BN_UNROLL * step) {
      f32x4 v[BN_UNROLL], g[BN_UNROLL], y[BN_UNROLL];
#pragma unroll
      for (int u = 0; u < BN_UNROLL; ++u) {
        const int64_t m = m0 + u * step;
        const bool ok = m < M;
        v[u] = ok ? ld4(x + m * C + c) : mu;
        g[u] = ok ? ld4(dy + m * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
        y[u] = (ok && relu_out) ? ld4(relu_out + m * C + c) : f32x4{1.f, 1.f, 1.f, 1.f};
      }
#pragma unroll
      for (int u = 0; u < BN_UNROLL; ++u) {
#pragma unroll
        for (int e = 0; e < 4; ++e) g[u][e] = y[u][e] > 0.f ? g[u][e] : 0.f;
        s0 += g[u];
        s1 += g[u] * ((v[u] - mu) * is);
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
    st4(partial + ((int64_t)blockIdx.y * 2 + 1) * C + c, t1);
  }
}

// Finishing reductions over the G slabs: 64 channels per workgroup, FIN_L slab lanes (slabs
// sl, sl + FIN_L, ...; loads four slabs ahead) combined in order, then the lanes in order.
constexpr int FIN_C = 64, FIN_L = 16;

__global__ __launch_bounds__(FIN_C * FIN_L) void bn_stats_finish_kernel(const float* __restrict__ partial, int G,
                                                                        int C, int64_t M, float eps, float momentum,
                                                                        float* __restrict__ mean,
                                                                        float* __restrict__ invstd,
                                                                        float* __restrict__ rmean,
                                                                        float* __restrict__ rvar) {
  __shared__ float sn[FIN_L][FIN_C], smu[FIN_L][FIN_C], sm2[FIN_L][FIN_C];
  const int ci = threadIdx.x % FIN_C, sl = threadIdx.x / FIN_C;
  const int c = blockIdx.x * FIN_C + ci;
  float n = 0.f, mu = 0.f, m2 = 0.f;
  if (c < C) {
    for (int g0 = sl; g0 < G; g0 += 4 * FIN_L) {
      float nb[4], mb[4], m2b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = g0 + u * FIN_L;
        const float* pp = partial + (int64_t)(g < G ? g : 0) * 3 * C;
        nb[u] = g < G ? pp[c] : 0.f;
        mb[u] = pp[C + c];
        m2b[u] = pp[2 * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (nb[u] == 0.f) continue;
        const float nt = n + nb[u], d = mb[u] - mu, fb = nb[u] / nt;
        mu += d * fb;
        m2 += m2b[u] + d * d * (n * fb);
        n = nt;
      }
    }
  }
  sn[sl][ci] = n;
  smu[sl][ci] = mu;
  sm2[sl][ci] = m2;
  __syncthreads();
  if (sl != 0 || c >= C) return;
  for (int l = 1; l < FIN_L; ++l) {
    const float nb = sn[l][ci];
    if (nb == 0.f) continue;
    const float mb = smu[l][ci], m2b = sm2[l][ci];
    const float nt = n + nb, d = mb - mu, fb = nb / nt;
    mu += d * fb;
    m2 += m2b + d * d * (n * fb);
    n = nt;
  }
  const float var = m2 / (float)M;
  mean[c] = mu;
  invstd[c] = 1.0f / sqrtf(var + eps);
  if (rmean) {
    const float unbiased = (float)((double)m2 / (double)(M - 1));
    rmean[c] = (1.0f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.0f - momentum) * rvar[c] + momentum * unbiased;
  }
}

__global__ __launch_bounds__(FIN_C * FIN_L) void bn_bwd_finish_kernel(const float* __restrict__ partial, int G, int C,
                                                                      int64_t M, float* __restrict__ d_gamma,
                                                                      float* __restrict__ d_beta,
                                                                      float* __restrict__ coef) {
  __shared__ float r0[FIN_L][FIN_C], r1[FIN_L][FIN_C];
  const int ci = threadIdx.x % FIN_C, sl = threadIdx.x / FIN_C;
  const int c = blockIdx.x * FIN_C + ci;
  float s0 = 0.f, s1 = 0.f;
  if (c < C) {
    for (int g0 = sl; g0 < G; g0 += 4 * FIN_L) {
      float a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int g = g0 + u * FIN_L;
        a[u] = g < G ? partial[((int64_t)g * 2) * C + c] : 0.f;
        b[u] = g < G ? partial[((int64_t)g * 2 + 1) * C + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        s0 += a[u];
        s1 += b[u];
      }
    }
  }
  r0[sl][ci] = s0;
  r1[sl][ci] = s1;
  __syncthreads();
  if (sl != 0 || c >= C) return;
  for (int l = 1; l < FIN_L; ++l) {
    s0 += r0[l][ci];
    s1 += r1[l][ci];
  }
  const float inv_m = 1.0f / (float)M;
  d_beta[c] = s0;
  d_gamma[c] = s1;
  coef[c] = s0 * inv_m;
  coef[C + c] = s1 * inv_m;
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

extern "C" int64_t pipnet_bn_workspace_floats(int C) { return C > 0 ? ((int64_t)BN_GMAX * 3 + 2) * C : 0; }

extern "C" int pipnet_bn_stats_f32(const float* x, int64_t M, int C, float eps, float momentum, float* mean,
                                   float* invstd, float* running_mean, float* running_var, float* workspace,
                                   void* stream) {
  if (!bn_shape_ok(M, C) || M < 2 || !x || !mean || !invstd || !workspace) return PIPNET_ERR_ARG;
  if ((running_mean == nullptr) != (running_var == nullptr)) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(mean) || !aligned16(workspace)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int Q = C / 4, QB = Q < 64 ? Q : 64;
  const int G = bn_slabs(M, C);
  hipLaunchKernelGGL(bn_welford_kernel, dim3((unsigned)((Q + QB - 1) / QB), (unsigned)G), dim3(BN_T), 0, s, x, M, C,
                     workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_stats_finish_kernel, dim3((unsigned)((C + FIN_C - 1) / FIN_C)), dim3(FIN_C * FIN_L), 0, s,
                     workspace, G, C, M, eps, momentum, mean, invstd, running_mean, running_var);
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
  const int G = bn_slabs(M, C);
  float* coef = workspace + (int64_t)BN_GMAX * 3 * C;
  hipLaunchKernelGGL(bn_bwd_partial_kernel, dim3((unsigned)((Q + QB - 1) / QB), (unsigned)G), dim3(BN_T), 0, s, x, dy,
                     relu_out, M, C, mean, invstd, workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3((unsigned)((C + FIN_C - 1) / FIN_C)), dim3(FIN_C * FIN_L), 0, s,
                     workspace, G, C, M, d_gamma, d_beta, coef);
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
