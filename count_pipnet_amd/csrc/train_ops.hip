// PIP-Net training-step kernels for the finetune phase (first slice):
// the loss of pipnet/train.py:calculate_loss (train.py:154-250) with its gradient w.r.t. the
// classifier output, the NonNegLinear weight/bias gradient (pipnet.py:54-71), and the
// torch.optim.AdamW update (util/args.py:327-328) fused with train.py:134-140's
// post-step clamps.  Everything after the (HIP, train-mode) forward of one
// train_pipnet iteration (train.py:75-140) when only the classifier trains.
//
// Layouts: proto features NHWC [2*Bh][HW][P] (the forward's own storage; the batch is
// cat([xs1, xs2]), so pixel n of the first half pairs with pixel n of the second), pooled
// [N][P], out / d_out [N][K] with N = 2*Bh, labels int64 [Bh] (ys = cat([ys1, ys1])).
// All reductions run in a fixed order (deterministic, grid-size independent for a given
// launch configuration).
#include <cmath>

#include "common.hpp"

namespace {

constexpr int ALIGN_T = 256;           // align partials: 4 waves, one pixel per wave step
constexpr int ALIGN_BLOCKS = 1024;     // fixed partial count (deterministic final sum)
constexpr int LOSS_T = 1024;           // single-workgroup loss kernel
constexpr int BWD_T = 256;

// align_loss(pf1, pf2) (train.py:259-265): per pixel -log(<pf1[n], pf2[n]> + 1e-12); this
// kernel writes one double partial sum per workgroup, the loss kernel adds them in order.
__global__ __launch_bounds__(ALIGN_T) void align_partial_kernel(const float* __restrict__ pf, int64_t npix, int P,
                                                                 double* __restrict__ partial) {
  __shared__ double wsum[ALIGN_T / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t stride = (int64_t)gridDim.x * (ALIGN_T / 64);
  const float* second = pf + npix * P;
  double acc = 0.0;                          // lane 0's running sum, pixels in increasing order
  for (int64_t n = (int64_t)blockIdx.x * (ALIGN_T / 64) + wv; n < npix; n += stride) {
    const float* a = pf + n * P;
    const float* b = second + n * P;
    float d = 0.f;
    if ((P & 3) == 0) {
      for (int c = 4 * lane; c < P; c += 256) {
        const f32x4 x = ld4(a + c), y = ld4(b + c);
        d = fmaf(x[0], y[0], d);
        d = fmaf(x[1], y[1], d);
        d = fmaf(x[2], y[2], d);
        d = fmaf(x[3], y[3], d);
      }
    } else {
      for (int c = lane; c < P; c += 64) d = fmaf(a[c], b[c], d);
    }
    d = wave_sum(d);
    acc += -(double)logf(d + 1e-12f);
  }
  if (lane == 0) wsum[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < ALIGN_T / 64; ++w) s += wsum[w];
    partial[blockIdx.x] = s;
  }
}

PIPNET_DEV double block_sum_d(double v, double* red) {   // LOSS_T threads, fixed order
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < LOSS_T / 64; ++w) s += red[w];
  return s;
}

// stats: [0] align loss, [1] tanh loss, [2] class loss, [3] total loss, [4] correct count,
//        [5] align weight, [6] tanh weight, [7] class weight (as used)
__global__ __launch_bounds__(LOSS_T) void loss_kernel(const double* __restrict__ align_partial, int nalign,
                                                      int64_t npix, const float* __restrict__ pooled,
                                                      const float* __restrict__ out, const int64_t* __restrict__ ys,
                                                      int Bh, int P, int K, const float* __restrict__ mult,
                                                      int enforce, float tanh_coeff, float w_align, float w_tanh,
                                                      float w_class, int mode, float* __restrict__ d_out,
                                                      float* __restrict__ stats) {
  __shared__ double red[LOSS_T / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int N = 2 * Bh;
  // ---- align: mean over the Bh*HW pixel pairs (both directions give the same value)
  double a = 0.0;
  for (int i = threadIdx.x; i < nalign; i += LOSS_T) a += align_partial[i];
  const double align = block_sum_d(a, red) / (double)npix;
  // ---- tanh: -(mean_p log(tanh(sum_b C*pooled1[b,p]) + 1e-8) + same for half 2) / 2
  double t1 = 0.0, t2 = 0.0;
  for (int p = threadIdx.x; p < P; p += LOSS_T) {
    float s1 = 0.f, s2 = 0.f;
    for (int b = 0; b < Bh; ++b) {
      s1 += tanh_coeff * pooled[(int64_t)b * P + p];
      s2 += tanh_coeff * pooled[(int64_t)(Bh + b) * P + p];
    }
    t1 += (double)logf(tanhf(s1) + 1e-8f);
    t2 += (double)logf(tanhf(s2) + 1e-8f);
  }
  t1 = block_sum_d(t1, red);
  t2 = block_sum_d(t2, red);
  const double tanh_loss = -(t1 / P + t2 / P) / 2.0;
  // ---- class: NLL(log_softmax(enforce ? log1p(out^m) : out), ys); d_out; argmax accuracy
  const float m = mult ? mult[0] : 1.f;
  const bool want_grad = mode != 1 && d_out != nullptr;   // mode 1 = pretrain (no class loss)
  const float gscale = w_class / (float)N;
  double nll = 0.0, correct = 0.0;
  for (int r = wv; r < N; r += LOSS_T / 64) {
    const float* o = out + (int64_t)r * K;
    const int y = (int)ys[r % Bh];
    float mx = -INFINITY, omx = -INFINITY;
    int oi = 0x7fffffff;
    for (int k = lane; k < K; k += 64) {
      const float ov = o[k];
      const float x = enforce ? log1pf(powf(ov, m)) : ov;
      mx = fmaxf(mx, x);
      if (ov > omx) { omx = ov; oi = k; }
    }
    mx = wave_max(mx);
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {         // argmax(out), first index on ties
      const float om = __shfl_xor(omx, sh, 64);
      const int oj = __shfl_xor(oi, sh, 64);
      if (om > omx || (om == omx && oj < oi)) { omx = om; oi = oj; }
    }
    float se = 0.f, xy = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float ov = o[k];
      const float x = enforce ? log1pf(powf(ov, m)) : ov;
      se += expf(x - mx);
      if (k == y) xy = x;
    }
    se = wave_sum(se);
    xy = wave_sum(xy);
    const float lse = mx + logf(se);
    if (lane == 0) {
      nll += (double)(lse - xy);
      correct += (oi == y) ? 1.0 : 0.0;
    }
    if (want_grad) {
      for (int k = lane; k < K; k += 64) {
        const float ov = o[k];
        float g;
        if (enforce) {
          const float pw = powf(ov, m);
          const float x = log1pf(pw);
          g = gscale * (expf(x - lse) - (k == y ? 1.f : 0.f));
          g = g / (1.f + pw);                                   // log1p backward
          g = g * (m == 0.f ? 0.f : m * powf(ov, m - 1.f));     // pow backward (masked at m == 0)
        } else {
          g = gscale * (expf(ov - lse) - (k == y ? 1.f : 0.f));
        }
        d_out[(int64_t)r * K + k] = g;
      }
    }
  }
  nll = block_sum_d(nll, red);
  correct = block_sum_d(correct, red);
  if (threadIdx.x == 0) {
    const double cls = nll / N;
    double loss = 0.0;
    if (mode == 0) loss = w_align * align + w_tanh * tanh_loss + w_class * cls;   // train
    if (mode == 1) loss = w_align * align + w_tanh * tanh_loss;                   // pretrain
    if (mode == 2) loss = w_class * cls;                                          // finetune
    stats[0] = (float)align;
    stats[1] = (float)tanh_loss;
    stats[2] = (float)cls;
    stats[3] = (float)loss;
    stats[4] = (float)correct;
    stats[5] = w_align;
    stats[6] = w_tanh;
    stats[7] = w_class;
  }
}

// NonNegLinear backward (F.linear(x, relu(W), b)): dW[k,p] = (W[k,p] > 0) * sum_r d_out[r,k] x[r,p]
// (threshold_backward of relu), db[k] = sum_r d_out[r,k].  One workgroup per (p-chunk, k);
// d_out[., k] is wave-uniform (scalar loads), x rows are read coalesced across p.
__global__ __launch_bounds__(BWD_T) void nonneg_linear_bwd_kernel(const float* __restrict__ d_out,
                                                                  const float* __restrict__ x, int N, int D,
                                                                  const float* __restrict__ W, int K,
                                                                  float* __restrict__ dW, float* __restrict__ db) {
  const int k = blockIdx.y;
  const int p = blockIdx.x * BWD_T + threadIdx.x;
  if (p < D) {
    float acc = 0.f;
    for (int r = 0; r < N; ++r) acc = fmaf(d_out[(int64_t)r * K + k], x[(int64_t)r * D + p], acc);
    dW[(int64_t)k * D + p] = W[(int64_t)k * D + p] > 0.f ? acc : 0.f;
  }
  if (db && blockIdx.x == 0 && threadIdx.x < 64) {
    float s = 0.f;
    for (int r = threadIdx.x; r < N; r += 64) s += d_out[(int64_t)r * K + k];
    s = wave_sum(s);
    if (threadIdx.x == 0) db[k] = s;
  }
}

// NonNegLinear input gradient: dx[r,p] = sum_k d_out[r,k] relu(W[k,p]) (the CountPIPNet finetune
// phase back-propagates into a trainable intermediate layer).  One thread per (r, p), K small.
__global__ __launch_bounds__(BWD_T) void nonneg_linear_dx_kernel(const float* __restrict__ d_out,
                                                                 const float* __restrict__ W, int N, int D, int K,
                                                                 float* __restrict__ dx) {
  const int p = blockIdx.x * BWD_T + threadIdx.x;
  const int r = blockIdx.y;
  if (p >= D) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc = fmaf(d_out[(int64_t)r * K + k], fmaxf(W[(int64_t)k * D + p], 0.f), acc);
  dx[(int64_t)r * D + p] = acc;
}

// BilinearIntermediate backward front (count_pipnet_utils.py:381-385, out = u * v with u = W(e),
// v = V(e)): du = g * v, dv = g * u.
__global__ __launch_bounds__(256) void bilinear_bwd_prep_kernel(const float* __restrict__ g,
                                                                const float* __restrict__ u,
                                                                const float* __restrict__ v, int64_t n,
                                                                float* __restrict__ du, float* __restrict__ dv) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gi = g[i];
    du[i] = gi * v[i];
    dv[i] = gi * u[i];
  }
}

// LinearIntermediate backward (count_pipnet_utils.py:471-519: out[n][e] = w[e] * x[n] for the
// rows n = (b, p), e < E, Linear(1, E, bias=False)): dx[n] = sum_e g[n][e] w[e] and per-
// workgroup partial sums of dw[e] = sum_n g[n][e] x[n] (fixed grid LI_BLOCKS, fixed lane /
// wave order), reduced in order by linear_inter_dw_kernel -> deterministic.
constexpr int LI_T = 256, LI_BLOCKS = 512, LI_EMAX = 16;

template <int E>
__global__ __launch_bounds__(LI_T) void linear_inter_bwd_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ g,
                                                                const float* __restrict__ w, int64_t n,
                                                                float* __restrict__ dx,
                                                                float* __restrict__ partial) {
  float wr[E], acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) { wr[e] = w[e]; acc[e] = 0.f; }
  for (int64_t i = (int64_t)blockIdx.x * LI_T + threadIdx.x; i < n; i += (int64_t)LI_BLOCKS * LI_T) {
    const float xi = x[i];
    const float* gi = g + i * E;
    float d = 0.f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float ge = gi[e];
      d = fmaf(ge, wr[e], d);
      acc[e] = fmaf(ge, xi, acc[e]);
    }
    if (dx) dx[i] = d;
  }
  __shared__ float red[LI_T / 64][E];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float v = acc[e];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wv][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < E) {
    float v = 0.f;
    for (int k = 0; k < LI_T / 64; ++k) v += red[k][threadIdx.x];
    partial[(int64_t)blockIdx.x * E + threadIdx.x] = v;
  }
}

__global__ __launch_bounds__(64) void linear_inter_dw_kernel(const float* __restrict__ partial, int E,
                                                             float* __restrict__ dw, int accumulate) {
  const int e = threadIdx.x;
  if (e >= E) return;
  float v = 0.f;
  for (int b = 0; b < LI_BLOCKS; ++b) v += partial[(int64_t)b * E + e];
  dw[e] = accumulate ? dw[e] + v : v;
}

// torch.optim.AdamW (decoupled weight decay, amsgrad off), one parameter tensor, in torch's
// float arithmetic (the host turns the double hyper-parameters into the same float
// constants torch's foreach kernels receive: 1 - lr*wd, 1 - beta1, beta2, 1 - beta2, ...):
//   p *= decay;  m = lerp(m, g, w1);  v = v*b2 + w2*g*g;
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps)       (step_size = lr / (1 - b1^t))
// then the reference's post-step clamp (train.py:134-140) when post != 0:
//   p = max(p - post_delta, post_floor).
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                    float decay, float w1, float b2, float w2, float eps,
                                                    float step_size, float bc2_sqrt, int post, float post_delta,
                                                    float post_floor) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float gi = g[i];
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + w1 * (gi - mi);                   // torch lerp, weight < 0.5 branch
    const float vi = v[i] * b2 + w2 * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    if (post) pi = fmaxf(pi - post_delta, post_floor);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ void clamp_min_kernel(float* __restrict__ x, int64_t n, float lo) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    x[i] = fmaxf(x[i], lo);
}

inline unsigned grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

}  // namespace

extern "C" int pipnet_train_align_partial_f32(const float* pf, int Bh, int HW, int P, double* partial, void* stream) {
  if (Bh <= 0 || HW <= 0 || P <= 0 || !pf || !partial) return PIPNET_ERR_ARG;
  if ((P & 3) == 0 && !aligned16(pf)) return PIPNET_ERR_ALIGN;
  hipLaunchKernelGGL(align_partial_kernel, dim3(ALIGN_BLOCKS), dim3(ALIGN_T), 0, (hipStream_t)stream, pf,
                     (int64_t)Bh * HW, P, partial);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_train_align_partials(void) { return ALIGN_BLOCKS; }

extern "C" int pipnet_train_loss_f32(const double* align_partial, int Bh, int HW, const float* pooled,
                                     const float* out, const int64_t* ys, int P, int K, const float* mult,
                                     int enforce, float tanh_coeff, float w_align, float w_tanh, float w_class,
                                     int mode, float* d_out, float* stats, void* stream) {
  if (Bh <= 0 || HW <= 0 || P <= 0 || K <= 0 || mode < 0 || mode > 2) return PIPNET_ERR_ARG;
  if (!align_partial || !pooled || !out || !ys || !stats) return PIPNET_ERR_ARG;
  if (mode != 1 && !d_out) return PIPNET_ERR_ARG;
  hipLaunchKernelGGL(loss_kernel, dim3(1), dim3(LOSS_T), 0, (hipStream_t)stream, align_partial, ALIGN_BLOCKS,
                     (int64_t)Bh * HW, pooled, out, ys, Bh, P, K, mult, enforce, tanh_coeff, w_align, w_tanh,
                     w_class, mode, d_out, stats);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_nonneg_linear_bwd_f32(const float* d_out, const float* x, int N, int D, const float* W,
                                            int K, float* dW, float* db, void* stream) {
  if (N <= 0 || D <= 0 || K <= 0 || K > 65535 || !d_out || !x || !W || !dW) return PIPNET_ERR_ARG;
  hipLaunchKernelGGL(nonneg_linear_bwd_kernel, dim3((unsigned)((D + BWD_T - 1) / BWD_T), (unsigned)K), dim3(BWD_T), 0,
                     (hipStream_t)stream, d_out, x, N, D, W, K, dW, db);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_adamw_step_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                     double lr, double beta1, double beta2, double eps, double weight_decay,
                                     int64_t step, int post, float post_delta, float post_floor, void* stream) {
  if (n < 0 || step < 1 || !param || !grad || !exp_avg || !exp_avg_sq) return PIPNET_ERR_ARG;
  if (!(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0)) return PIPNET_ERR_ARG;
  if (n == 0) return PIPNET_OK;
  const double bc1 = 1.0 - std::pow(beta1, (double)step), bc2 = 1.0 - std::pow(beta2, (double)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, param, grad, exp_avg,
                     exp_avg_sq, n, (float)(1.0 - lr * weight_decay), (float)(1.0 - beta1), (float)beta2,
                     (float)(1.0 - beta2), (float)eps, (float)(lr / bc1), (float)std::sqrt(bc2), post, post_delta,
                     post_floor);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_clamp_min_f32(float* x, int64_t n, float lo, void* stream) {
  if (n < 0 || !x) return PIPNET_ERR_ARG;
  if (n == 0) return PIPNET_OK;
  hipLaunchKernelGGL(clamp_min_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, lo);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_nonneg_linear_dx_f32(const float* d_out, const float* W, int N, int D, int K, float* dx,
                                           void* stream) {
  if (N < 0 || D <= 0 || K <= 0 || N > 65535 || !d_out || !W || !dx) return PIPNET_ERR_ARG;
  if (N == 0) return PIPNET_OK;
  hipLaunchKernelGGL(nonneg_linear_dx_kernel, dim3((unsigned)((D + BWD_T - 1) / BWD_T), (unsigned)N), dim3(BWD_T), 0,
                     (hipStream_t)stream, d_out, W, N, D, K, dx);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_bilinear_bwd_prep_f32(const float* g, const float* u, const float* v, int64_t n, float* du,
                                            float* dv, void* stream) {
  if (n < 0 || !g || !u || !v || !du || !dv) return PIPNET_ERR_ARG;
  if (n == 0) return PIPNET_OK;
  hipLaunchKernelGGL(bilinear_bwd_prep_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, g, u, v, n, du,
                     dv);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_linear_inter_partials_floats(int E) { return E > 0 ? LI_BLOCKS * E : 0; }

extern "C" int pipnet_linear_inter_bwd_f32(const float* x, int64_t n, int E, const float* g, const float* w,
                                           float* dx, float* dw, int accumulate, float* partial, void* stream) {
  if (n < 0 || E <= 0 || E > LI_EMAX || !x || !g || !w || !dw || !partial) return PIPNET_ERR_ARG;
  const hipStream_t s = (hipStream_t)stream;
  switch (E) {
#define LI_CASE(EE)                                                                                             \
  case EE:                                                                                                      \
    hipLaunchKernelGGL(linear_inter_bwd_kernel<EE>, dim3(LI_BLOCKS), dim3(LI_T), 0, s, x, g, w, n, dx, partial); \
    break;
    LI_CASE(1) LI_CASE(2) LI_CASE(3) LI_CASE(4) LI_CASE(5) LI_CASE(6) LI_CASE(7) LI_CASE(8)
    LI_CASE(9) LI_CASE(10) LI_CASE(11) LI_CASE(12) LI_CASE(13) LI_CASE(14) LI_CASE(15) LI_CASE(16)
#undef LI_CASE
    default: return PIPNET_ERR_ARG;
  }
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(linear_inter_dw_kernel, dim3(1), dim3(64), 0, s, partial, E, dw, accumulate);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
