// Backward building blocks for training the trainable ConvNeXt stages:
//
//   * wgrad: C[N1][N2] (+)= sum_m A[m][N1] B[m][N2] -- the weight gradient of a Linear /
//     1x1 conv (dW = dY^T X) with the reduction over the B*H*W pixel rows.  Both operands are
//     pixel-major exactly as the forward stores them, and that is the layout the fp32 MFMA
//     32x32x2 wants: its A operand A[i][k] (i = output row = N1 index, k = reduction = pixel)
//     and B operand B[k][j] are read from LDS tiles stored [pixel][channel] as written by
//     coalesced row loads -- no transposes anywhere.  128x128 output tile per workgroup,
//     32 pixels per K-tile, register-staged double buffer (one barrier per K-tile), split
//     over pixels into fixed slabs reduced in a fixed order (deterministic).
//   * colsum: out[n] (+)= sum_m A[m][n] (bias / LayerNorm-shift gradients), fixed-order
//     split reduction.
#include "common.hpp"

namespace {

constexpr int WG_T = 256, WB1 = 128, WB2 = 128, WBK = 32, WPAD = 4;
constexpr int WLD1 = WB1 + WPAD, WLD2 = WB2 + WPAD;    // padded rows: the two half-waves
                                                         // (k and k+1) hit different banks

// B operand gather of a KHxKW (stride s, zero padding p) conv's weight gradient -- the 2x2
// downsample convs, the 4x4/4 ConvNeXt stem and the ResNet 3x3 / strided 1x1 convs: row m =
// output pixel (b, oy, ox), column k = tap * Cin + ci -> input x[b][oy*s - p + tap/KW]
// [ox*s - p + tap%KW][ci] (zero outside the image).
struct Conv2x2Geom {
  int H, W, Cin, OH, OW, stride, KW, pad;
};

template <int BCONV>
__global__ __launch_bounds__(WG_T, 2) void wgrad_kernel(const float* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ B, int64_t ldb, int M, int N1,
                                                        int N2, int mchunk, int t2n, float* __restrict__ out,
                                                        int64_t ldo, int64_t split_stride, Conv2x2Geom cg) {
  __shared__ __attribute__((aligned(16))) float As[2][WBK * WLD1];
  __shared__ __attribute__((aligned(16))) float Bs[2][WBK * WLD2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int t1 = blockIdx.x / t2n, t2 = blockIdx.x - t1 * t2n;
  const int n1_0 = t1 * WB1, n2_0 = t2 * WB2;
  const int m_beg = blockIdx.y * mchunk;
  const int m_end = min(M, m_beg + mchunk);
  const int ntiles = m_end > m_beg ? (m_end - m_beg + WBK - 1) / WBK : 0;
  const int lr = tid >> 5, lc = 4 * (tid & 31);      // loader: rows lr + 8q, columns lc..lc+3
  const bool a_ok = n1_0 + lc < N1, b_ok = n2_0 + lc < N2;
  int t_ky = 0, t_kx = 0, t_ci = 0;                   // conv gather: this thread's tap / channel
  if (BCONV) {
    const int k = n2_0 + lc, tap = k / cg.Cin;
    t_ci = k - tap * cg.Cin;
    t_ky = tap / cg.KW - cg.pad;
    t_kx = tap % cg.KW - cg.pad;
  }
  f32x4 ra[4], rb[4];
  auto gload = [&](int m0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = m0 + lr + 8 * q;
      const bool mok = m < m_end;
      ra[q] = (mok && a_ok) ? ld4(A + (int64_t)m * lda + n1_0 + lc) : f32x4{0.f, 0.f, 0.f, 0.f};
      if (BCONV) {
        const int mm = mok ? m : 0, ohw = cg.OH * cg.OW;
        const int b = mm / ohw, r = mm - b * ohw, oy = r / cg.OW, ox = r - oy * cg.OW;
        const int iy = oy * cg.stride + t_ky, ix = ox * cg.stride + t_kx;
        const bool in = (unsigned)iy < (unsigned)cg.H && (unsigned)ix < (unsigned)cg.W;
        const float* src = B + (((int64_t)b * cg.H + (in ? iy : 0)) * cg.W + (in ? ix : 0)) * cg.Cin + t_ci;
        rb[q] = (mok && b_ok && in) ? ld4(src) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
        rb[q] = (mok && b_ok) ? ld4(B + (int64_t)m * ldb + n2_0 + lc) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      st4(&As[buf][(lr + 8 * q) * WLD1 + lc], ra[q]);
      st4(&Bs[buf][(lr + 8 * q) * WLD2 + lc], rb[q]);
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
  const int wn1 = (wid >> 1) * 64, wn2 = (wid & 1) * 64;
  const int li = lane & 31, lk = lane >> 5;
  if (ntiles > 0) {
    gload(m_beg);
    sstore(0);
  }
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < ntiles) gload(m_beg + (kt + 1) * WBK);   // next K-tile in flight during the MFMAs
    const float* as = As[buf];
    const float* bs = Bs[buf];
#pragma unroll
    for (int kk = 0; kk < WBK / 2; ++kk) {
      const int row = 2 * kk + lk;
      const float a0 = as[row * WLD1 + wn1 + li], a1 = as[row * WLD1 + wn1 + 32 + li];
      const float b0 = bs[row * WLD2 + wn2 + li], b1 = bs[row * WLD2 + wn2 + 32 + li];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < ntiles) sstore(buf ^ 1);    // buf^1 was last read before the previous barrier
    __syncthreads();
  }
  float* o = out + (int64_t)blockIdx.y * split_stride;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n2 = n2_0 + wn2 + 32 * j + li;
      if (n2 >= N2) continue;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int n1 = n1_0 + wn1 + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * lk;
        if (n1 < N1) o[(int64_t)n1 * ldo + n2] = acc[i][j][v];
      }
    }
}

// C = (accumulate ? C : 0) + sum_s ws[s], s in increasing order.
__global__ __launch_bounds__(256) void split_reduce_kernel(const float* __restrict__ ws, int splits, int N1, int N2,
                                                           float* __restrict__ C, int64_t ldc, int accumulate) {
  const int64_t total = (int64_t)N1 * N2;
  const int64_t slab = total;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int n1 = (int)(i / N2), n2 = (int)(i - (int64_t)n1 * N2);
    float s = ws[i];
    for (int sp = 1; sp < splits; ++sp) s += ws[sp * slab + i];
    float* c = C + (int64_t)n1 * ldc + n2;
    *c = accumulate ? *c + s : s;
  }
}

constexpr int CS_SPLITS = 64;

// partial[s][n] = sum over rows m = s, s + S, ... (S = gridDim.y) -- strided so each slab
// touches the whole matrix evenly; fixed order within a slab.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const float* __restrict__ A, int64_t lda, int M, int N,
                                                             float* __restrict__ partial) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int m = blockIdx.y; m < M; m += gridDim.y) s += A[(int64_t)m * lda + n];
  partial[(int64_t)blockIdx.y * N + n] = s;
}

__global__ __launch_bounds__(256) void colsum_finish_kernel(const float* __restrict__ partial, int splits, int N,
                                                            float* __restrict__ out, int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int sp = 0; sp < splits; ++sp) s += partial[(int64_t)sp * N + n];
  out[n] = accumulate ? out[n] + s : s;
}

// Slabs over the pixel rows: the fewest slabs s within 3 % of the minimum of the workgroup
// rounds per unit of work, ceil(tiles * s / 512) / s (2 workgroups per CU), every slab >= 8
// K-tiles.  (The
// earlier ceil(512 / tiles) overshot 512 workgroups by a few -- 36 tiles x 15 = 540 -- and paid
// a whole second round for them: the ResNet 3x3 weight gradients ran at ~40 TF/s.)
int wgrad_splits(int M, int N1, int N2) {
  const int tiles = ((N1 + WB1 - 1) / WB1) * ((N2 + WB2 - 1) / WB2);
  const int ktiles = (M + WBK - 1) / WBK;
  const int smax = ktiles / 8 < 256 ? ktiles / 8 : 256;
  auto cost = [&](int s) { return (double)(((int64_t)tiles * s + 511) / 512) / s; };
  double best_cost = 1e30;
  for (int s = 1; s <= smax; ++s) best_cost = cost(s) < best_cost ? cost(s) : best_cost;
  // the fewest slabs within 3 % of the best (each slab adds an N1 x N2 partial to reduce)
  for (int s = 1; s <= smax; ++s)
    if (cost(s) <= best_cost * 1.03) return s;
  return 1;
}

}  // namespace

extern "C" int64_t pipnet_wgrad_workspace_bytes(int M, int N1, int N2) {
  if (M <= 0 || N1 <= 0 || N2 <= 0) return 0;
  const int s = wgrad_splits(M, N1, N2);
  return (int64_t)s * N1 * N2 * (int64_t)sizeof(float);
}

namespace {
int wgrad_launch(const float* A, int64_t lda, const float* B, int64_t ldb, int M, int N1, int N2, float* C,
                 int64_t ldc, int accumulate, float* workspace, hipStream_t s, const Conv2x2Geom* cg) {
  const int splits = M > 0 ? wgrad_splits(M, N1, N2) : 1;
  const int t2n = (N2 + WB2 - 1) / WB2;
  const int tiles = ((N1 + WB1 - 1) / WB1) * t2n;
  const int ktiles = (M + WBK - 1) / WBK;
  const int mchunk = ((ktiles + splits - 1) / splits) * WBK;
  const bool direct = splits == 1 && !accumulate;
  if (!direct && !workspace) return PIPNET_ERR_ARG;
  float* out = direct ? C : workspace;
  const int64_t ldo = direct ? ldc : N2;
  const Conv2x2Geom g = cg ? *cg : Conv2x2Geom{0, 0, 1, 0, 0, 1, 1, 0};
  if (cg)
    hipLaunchKernelGGL(wgrad_kernel<1>, dim3((unsigned)tiles, (unsigned)splits), dim3(WG_T), 0, s, A, lda, B, ldb, M,
                       N1, N2, mchunk, t2n, out, ldo, (int64_t)N1 * N2, g);
  else
    hipLaunchKernelGGL(wgrad_kernel<0>, dim3((unsigned)tiles, (unsigned)splits), dim3(WG_T), 0, s, A, lda, B, ldb, M,
                       N1, N2, mchunk, t2n, out, ldo, (int64_t)N1 * N2, g);
  PIPNET_CHECK_LAUNCH();
  if (!direct) {
    const int64_t total = (int64_t)N1 * N2;
    const int64_t gsz = (total + 255) / 256;
    hipLaunchKernelGGL(split_reduce_kernel, dim3((unsigned)(gsz < 8192 ? gsz : 8192)), dim3(256), 0, s, workspace,
                       splits, N1, N2, C, ldc, accumulate);
    PIPNET_CHECK_LAUNCH();
  }
  return PIPNET_OK;
}
}  // namespace

extern "C" int pipnet_wgrad_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int M, int N1, int N2,
                                float* C, int64_t ldc, int accumulate, float* workspace, void* stream) {
  if (M < 0 || N1 <= 0 || N2 <= 0 || !A || !B || !C) return PIPNET_ERR_ARG;
  if ((N1 & 3) || (N2 & 3) || (lda & 3) || (ldb & 3) || lda < N1 || ldb < N2 || ldc < N2) return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(B)) return PIPNET_ERR_ALIGN;
  return wgrad_launch(A, lda, B, ldb, M, N1, N2, C, ldc, accumulate, workspace, (hipStream_t)stream, nullptr);
}

extern "C" int pipnet_wgrad_conv2x2_f32(const float* dY, const float* x, int B, int H, int W, int Cin, int stride,
                                        int Cout, float* dW, int accumulate, float* workspace, void* stream) {
  if (B <= 0 || H < 2 || W < 2 || Cin <= 0 || Cout <= 0 || (Cin & 3) || (Cout & 3) || (stride != 1 && stride != 2))
    return PIPNET_ERR_ARG;
  if (!dY || !x || !dW) return PIPNET_ERR_ARG;
  if (!aligned16(dY) || !aligned16(x)) return PIPNET_ERR_ALIGN;
  const int OH = (H - 2) / stride + 1, OW = (W - 2) / stride + 1;
  const Conv2x2Geom g{H, W, Cin, OH, OW, stride, 2, 0};
  return wgrad_launch(dY, Cout, x, 4 * Cin, B * OH * OW, Cout, 4 * Cin, dW, 4 * Cin, accumulate, workspace,
                      (hipStream_t)stream, &g);
}

extern "C" int pipnet_wgrad_conv_f32(const float* dY, const float* x, int B, int H, int W, int Cin, int KH, int KW,
                                     int stride, int pad, int Cout, float* dW, int accumulate, float* workspace,
                                     void* stream) {
  if (B <= 0 || KH <= 0 || KW <= 0 || pad < 0 || pad >= KH || pad >= KW || H + 2 * pad < KH || W + 2 * pad < KW ||
      Cin <= 0 || Cout <= 0 || (Cin & 3) || (Cout & 3) || stride <= 0)
    return PIPNET_ERR_ARG;
  if (!dY || !x || !dW) return PIPNET_ERR_ARG;
  if (!aligned16(dY) || !aligned16(x)) return PIPNET_ERR_ALIGN;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  const int K = KH * KW * Cin;
  const Conv2x2Geom g{H, W, Cin, OH, OW, stride, KW, pad};
  return wgrad_launch(dY, Cout, x, K, B * OH * OW, Cout, K, dW, K, accumulate, workspace, (hipStream_t)stream, &g);
}

extern "C" int pipnet_colsum_workspace_bytes(int N) { return N > 0 ? CS_SPLITS * N * (int)sizeof(float) : 0; }

extern "C" int pipnet_colsum_f32(const float* A, int64_t lda, int M, int N, float* out, int accumulate,
                                 float* workspace, void* stream) {
  if (M < 0 || N <= 0 || lda < N || !A || !out || !workspace) return PIPNET_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const unsigned gx = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(gx, CS_SPLITS), dim3(256), 0, s, A, lda, M, N, workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_finish_kernel, dim3(gx), dim3(256), 0, s, workspace, CS_SPLITS, N, out, accumulate);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// =========================================================================================
// Training-step kernels for the trainable ConvNeXt suffix (features[j:], add-on, head).
// Per-channel parameter gradients are accumulated per workgroup (lanes own channels, waves
// own pixels) into partials [G][n][C] and summed in a fixed order (deterministic).
// =========================================================================================
namespace {

constexpr int TB_T = 256;                  // 4 waves
constexpr int TB_G = 512;                  // workgroups of the per-pixel reduction kernels
constexpr float TB_LN_EPS = 1e-6f;

// partial [G][N] -> out[N] (+)= sum_g partial[g][n]
__global__ __launch_bounds__(256) void sum_partials_kernel(const float* __restrict__ partial, int G, int N,
                                                           float* __restrict__ out, int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += partial[(int64_t)g * N + n];
  out[n] = accumulate ? out[n] + s : s;
}

// Reduce per-wave accumulators (NV vectors of C channels, lane-owned float4 chunks) over the
// workgroup's 4 waves in a fixed order and write partial[blockIdx][v][c].
template <int NJ4, int NV>
PIPNET_DEV void wg_partials(f32x4 (&acc)[NV][NJ4], int C, float* __restrict__ partial, float* red) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int v = 0; v < NV; ++v) {
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      if (c < C) st4(red + (wv * C) + c, acc[v][j]);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += TB_T) {
      float s = 0.f;
      for (int w = 0; w < TB_T / 64; ++w) s += red[w * C + c];
      partial[((int64_t)blockIdx.x * NV + v) * C + c] = s;
    }
    __syncthreads();
  }
}

// ---- GELU forward (exact erf, training forward keeps the pre-activation for the backward)
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const float* __restrict__ h, float* __restrict__ g,
                                                       int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 x = ld4(h + 4 * i);
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = gelu_erf(x[e]);
    st4(g + 4 * i, y);
  }
}

// ---- out = x + rs[m / rps] * (ls * y2)    (CNBlock residual with layer scale + stochastic depth)
__global__ __launch_bounds__(256) void resid_scale_kernel(const float* __restrict__ x, const float* __restrict__ y2,
                                                          const float* __restrict__ ls, const float* __restrict__ rs,
                                                          int rps, int C, int64_t n4, float* __restrict__ out) {
  const int c4 = C / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i / c4;
    const int c = 4 * (int)(i - m * c4);
    const float r = rs ? rs[m / rps] : 1.f;
    const f32x4 t = ld4(ls + c) * ld4(y2 + 4 * i);
    st4(out + 4 * i, ld4(x + 4 * i) + r * t);
  }
}

// ---- layer scale / stochastic depth backward, one wave per pixel:
//   dy2 = dy * ls * r;  partial dls += dy * r * y2;  partial db2 += dy2
template <int NJ4>
__global__ __launch_bounds__(TB_T) void ls_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y2,
                                                      const float* __restrict__ ls, const float* __restrict__ rs,
                                                      int rps, int64_t M, int C, float* __restrict__ dy2,
                                                      float* __restrict__ partial) {
  extern __shared__ float red[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  f32x4 acc[2][NJ4];
#pragma unroll
  for (int j = 0; j < NJ4; ++j) acc[0][j] = acc[1][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t m = (int64_t)blockIdx.x * 4 + wv; m < M; m += (int64_t)gridDim.x * 4) {
    const float r = rs ? rs[m / rps] : 1.f;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      if (c < C) {
        const f32x4 d = ld4(dy + m * C + c);
        const f32x4 d2 = d * ld4(ls + c) * r;
        st4(dy2 + m * C + c, d2);
        acc[0][j] += d * r * ld4(y2 + m * C + c);
        acc[1][j] += d2;
      }
    }
  }
  wg_partials<NJ4, 2>(acc, C, partial, red);
}

// ---- LayerNorm backward over C per pixel (torch F.layer_norm, biased variance, eps 1e-6):
//   xh = (z - mu) * rstd;  a = gamma * dt;
//   dz = rstd * (a - mean(a) - xh * mean(a * xh))      (written when dz != NULL)
//   partial dgamma += dt * xh;  partial dbeta += dt
template <int NJ4>
__global__ __launch_bounds__(TB_T) void ln_bwd_kernel(const float* __restrict__ z, const float* __restrict__ dt,
                                                      const float* __restrict__ gamma, int64_t M, int C,
                                                      float* __restrict__ dz, float* __restrict__ partial) {
  extern __shared__ float red[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  f32x4 acc[2][NJ4];
#pragma unroll
  for (int j = 0; j < NJ4; ++j) acc[0][j] = acc[1][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float invC = 1.0f / C;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wv; m < M; m += (int64_t)gridDim.x * 4) {
    f32x4 zv[NJ4], dv[NJ4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      const bool ok = c < C;
      zv[j] = ok ? ld4(z + m * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      dv[j] = ok ? ld4(dt + m * C + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      s += (zv[j][0] + zv[j][1]) + (zv[j][2] + zv[j][3]);
    }
    const float mu = wave_sum(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      if (4 * lane + 256 * j < C) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = zv[j][e] - mu;
          q = fmaf(d, d, q);
        }
      }
    }
    const float rstd = 1.0f / sqrtf(wave_sum(q) * invC + TB_LN_EPS);
    float sa = 0.f, sax = 0.f;
    f32x4 xh[NJ4], av[NJ4];
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      xh[j] = (zv[j] - mu) * rstd;
      av[j] = (c < C) ? ld4(gamma + c) * dv[j] : f32x4{0.f, 0.f, 0.f, 0.f};
      if (c < C) {
        acc[0][j] += dv[j] * xh[j];
        acc[1][j] += dv[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          sa += av[j][e];
          sax = fmaf(av[j][e], xh[j][e], sax);
        }
      }
    }
    if (dz) {
      const float ma = wave_sum(sa) * invC, max_ = wave_sum(sax) * invC;
#pragma unroll
      for (int j = 0; j < NJ4; ++j) {
        const int c = 4 * lane + 256 * j;
        if (c < C) st4(dz + m * C + c, (av[j] - ma - xh[j] * max_) * rstd);
      }
    }
  }
  wg_partials<NJ4, 2>(acc, C, partial, red);
}

// ---- depthwise 7x7 (pad 3) on NHWC, generic C:  y (+)= [bias] + sum_k x[p + k - 3] * w[k][c]
// (w packed [49][C]; the input gradient passes the spatially flipped taps, no bias, accumulate)
__global__ __launch_bounds__(256) void dwconv7_plain_kernel(const float* __restrict__ x, int B, int H, int W, int C,
                                                            const float* __restrict__ wp,
                                                            const float* __restrict__ bias, int accumulate,
                                                            float* __restrict__ y) {
  const int c4 = C / 4;
  const int64_t total = (int64_t)B * H * W * c4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t px = i / c4;
    const int c = 4 * (int)(i - px * c4);
    const int xx = (int)(px % W);
    const int64_t r = px / W;
    const int yy = (int)(r % H);
    const int b = (int)(r / H);
    f32x4 acc = bias ? ld4(bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ky = 0; ky < 7; ++ky) {
      const int iy = yy + ky - 3;
      if ((unsigned)iy >= (unsigned)H) continue;
      const float* row = x + (((int64_t)b * H + iy) * W) * C + c;
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        const int ix = xx + kx - 3;
        if ((unsigned)ix < (unsigned)W) acc += ld4(row + (int64_t)ix * C) * ld4(wp + (ky * 7 + kx) * C + c);
      }
    }
    float* o = y + px * C + c;
    st4(o, accumulate ? ld4(o) + acc : acc);
  }
}

// ---- depthwise 7x7 weight / bias gradient: dw[k][c] = sum_p dz[p][c] * x[p + k - 3][c],
// db[c] = sum_p dz[p][c].  Workgroup (channel quads, kernel row ky, pixel slab): 7 float4
// accumulators per thread; partial [S][50][C] (rows 0..48 taps, 49 bias).
constexpr int DWG_S = 64;
__global__ __launch_bounds__(64) void dwconv7_wgrad_kernel(const float* __restrict__ dz, const float* __restrict__ x,
                                                           int B, int H, int W, int C, float* __restrict__ partial) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  const int ky = blockIdx.y;
  const int s = blockIdx.z;
  const int c = 4 * q;
  if (c >= C) return;
  const int64_t P = (int64_t)B * H * W;
  const int64_t chunk = (P + gridDim.z - 1) / gridDim.z;
  const int64_t p0 = s * chunk, p1 = min(P, p0 + chunk);
  f32x4 acc[7], db = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 7; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t p = p0; p < p1; ++p) {
    const int xx = (int)(p % W);
    const int64_t r = p / W;
    const int yy = (int)(r % H);
    const int b = (int)(r / H);
    const f32x4 d = ld4(dz + p * C + c);
    if (ky == 0) db += d;
    const int iy = yy + ky - 3;
    if ((unsigned)iy >= (unsigned)H) continue;
    const float* row = x + (((int64_t)b * H + iy) * W) * C + c;
#pragma unroll
    for (int kx = 0; kx < 7; ++kx) {
      const int ix = xx + kx - 3;
      if ((unsigned)ix < (unsigned)W) acc[kx] += d * ld4(row + (int64_t)ix * C);
    }
  }
  float* base = partial + (int64_t)s * 50 * C;
#pragma unroll
  for (int kx = 0; kx < 7; ++kx) st4(base + (ky * 7 + kx) * C + c, acc[kx]);
  if (ky == 0) st4(base + 49 * C + c, db);
}

// ---- PIP-Net head backward -----------------------------------------------------------------
// argmax over the h*w pixels of every (image, prototype) -- AdaptiveMaxPool2d's index (first
// maximum in row-major pixel order)
__global__ __launch_bounds__(256) void argmax_hw_kernel(const float* __restrict__ proto, int N, int HW, int P,
                                                        int32_t* __restrict__ idx) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * P) return;
  const int b = (int)(t / P), p = (int)(t - (int64_t)b * P);
  const float* col = proto + (int64_t)b * HW * P + p;
  float best = col[0];
  int bi = 0;
  for (int i = 1; i < HW; ++i) {
    const float v = col[(int64_t)i * P];
    if (v > best) { best = v; bi = i; }
  }
  idx[t] = bi;
}

// d loss / d pooled[b,p] = sum_k d_out[b,k] relu(W[k,p])                      (classifier)
//                        - w_tanh/2 * C/P * (1 - t^2) / (t + 1e-8),  t = tanh(C * sum_{b' in half} pooled[b',p])
__global__ __launch_bounds__(256) void pool_grad_kernel(const float* __restrict__ pooled, int Bh, int P,
                                                        const float* __restrict__ d_out, const float* __restrict__ W,
                                                        int K, float w_tanh, float coeff,
                                                        const float* __restrict__ extra,
                                                        float* __restrict__ dpool) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int N = 2 * Bh;
  if (t >= (int64_t)N * P) return;
  const int b = (int)(t / P), p = (int)(t - (int64_t)b * P);
  float g = 0.f;
  if (d_out) {
    for (int k = 0; k < K; ++k) g = fmaf(d_out[(int64_t)b * K + k], fmaxf(W[(int64_t)k * P + p], 0.f), g);
  }
  if (w_tanh != 0.f) {
    const int h0 = (b / Bh) * Bh;
    float s = 0.f;
    for (int i = 0; i < Bh; ++i) s += coeff * pooled[(int64_t)(h0 + i) * P + p];
    const float th = tanhf(s);
    g += -0.5f * w_tanh / (float)P * coeff * (1.f - th * th) / (th + 1e-8f);
  }
  if (extra) g += extra[t];
  dpool[t] = g;
}

// One wave per pixel pair (view 1 pixel n, view 2 pixel n): align gradient, max-pool
// scatter, softmax backward -> d logits.  a = align weight / 2 / (Bh*HW).
// SUM (CountPIPNet, count_pipnet.py:88 counts = proto.sum((2,3))): every pixel receives
// dpool[b,p]; the softmax backward is scaled by oscale = 1/tau (soft Gumbel-softmax,
// y = softmax((x + g)/tau), the noise g a constant).
template <int NJ4, bool SUM = false>
__global__ __launch_bounds__(TB_T) void head_bwd_kernel(const float* __restrict__ proto, int Bh, int HW, int P,
                                                        const int32_t* __restrict__ amax,
                                                        const float* __restrict__ dpool, float a,
                                                        float* __restrict__ dlogits, float oscale = 1.f) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t npix = (int64_t)Bh * HW;
  for (int64_t n = (int64_t)blockIdx.x * 4 + wv; n < npix; n += (int64_t)gridDim.x * 4) {
    const int b1 = (int)(n / HW), hw = (int)(n - (int64_t)b1 * HW), b2 = b1 + Bh;
    const float* y1p = proto + n * P;
    const float* y2p = proto + (npix + n) * P;
    f32x4 y1[NJ4], y2[NJ4];
    float d = 0.f;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      const bool ok = c < P;
      y1[j] = ok ? ld4(y1p + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      y2[j] = ok ? ld4(y2p + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) d = fmaf(y1[j][e], y2[j][e], d);
    }
    const float g = -a / (wave_sum(d) + 1e-12f);
    f32x4 g1[NJ4], g2[NJ4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      g1[j] = y2[j] * g;
      g2[j] = y1[j] * g;
      if (c < P) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (SUM || amax[(int64_t)b1 * P + c + e] == hw) g1[j][e] += dpool[(int64_t)b1 * P + c + e];
          if (SUM || amax[(int64_t)b2 * P + c + e] == hw) g2[j][e] += dpool[(int64_t)b2 * P + c + e];
          s1 = fmaf(g1[j][e], y1[j][e], s1);
          s2 = fmaf(g2[j][e], y2[j][e], s2);
        }
      }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      if (c < P) {
        st4(dlogits + n * P + c, y1[j] * (g1[j] - s1) * oscale);
        st4(dlogits + (npix + n) * P + c, y2[j] * (g2[j] - s2) * oscale);
      }
    }
  }
}

inline unsigned grid_cap(int64_t n, int64_t cap = 8192) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

// partial [G][N0 + N1] -> out0[n] (+)= sum_g partial[g][n] (n < N0), out1[n - N0] for the rest
__global__ __launch_bounds__(256) void sum_partials2_kernel(const float* __restrict__ partial, int G, int N0, int N1,
                                                            float* __restrict__ out0, float* __restrict__ out1,
                                                            int accumulate) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  const int N = N0 + N1;
  if (n >= N) return;
  float s = 0.f;
  for (int g = 0; g < G; ++g) s += partial[(int64_t)g * N + n];
  float* o = n < N0 ? out0 + n : out1 + (n - N0);
  *o = accumulate ? *o + s : s;
}

int finish2(const float* partial, int G, int N0, int N1, float* out0, float* out1, int accumulate, hipStream_t s) {
  hipLaunchKernelGGL(sum_partials2_kernel, dim3((unsigned)((N0 + N1 + 255) / 256)), dim3(256), 0, s, partial, G, N0,
                     N1, out0, out1, accumulate);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

}  // namespace

extern "C" int64_t pipnet_train_partials_floats(int C) {
  const int64_t a = (int64_t)TB_G * 2 * C, b = (int64_t)DWG_S * 50 * C;
  return a > b ? a : b;
}

extern "C" int pipnet_gelu_fwd_f32(const float* h, float* g, int64_t n, void* stream) {
  if (n < 0 || (n & 3) || !h || !g) return PIPNET_ERR_ARG;
  if (!aligned16(h) || !aligned16(g)) return PIPNET_ERR_ALIGN;
  if (n == 0) return PIPNET_OK;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(grid_cap(n / 4)), dim3(256), 0, (hipStream_t)stream, h, g, n / 4);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_resid_scale_f32(const float* x, const float* y2, const float* ls, const float* row_scale,
                                      int rows_per_scale, int64_t M, int C, float* out, void* stream) {
  if (M < 0 || C <= 0 || (C & 3) || !x || !y2 || !ls || !out || (row_scale && rows_per_scale <= 0))
    return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(y2) || !aligned16(ls) || !aligned16(out)) return PIPNET_ERR_ALIGN;
  const int64_t n4 = M * (C / 4);
  if (n4 == 0) return PIPNET_OK;
  hipLaunchKernelGGL(resid_scale_kernel, dim3(grid_cap(n4)), dim3(256), 0, (hipStream_t)stream, x, y2, ls, row_scale,
                     rows_per_scale, C, n4, out);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}


#define PIPNET_BY_NJ4(C, MACRO)                                         \
  if ((C) <= 256) { MACRO(1) }                                          \
  else if ((C) <= 512) { MACRO(2) }                                     \
  else if ((C) <= 768) { MACRO(3) }                                     \
  else if ((C) <= 1024) { MACRO(4) }                                    \
  else if ((C) <= 2048) { MACRO(8) }                                    \
  else return PIPNET_ERR_ARG;

extern "C" int pipnet_ls_bwd_f32(const float* dy, const float* y2, const float* ls, const float* row_scale,
                                 int rows_per_scale, int64_t M, int C, float* dy2, float* d_ls, float* d_b2,
                                 int accumulate, float* partial, void* stream) {
  if (M <= 0 || C <= 0 || (C & 3) || !dy || !y2 || !ls || !dy2 || !d_ls || !d_b2 || !partial) return PIPNET_ERR_ARG;
  if (row_scale && rows_per_scale <= 0) return PIPNET_ERR_ARG;
  if (!aligned16(dy) || !aligned16(y2) || !aligned16(ls) || !aligned16(dy2)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const size_t sh = (size_t)(TB_T / 64) * C * sizeof(float);
#define PIPNET_LS(NJ)                                                                                      \
  hipLaunchKernelGGL(ls_bwd_kernel<NJ>, dim3(TB_G), dim3(TB_T), sh, s, dy, y2, ls, row_scale, rows_per_scale, \
                     M, C, dy2, partial);
  PIPNET_BY_NJ4(C, PIPNET_LS)
#undef PIPNET_LS
  PIPNET_CHECK_LAUNCH();
  return finish2(partial, TB_G, C, C, d_ls, d_b2, accumulate, s);
}

extern "C" int pipnet_ln_bwd_f32(const float* z, const float* dt, const float* gamma, int64_t M, int C, float* dz,
                                 float* d_gamma, float* d_beta, int accumulate, float* partial, void* stream) {
  if (M <= 0 || C <= 0 || (C & 3) || !z || !dt || !gamma || !d_gamma || !d_beta || !partial) return PIPNET_ERR_ARG;
  if (!aligned16(z) || !aligned16(dt) || !aligned16(gamma) || (dz && !aligned16(dz))) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const size_t sh = (size_t)(TB_T / 64) * C * sizeof(float);
#define PIPNET_LN(NJ)                                                                                            \
  hipLaunchKernelGGL(ln_bwd_kernel<NJ>, dim3(TB_G), dim3(TB_T), sh, s, z, dt, gamma, M, C, dz, partial);
  PIPNET_BY_NJ4(C, PIPNET_LN)
#undef PIPNET_LN
  PIPNET_CHECK_LAUNCH();
  return finish2(partial, TB_G, C, C, d_gamma, d_beta, accumulate, s);
}

extern "C" int pipnet_dwconv7_plain_f32(const float* x, int B, int H, int W, int C, const float* w_packed,
                                        const float* bias, int accumulate, float* y, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || (C & 3) || !x || !w_packed || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(y) || (bias && !aligned16(bias))) return PIPNET_ERR_ALIGN;
  const int64_t total = (int64_t)B * H * W * (C / 4);
  if (total == 0) return PIPNET_OK;
  hipLaunchKernelGGL(dwconv7_plain_kernel, dim3(grid_cap(total, 16384)), dim3(256), 0, (hipStream_t)stream, x, B, H, W,
                     C, w_packed, bias, accumulate, y);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_dwconv7_wgrad_f32(const float* dz, const float* x, int B, int H, int W, int C, float* dw_packed,
                                        float* db, int accumulate, float* partial, void* stream) {
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0 || (C & 3) || !dz || !x || !dw_packed || !db || !partial)
    return PIPNET_ERR_ARG;
  if (!aligned16(dz) || !aligned16(x)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(dwconv7_wgrad_kernel, dim3((unsigned)((C / 4 + 63) / 64), 7, DWG_S), dim3(64), 0, s, dz, x, B, H,
                     W, C, partial);
  PIPNET_CHECK_LAUNCH();
  // partial [S][50][C]: rows 0..48 -> dw_packed [49][C], row 49 -> db
  return finish2(partial, DWG_S, 49 * C, C, dw_packed, db, accumulate, s);
}

extern "C" int pipnet_head_bwd_f32(const float* proto, const float* pooled, int Bh, int HW, int P, const float* d_out,
                                   const float* W, int K, float w_align, float w_tanh, float tanh_coeff,
                                   int32_t* argmax_ws, float* dpool_ws, float* d_logits, void* stream) {
  if (Bh <= 0 || HW <= 0 || P <= 0 || (P & 3) || !proto || !pooled || !argmax_ws || !dpool_ws || !d_logits)
    return PIPNET_ERR_ARG;
  if (d_out && (!W || K <= 0)) return PIPNET_ERR_ARG;
  if (!aligned16(proto) || !aligned16(d_logits)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int64_t NP = (int64_t)2 * Bh * P;
  hipLaunchKernelGGL(argmax_hw_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, proto, 2 * Bh, HW, P,
                     argmax_ws);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(pool_grad_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, pooled, Bh, P, d_out, W,
                     K, w_tanh, tanh_coeff, nullptr, dpool_ws);
  PIPNET_CHECK_LAUNCH();
  const float a = 0.5f * w_align / (float)((int64_t)Bh * HW);
#define PIPNET_HB(NJ)                                                                                            \
  hipLaunchKernelGGL(head_bwd_kernel<NJ>, dim3(TB_G * 2), dim3(TB_T), 0, s, proto, Bh, HW, P, argmax_ws, dpool_ws, \
                     a, d_logits);
  PIPNET_BY_NJ4(P, PIPNET_HB)
#undef PIPNET_HB
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// ---- CountPIPNet head / count backward (pretrain and joint phases) -------------------------
// d counts of the STE chain (count_pipnet.py:90-97): counts_raw -> [STE_Round] -> ClampSTE(0,
// max) -> intermediate.  STE_Round passes the gradient through (count_pipnet_utils.py:52-55);
// ClampSTE "Gated" (:67-84) keeps it where its input lies in [0, max], "Identity" passes it.
// Without STE the forward is torch.clamp(counts) (train mode: no rounding), whose backward is
// the same gate on the raw counts.
__global__ __launch_bounds__(256) void count_ste_bwd_kernel(const float* __restrict__ counts, int64_t n,
                                                            float max_count, int use_ste, int gated,
                                                            const float* __restrict__ d_clamped,
                                                            float* __restrict__ d_counts) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float x = use_ste ? rintf(counts[i]) : counts[i];
    const bool pass = !gated || (x >= 0.f && x <= max_count);
    d_counts[i] = pass ? d_clamped[i] : 0.f;
  }
}

// ModifiedSTEFunction.backward (count_pipnet_utils.py:226-321) over rows (b,p) of the
// encoding gradient g [rows][M].  x = the encoder's input (clamped counts); r = rint(x);
// cur = clamp(int(r) - 1, 0, M - 1).  Rows with r < 0.1 get 0 (the reference's chained
// mask assignment `counts_grad[zero_mask][neg] = ...` writes a temporary).  Otherwise, with
// (mn, mi) = min over M (first index) and allpos = mn > 0:
//   strategy 2 ('max_grad') and some non-zero row of the batch allpos: allpos rows -> max
//     over M; the others 0 (`final_grad_nz[std][dec] = ...` also writes a temporary);
//   else: mag = |mn| (strategy 1 'current_grad' and allpos: g[cur]); mi < cur -> +mag,
//     mi > cur -> -mag, else 0;
//   respect_active and g[cur] < 0 -> 0.
__device__ __forceinline__ void onehot_row(const float* __restrict__ g, int M, float& mn, int& mi, float& mx) {
  mn = g[0]; mi = 0; mx = g[0];
  for (int k = 1; k < M; ++k) {
    const float v = g[k];
    if (v < mn) { mn = v; mi = k; }
    mx = fmaxf(mx, v);
  }
}

__global__ __launch_bounds__(256) void onehot_ste_flag_kernel(const float* __restrict__ x, int64_t rows, int M,
                                                              const float* __restrict__ g, int* __restrict__ flag) {
  bool any = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < rows; i += (int64_t)gridDim.x * 256) {
    if (!(rintf(x[i]) < 0.1f)) {
      float mn, mx;
      int mi;
      onehot_row(g + i * M, M, mn, mi, mx);
      any |= mn > 0.f;
    }
  }
  if (__ballot(any) != 0 && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

__global__ void zero_flag_kernel(int* __restrict__ flag) {
  if (threadIdx.x == 0) *flag = 0;
}

__global__ __launch_bounds__(256) void onehot_ste_bwd_kernel(const float* __restrict__ x, int64_t rows, int M,
                                                             const float* __restrict__ g, int strategy,
                                                             int respect_active, const int* __restrict__ flag,
                                                             float* __restrict__ dx) {
  const bool global_allpos = strategy == 2 && *flag;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < rows; i += (int64_t)gridDim.x * 256) {
    const float r = rintf(x[i]);
    float out = 0.f;
    if (!(r < 0.1f)) {
      const float* gi = g + i * M;
      int cur = (int)r - 1;
      cur = cur < 0 ? 0 : (cur > M - 1 ? M - 1 : cur);
      float mn, mx;
      int mi;
      onehot_row(gi, M, mn, mi, mx);
      const bool allpos = mn > 0.f;
      if (global_allpos) {
        out = allpos ? mx : 0.f;
      } else {
        const float mag = (strategy == 1 && allpos) ? gi[cur] : fabsf(mn);
        out = mi < cur ? mag : (mi > cur ? -mag : 0.f);
      }
      if (respect_active && gi[cur] < 0.f) out = 0.f;
    }
    dx[i] = out;
  }
}

extern "C" int pipnet_count_ste_bwd_f32(const float* counts, int64_t n, int max_count, int use_ste, int gated,
                                        const float* d_clamped, float* d_counts, void* stream) {
  if (n < 0 || max_count < 0 || !counts || !d_clamped || !d_counts) return PIPNET_ERR_ARG;
  if (n == 0) return PIPNET_OK;
  hipLaunchKernelGGL(count_ste_bwd_kernel, dim3(grid_cap(n)), dim3(256), 0, (hipStream_t)stream, counts, n,
                     (float)max_count, use_ste, gated, d_clamped, d_counts);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_onehot_ste_bwd_f32(const float* x, int64_t rows, int M, const float* g, int strategy,
                                         int respect_active, int* flag_ws, float* dx, void* stream) {
  if (rows < 0 || M <= 0 || strategy < 0 || strategy > 2 || !x || !g || !flag_ws || !dx) return PIPNET_ERR_ARG;
  if (rows == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(zero_flag_kernel, dim3(1), dim3(64), 0, s, flag_ws);
  PIPNET_CHECK_LAUNCH();
  if (strategy == 2) {
    hipLaunchKernelGGL(onehot_ste_flag_kernel, dim3(grid_cap(rows)), dim3(256), 0, s, x, rows, M, g, flag_ws);
    PIPNET_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(onehot_ste_bwd_kernel, dim3(grid_cap(rows)), dim3(256), 0, s, x, rows, M, g, strategy,
                     respect_active, flag_ws, dx);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// d logits of the CountPIPNet head: counts = spatial sums of proto = softmax((logits + g)/tau)
// (tau = 1, g = 0 for the plain Softmax add-on).  d counts = d_counts_in (the classifier /
// intermediate / STE chain, may be NULL) + the tanh term on C * counts; the align term as the
// PIP-Net head.  proto NHWC [2Bh][HW][P], counts [2Bh][P], dcnt_ws float [2Bh*P].
extern "C" int pipnet_count_head_bwd_f32(const float* proto, const float* counts, int Bh, int HW, int P,
                                         const float* d_counts_in, float w_align, float w_tanh, float tanh_coeff,
                                         float inv_tau, float* dcnt_ws, float* d_logits, void* stream) {
  if (Bh <= 0 || HW <= 0 || P <= 0 || (P & 3) || !proto || !counts || !dcnt_ws || !d_logits) return PIPNET_ERR_ARG;
  if (!aligned16(proto) || !aligned16(d_logits)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int64_t NP = (int64_t)2 * Bh * P;
  hipLaunchKernelGGL(pool_grad_kernel, dim3((unsigned)((NP + 255) / 256)), dim3(256), 0, s, counts, Bh, P, nullptr,
                     nullptr, 0, w_tanh, tanh_coeff, d_counts_in, dcnt_ws);
  PIPNET_CHECK_LAUNCH();
  const float a = 0.5f * w_align / (float)((int64_t)Bh * HW);
#define PIPNET_CHB(NJ)                                                                                           \
  hipLaunchKernelGGL((head_bwd_kernel<NJ, true>), dim3(TB_G * 2), dim3(TB_T), 0, s, proto, Bh, HW, P, nullptr,  \
                     dcnt_ws, a, d_logits, inv_tau);
  PIPNET_BY_NJ4(P, PIPNET_CHB)
#undef PIPNET_CHB
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
