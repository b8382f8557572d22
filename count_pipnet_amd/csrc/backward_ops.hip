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

__global__ __launch_bounds__(WG_T, 2) void wgrad_kernel(const float* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ B, int64_t ldb, int M, int N1,
                                                        int N2, int mchunk, int t2n, float* __restrict__ out,
                                                        int64_t ldo, int64_t split_stride) {
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
  f32x4 ra[4], rb[4];
  auto gload = [&](int m0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = m0 + lr + 8 * q;
      const bool mok = m < m_end;
      ra[q] = (mok && a_ok) ? ld4(A + (int64_t)m * lda + n1_0 + lc) : f32x4{0.f, 0.f, 0.f, 0.f};
      rb[q] = (mok && b_ok) ? ld4(B + (int64_t)m * ldb + n2_0 + lc) : f32x4{0.f, 0.f, 0.f, 0.f};
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

int wgrad_splits(int M, int N1, int N2) {
  const int tiles = ((N1 + WB1 - 1) / WB1) * ((N2 + WB2 - 1) / WB2);
  const int ktiles = (M + WBK - 1) / WBK;
  int s = (512 + tiles - 1) / tiles;                   // >= 2 workgroups per CU
  s = s < ktiles / 8 ? s : ktiles / 8;                 // every slab >= 8 K-tiles
  return s < 1 ? 1 : (s > 256 ? 256 : s);
}

}  // namespace

extern "C" int64_t pipnet_wgrad_workspace_bytes(int M, int N1, int N2) {
  if (M <= 0 || N1 <= 0 || N2 <= 0) return 0;
  const int s = wgrad_splits(M, N1, N2);
  return (int64_t)s * N1 * N2 * (int64_t)sizeof(float);
}

extern "C" int pipnet_wgrad_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int M, int N1, int N2,
                                float* C, int64_t ldc, int accumulate, float* workspace, void* stream) {
  if (M < 0 || N1 <= 0 || N2 <= 0 || !A || !B || !C) return PIPNET_ERR_ARG;
  if ((N1 & 3) || (N2 & 3) || (lda & 3) || (ldb & 3) || lda < N1 || ldb < N2 || ldc < N2) return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(B)) return PIPNET_ERR_ALIGN;
  hipStream_t s = (hipStream_t)stream;
  const int splits = M > 0 ? wgrad_splits(M, N1, N2) : 1;
  const int t2n = (N2 + WB2 - 1) / WB2;
  const int tiles = ((N1 + WB1 - 1) / WB1) * t2n;
  const int ktiles = (M + WBK - 1) / WBK;
  const int mchunk = ((ktiles + splits - 1) / splits) * WBK;
  const bool direct = splits == 1 && !accumulate;
  if (!direct && !workspace) return PIPNET_ERR_ARG;
  float* out = direct ? C : workspace;
  const int64_t ldo = direct ? ldc : N2;
  hipLaunchKernelGGL(wgrad_kernel, dim3((unsigned)tiles, (unsigned)splits), dim3(WG_T), 0, s, A, lda, B, ldb, M, N1,
                     N2, mchunk, t2n, out, ldo, (int64_t)N1 * N2);
  PIPNET_CHECK_LAUNCH();
  if (!direct) {
    const int64_t total = (int64_t)N1 * N2;
    const int64_t g = (total + 255) / 256;
    hipLaunchKernelGGL(split_reduce_kernel, dim3((unsigned)(g < 8192 ? g : 8192)), dim3(256), 0, s, workspace, splits,
                       N1, N2, C, ldc, accumulate);
    PIPNET_CHECK_LAUNCH();
  }
  return PIPNET_OK;
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
