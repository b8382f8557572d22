// fp64-accumulated fp32 matrix product on gfx950 matrix cores (v_mfma_f64_16x16x4_f64):
//   C[M,N] (fp32) = RNE_f32( sum_k double(A[m,k]) * double(B[k,n]) ),  A, B row-major fp32.
//
// Folds CountPIPNet's BilinearIntermediate embedding into its two projections for inference
// (count_pipnet_utils.py:378-385: W(embed(x)) * V(embed(x)) with three bias-free Linears, so
// W(E x) = (W E) x): the folded [D, P] weights W.E and V.E are taken here, once per weight
// version (count_pipnet._bilinear_folded), instead of through a vendor DGEMM.  fp32 inputs
// convert exactly to fp64, every product is exact in fp64, the sums carry ~1e-16 relative
// error, and the result is rounded once to fp32 -- the same values as a float64 torch matmul
// rounded to float32 except where a sum lies within 1e-16 of an fp32 rounding midpoint.
//
// Tile: 64 x 64 outputs per 256-thread workgroup, 16-deep K tiles staged in LDS as fp64; each
// wave owns a 32 x 32 quadrant = 2 x 2 MFMA 16x16 tiles.  f64 operand maps (gfx950,
// cdna_hip_programming.md section 3): lane l holds A[l & 15][k = l >> 4], B[k = l >> 4][l & 15];
// the accumulator element r of lane l is row (l >> 4) + 4 r, column l & 15.  This runs off the
// steady-state forward (a weight change triggers it), so the tile favours simplicity: one LDS
// stage, plain loads with bounds checks, any M, N, K.
#include "common.hpp"

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, BK = 16, NT = 256;
constexpr int ALD = BK + 1;       // A rows padded: the 16 rows of an operand read hit distinct banks
constexpr int BLD = BN + 2;

__global__ __launch_bounds__(NT) void fold_f64_kernel(const float* __restrict__ A, int64_t lda,
                                                      const float* __restrict__ B, int64_t ldb, float* __restrict__ C,
                                                      int64_t ldc, int M, int N, int K) {
  __shared__ double As[BM * ALD];
  __shared__ double Bs[BK * BLD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int ar = tid >> 2, ak = (tid & 3) * 4;      // A: 64 rows x 16 k, 4 per thread
  const int bk = tid >> 4, bn = (tid & 15) * 4;     // B: 16 k x 64 columns, 4 per thread
  f64x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

  for (int k0 = 0; k0 < K; k0 += BK) {
    const int gm = m0 + ar, gka = k0 + ak;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      As[ar * ALD + ak + e] = (gm < M && gka + e < K) ? (double)A[(int64_t)gm * lda + gka + e] : 0.0;
    const int gkb = k0 + bk, gn = n0 + bn;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      Bs[bk * BLD + bn + e] = (gkb < K && gn + e < N) ? (double)B[(int64_t)gkb * ldb + gn + e] : 0.0;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int k = kk + (lane >> 4);
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[(wm * 32 + i * 16 + (lane & 15)) * ALD + k];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[k * BLD + wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + (lane >> 4) + 4 * r;
        const int n = n0 + wn * 32 + j * 16 + (lane & 15);
        if (m < M && n < N) C[(int64_t)m * ldc + n] = (float)acc[i][j][r];
      }
}

}  // namespace

extern "C" int pipnet_matmul_f64acc_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                                        int64_t ldc, int M, int N, int K, void* stream) {
  if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < N || ldc < N) return PIPNET_ERR_ARG;
  if ((M + BM - 1) / BM > 65535) return PIPNET_ERR_ARG;
  const dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM);
  hipLaunchKernelGGL(fold_f64_kernel, grid, dim3(NT), 0, (hipStream_t)stream, A, lda, B, ldb, C, ldc, M, N, K);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
