// fp64-accumulated fp32 matrix product on gfx950 matrix cores (v_mfma_f64_16x16x4_f64):
//   C[M,N] (fp32) = RNE_f32( sum_k double(A[m,k]) * double(B[k,n]) ),  A, B row-major fp32.
//
// Folds CountPIPNet's BilinearIntermediate embedding into its two projections for inference
// (count_pipnet_utils.py:378-385: W(embed(x)) * V(embed(x)) with three bias-free Linears, so
// W(E x) = (W E) x): the folded [D, P] weights W.E and V.E are taken here, once per weight
// version (count_pipnet._bilinear_folded), as ONE launch of two products sharing B, instead of
// through a vendor DGEMM.  fp32 inputs convert exactly to fp64, every product is exact in fp64,
// the sums carry ~1e-16 relative error, and the result is rounded once to fp32 -- the same
// values as a float64 torch matmul rounded to float32 except where a sum lies within 1e-16 of
// an fp32 rounding midpoint.
//
// Tile (round 5; the round-4 64x64 tile with one LDS stage and scalar loads read 7.7x its
// operands and ran at 0.44 of the fp64 matrix peak): 128 x 128 outputs per 256-thread
// workgroup, 16-deep K-tiles kept in LDS as fp32 (converted to fp64 at the fragment read), two
// LDS stages with the next K-tile's float4 global loads in registers under the current one's
// 64 MFMAs per wave, one barrier per K-tile.  Each wave owns 64 x 64 outputs = 4 x 4 MFMA 16x16
// blocks, and the block -> row map is interleaved (block i, MFMA row j -> tile row 4 j + i, the
// same for columns) so ONE ds_read_b128 gives a lane its operand for all four blocks, and the
// four column blocks of an accumulator row leave as one float4 store.
// f64 operand maps (gfx950, cdna_hip_programming.md section 3): lane l holds A[l & 15][k = l >> 4]
// and B[k = l >> 4][l & 15]; accumulator element r of lane l is row (l >> 4) + 4 r, column l & 15.
// Raster: 1-D grid, XCD-contiguous tile ranges, n fastest -- the ~64 tiles resident on an XCD
// are 4 row panels x 16 column panels moving through K together, so each K-slice of A and B is
// fetched into that XCD's L2 once and re-read from there.
#include "common.hpp"

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 16, NT = 256;
constexpr int LDS_LD = 128 + 4;   // fp32 per LDS k-row (16-B pad: the transposed A writes hit 64 banks)

struct FoldParams {
  const float* A[2];
  float* C[2];
  const float* B;
  int64_t lda, ldb, ldc;
  int M, N, K, mt, nt, ntiles;
};

PIPNET_DEV f32x4 ld4_guard(const float* row, int k, int K, bool ok, bool vec) {
  if (!ok) return f32x4{0.f, 0.f, 0.f, 0.f};
  if (vec && k + 3 < K) return ld4(row + k);
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = k + e < K ? row[k + e] : 0.f;
  return v;
}

template <bool VEC>
__global__ __launch_bounds__(NT, 2) void fold_f64_kernel(FoldParams p) {
  __shared__ __attribute__((aligned(16))) float As[2][BK * LDS_LD];   // [k][m]
  __shared__ __attribute__((aligned(16))) float Bs[2][BK * LDS_LD];   // [k][n]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tile = xcd_remap(blockIdx.x, p.ntiles);
  const int ntile = tile % p.nt, mrow = tile / p.nt;
  const int prod = mrow / p.mt;
  const int m0 = (mrow - prod * p.mt) * BM, n0 = ntile * BN;
  const float* __restrict__ A = p.A[prod];
  float* __restrict__ C = p.C[prod];

  // global -> register staging: A rows m = (tid >> 2) + 64 i, k = 4 (tid & 3) (four lanes read
  // one row's 64 B); B k-rows (tid >> 5) + 8 i, columns 4 (tid & 31) (512 B per k-row)
  const int akq = tid & 3, arow = tid >> 2;
  const int bc4 = tid & 31, bkr = tid >> 5;
  const float* arp[2];
  bool aok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + arow + 64 * i;
    aok[i] = m < p.M;
    arp[i] = A + (int64_t)(aok[i] ? m : 0) * p.lda;
  }
  const int bn = n0 + 4 * bc4;
  const bool bvec = VEC && bn + 3 < p.N;
  f32x4 ra[2], rb[2];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = ld4_guard(arp[i], k0 + 4 * akq, p.K, aok[i], VEC);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int k = k0 + bkr + 8 * i;
      const float* row = p.B + (int64_t)(k < p.K ? k : 0) * p.ldb;
      if (k >= p.K) {
        rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else if (bvec) {
        rb[i] = ld4(row + bn);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) rb[i][e] = bn + e < p.N ? row[bn + e] : 0.f;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) As[buf][(4 * akq + e) * LDS_LD + arow + 64 * i] = ra[i][e];
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<f32x4*>(&Bs[buf][(bkr + 8 * i) * LDS_LD + 4 * bc4]) = rb[i];
  };

  f64x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

  const int nk = (p.K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  // fragment offsets: k-row (lane >> 4) of each 4-deep step, 4 consecutive rows / columns 4 (lane & 15)
  const int fa = (lane >> 4) * LDS_LD + wm * 64 + 4 * (lane & 15);
  const int fb = (lane >> 4) * LDS_LD + wn * 64 + 4 * (lane & 15);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const f32x4 av = ld4(&As[cur][ks * 4 * LDS_LD + fa]);
      const f32x4 bv = ld4(&Bs[cur][ks * 4 * LDS_LD + fb]);
      double bd[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bd[j] = (double)bv[j];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double ad = (double)av[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ad, bd[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  // block i, accumulator row rho = (lane >> 4) + 4 r -> tile row 4 rho + i; column block j,
  // lane column c = lane & 15 -> tile column 4 c + j: the four j of one (i, r) are 4 adjacent floats
  const int nb = n0 + wn * 64 + 4 * (lane & 15);
  const bool nvec = VEC && nb + 3 < p.N;
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + 4 * ((lane >> 4) + 4 * r) + i;
      if (m >= p.M) continue;
      float* dst = C + (int64_t)m * p.ldc + nb;
      const f32x4 v = {(float)acc[i][0][r], (float)acc[i][1][r], (float)acc[i][2][r], (float)acc[i][3][r]};
      if (nvec) {
        *reinterpret_cast<f32x4*>(dst) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (nb + e < p.N) dst[e] = v[e];
      }
    }
}

int launch_fold(const float* A0, const float* A1, int64_t lda, const float* B, int64_t ldb, float* C0, float* C1,
                int64_t ldc, int M, int N, int K, hipStream_t s) {
  if (!A0 || !B || !C0 || (A1 == nullptr) != (C1 == nullptr)) return PIPNET_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0 || lda < K || ldb < N || ldc < N) return PIPNET_ERR_ARG;
  FoldParams p{};
  p.A[0] = A0; p.A[1] = A1 ? A1 : A0;
  p.C[0] = C0; p.C[1] = C1 ? C1 : C0;
  p.B = B; p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.mt = (M + BM - 1) / BM;
  p.nt = (N + BN - 1) / BN;
  const int64_t tiles = (int64_t)p.mt * p.nt * (A1 ? 2 : 1);
  if (tiles > (1LL << 30)) return PIPNET_ERR_ARG;
  p.ntiles = (int)tiles;
  const bool vec = (lda % 4 == 0) && (ldb % 4 == 0) && (ldc % 4 == 0) && aligned16(A0) && aligned16(B) &&
                   aligned16(C0) && (!A1 || (aligned16(A1) && aligned16(C1)));
  if (vec) hipLaunchKernelGGL(fold_f64_kernel<true>, dim3(p.ntiles), dim3(NT), 0, s, p);
  else hipLaunchKernelGGL(fold_f64_kernel<false>, dim3(p.ntiles), dim3(NT), 0, s, p);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

}  // namespace

extern "C" int pipnet_matmul_f64acc_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* C,
                                        int64_t ldc, int M, int N, int K, void* stream) {
  return launch_fold(A, nullptr, lda, B, ldb, C, nullptr, ldc, M, N, K, (hipStream_t)stream);
}

extern "C" int pipnet_matmul2_f64acc_f32(const float* A0, const float* A1, int64_t lda, const float* B, int64_t ldb,
                                         float* C0, float* C1, int64_t ldc, int M, int N, int K, void* stream) {
  if (!A1 || !C1) return PIPNET_ERR_ARG;
  return launch_fold(A0, A1, lda, B, ldb, C0, C1, ldc, M, N, K, (hipStream_t)stream);
}
