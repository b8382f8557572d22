// Product instantiation of the fp32 MFMA GEMM (templates + design notes: gemm_f32_impl.hpp).
#include "gemm_f32_impl.hpp"

using namespace pipnet_gemm;

namespace {

// Raster: consecutive tile ids walk group_m M-tiles before advancing N, sized so the A
// panels of one group (group_m x 128 rows x K) stay within ~2 MiB of an XCD's 4 MiB L2.
#ifndef PIPNET_GROUP_BUDGET
#define PIPNET_GROUP_BUDGET (2.0 * 1024 * 1024)
#endif
int choose_group_m(const GemmParams& p) {
  const double panel = 128.0 * p.K * 4.0;
  int g = (int)(PIPNET_GROUP_BUDGET / panel);
  return g < 1 ? 1 : (g > 16 ? 16 : g);
}

// Variant selection (measured with tools/gemm_lab.py on the network's shapes, MI355X,
// float4 epilogue, profiles/r01/gemm_lab_*.txt):
//   K <= 96, N > 192          BK=16, 128-row tiles, 3 LDS stages      (+11 % on stage-1 fc1)
//   N <= 384 or K <= 192      BK=32,  64-row tiles, 3 workgroups/CU   (+5..+8 %: shallow grids)
//   or M <= 64
//   otherwise                 BK=32, 128-row tiles, 2 LDS stages      (stage-3/4 fc1, fc2)
//   N = 384, K >= 768         BK=32, 192 x 384 tiles, 12 waves        (stage-3 fc2, round 6)
// 0 = register-staged K-tail kernel, 1 = BK16x128 rows x3 stages, 2 = BK32x64 rows,
// 3 = BK32x128 rows, 5 = BK32 192 x 384 wide tile on 12 waves (exported by pipnet_linear_f32_plan;
// the profiling labels of count_pipnet_amd/kernels.py:gemm_kernel_name come from it).  An 8-wave 256 x 128 workgroup
// (gemm_f32_impl.hpp gemm_f32_tn8_kernel, tools/gemm_lab.hip 60+) beat variant 3 by 4-8 % on the
// stage-4 shapes in the lab but not inside C2 (profiles/r06/gemm_tn8_ab.txt): not dispatched.
// (PIPNET_AB_GEMM_RULE: build-time A/B hook for tools/ab_build.py, 0 in the product)
#ifndef PIPNET_AB_GEMM_RULE
#define PIPNET_AB_GEMM_RULE 0
#endif
int gemm_variant(int M, int N, int K, bool vec, int epi, int aload, bool vec_epi) {
  if (!vec) return 0;
  if (K % 16 == 0 && K <= 96 && N > 192 && M > 64) return 1;
  if (K % 32) return K % 16 == 0 && M > 64 ? 1 : 0;
  if (PIPNET_AB_GEMM_RULE == 1 && N == 384 && K >= 1536 && M > 64) return 3;   // stage-3 fc2 on 128-row tiles
  if (PIPNET_AB_GEMM_RULE == 2 && N == 1536 && K == 384) return 2;              // stage-3 fc1 on 64-row tiles
  // wide short-K (C5's add-on 1x1 conv, 192 -> 2048 prototypes): 128-row tiles -- 2,048 tiles in
  // four full rounds of 2 per CU instead of 4,096 64-row tiles in 5.3 rounds of 3; C5 +0.8 % in
  // four interleaved rounds (profiles/r05/ab_c5_addon_tile.txt).  Same K order: bitwise equal.
  if (N >= 1024 && N % BN == 0 && K <= 192 && M > 64) return 3;
  // 384 columns at K >= 768 (C2's stage-3 fc2 and the stage-2 -> 3 downsample): the wide 192 x 384
  // tile (gemm_f32_tnw_kernel) -- each A panel fetched once, 243 tiles = one round at 64 images;
  // s384 fc2 451 -> 424 us (0.776 -> 0.826 of the fp32 peak), C2 +0.9 % (two streams) / +1.7 % (one)
  // in interleaved rounds (profiles/r06/gemm_wide_ab.txt).  Same wave K order: bitwise the 64-row
  // tile's rows.  From 100 tiles, so the two-stream sub-batches (23,328 rows) take it as well.  On
  // N = 1536 / 3072 / 768 (s384 fc1, s768 fc1 / fc2) it loses 2-10 % to the 128-row tile: 4 / 8 / 2
  // column tiles per row band put 3.8 / 7.1 / 1.8 rounds on the CUs (gemm_wide_ab.txt part 4).
  if (PIPNET_AB_GEMM_RULE != 6 && N == 384 && K >= 768 && M >= 192 * 100 && epi != PIPNET_EPI_GELU_BWD &&
      aload != ALOAD_CONV && vec_epi)
    return 5;
  if (N <= 384 || K <= 192 || M <= 64) return 2;
  return 3;
}

// split-K reduction + epilogue: C = epi(sum_s slab_s), float4 per thread.
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int64_t slab,
                                                            int M, int N, const float* __restrict__ bias,
                                                            const float* __restrict__ scale, const float* R,
                                                            int64_t ldr, float* C, int64_t ldc) {
  const int n4 = N / 4;
  const int64_t total = (int64_t)M * n4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / n4), n = 4 * (int)(i - (int64_t)m * n4);
    f32x4 acc = ld4(ws + (int64_t)m * N + n);
    for (int sp = 1; sp < splits; ++sp) acc += ld4(ws + sp * slab + (int64_t)m * N + n);
    const f32x4 bn = bias ? ld4(bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 sn = scale ? ld4(scale + n) : f32x4{1.f, 1.f, 1.f, 1.f};
    const f32x4 r = R ? ld4(R + (int64_t)m * ldr + n) : f32x4{0.f, 0.f, 0.f, 0.f};
    st4(C + (int64_t)m * ldc + n, epi_math<EPI>(acc, bn, sn, r));
  }
}

// split-K reduction of a paired GEMM (N = 2 Nh columns: [A W1^T | A W2^T]) with the pair multiplied:
// C[m][n] = (sum_s slab_s[m][Nh + n]) * (sum_s slab_s[m][n]), n < Nh -- BilinearIntermediate's
// W(e) * V(e) on the folded pair (count_pipnet_utils.py:378-385), the same product as the
// EPI_MUL epilogue of the V GEMM with the W GEMM's output as R.
__global__ __launch_bounds__(256) void splitk_pair_mul_kernel(const float* __restrict__ ws, int splits, int64_t slab,
                                                              int M, int Nh, float* C, int64_t ldc) {
  const int n4 = Nh / 4;
  const int64_t total = (int64_t)M * n4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int m = (int)(i / n4), n = 4 * (int)(i - (int64_t)m * n4);
    const float* r = ws + (int64_t)m * 2 * Nh + n;
    f32x4 a = ld4(r), v = ld4(r + Nh);
    for (int sp = 1; sp < splits; ++sp) {
      a += ld4(r + sp * slab);
      v += ld4(r + sp * slab + Nh);
    }
    st4(C + (int64_t)m * ldc + n, v * a);
  }
}

// compute units of the current device (queried per launch: no process-wide cache, so every
// device of a multi-GPU process gets its own answer; the runtime serves it from its device table)
int num_cus() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      v > 0)
    return v;
  return 256;
}

template <int ALOAD>
int launch_gemm(GemmParams& p, int epi, hipStream_t s) {
  p.nt = (p.N + BN - 1) / BN;
  p.group_m = choose_group_m(p);
  p.vec_epi = (p.N % 4 == 0) && (p.ldc % 4 == 0) && aligned16(p.C) &&
              (!p.R || ((p.ldr % 4 == 0) && aligned16(p.R))) && (!p.bias || aligned16(p.bias)) &&
              (!p.scale || aligned16(p.scale));
  const bool vec = aligned16(p.A) && aligned16(p.W) && (ALOAD != ALOAD_DENSE || (p.lda & 3) == 0);
  const int v = gemm_variant(p.M, p.N, p.K, vec, epi, ALOAD, p.vec_epi);
  if (v == 5) {
    p.nt = p.N / 384;
    p.mt = (p.M + 191) / 192;
  } else {
    p.mt = (p.M + (v == 2 ? 63 : 127)) / (v == 2 ? 64 : 128);
  }
  const dim3 grid(p.mt * p.nt), block(v == 5 ? 768 : NTHREADS);
#define PIPNET_EPI_CASE(E)                                                                                 \
  case E:                                                                                                 \
    if constexpr (ALOAD != ALOAD_CONV && E != PIPNET_EPI_GELU_BWD) {                                      \
      if (v == 5) {                                                                                       \
        hipLaunchKernelGGL((gemm_f32_tnw_kernel<E, ALOAD>), grid, block, 0, s, p);                        \
        break;                                                                                            \
      }                                                                                                   \
    }                                                                                                     \
    if (v == 1) hipLaunchKernelGGL((gemm_f32_tn_kernel<16, 2, E, ALOAD, 2, 3>), grid, block, 0, s, p);    \
    else if (v == 2 && p.N % BN) hipLaunchKernelGGL((gemm_f32_tn_kernel<32, 1, E, ALOAD, 3, 2, 0, true>), grid, \
                                                   block, 0, s, p);                                         \
    else if (v == 2) hipLaunchKernelGGL((gemm_f32_tn_kernel<32, 1, E, ALOAD, 3, 2>), grid, block, 0, s, p); \
    else if (v == 3) hipLaunchKernelGGL((gemm_f32_tn_kernel<32, 2, E, ALOAD, 2, 2>), grid, block, 0, s, p); \
    else hipLaunchKernelGGL((gemm_f32_tn_ktail_kernel<E, ALOAD>), grid, block, 0, s, p);                   \
    break;
  switch (epi) {
    PIPNET_EPI_CASE(PIPNET_EPI_NONE)
    PIPNET_EPI_CASE(PIPNET_EPI_BIAS)
    PIPNET_EPI_CASE(PIPNET_EPI_BIAS_GELU)
    PIPNET_EPI_CASE(PIPNET_EPI_RESID)
    PIPNET_EPI_CASE(PIPNET_EPI_MUL)
    PIPNET_EPI_CASE(PIPNET_EPI_BIAS_RELU)
    PIPNET_EPI_CASE(PIPNET_EPI_BIAS_RESID_RELU)
    PIPNET_EPI_CASE(PIPNET_EPI_RESID_ROWSCALE)
    PIPNET_EPI_CASE(PIPNET_EPI_GELU_BWD)
    default: return PIPNET_ERR_ARG;
  }
#undef PIPNET_EPI_CASE
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

}  // namespace

// The variant pipnet_linear_f32 / _rowscale / pipnet_conv2x2_f32 / pipnet_conv2d_nhwc_f32 launch for an
// M x N x K product with dense, unit-stride, 16-B aligned operands (what torch allocations give).
extern "C" int pipnet_linear_f32_plan(int M, int N, int K, int epilogue, int aload) {
  if (M < 0 || N < 0 || K <= 0 || aload < ALOAD_DENSE || aload > ALOAD_CONV) return -PIPNET_ERR_ARG;
  if (epilogue < PIPNET_EPI_NONE || epilogue > PIPNET_EPI_GELU_BWD) return -PIPNET_ERR_ARG;
  return gemm_variant(M, N, K, true, epilogue, aload, N % 4 == 0);
}

extern "C" int pipnet_linear_f32(const float* A, int64_t lda, const float* W, const float* bias,
                                 const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                                 int M, int N, int K, int epilogue, void* stream) {
  if (M < 0 || N < 0 || K <= 0) return PIPNET_ERR_ARG;
  if (M == 0 || N == 0) return PIPNET_OK;
  if (epilogue < PIPNET_EPI_NONE || epilogue > PIPNET_EPI_GELU_BWD || epilogue == PIPNET_EPI_RESID_ROWSCALE)
    return PIPNET_ERR_ARG;
  if ((K & 3) || (lda & 3) || lda < K || ldc < N) return PIPNET_ERR_ARG;
  if (!A || !W || !C) return PIPNET_ERR_ARG;
  if ((epilogue == PIPNET_EPI_RESID || epilogue == PIPNET_EPI_MUL || epilogue == PIPNET_EPI_BIAS_RESID_RELU ||
       epilogue == PIPNET_EPI_GELU_BWD) &&
      (!R || ldr < N))
    return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(W)) return PIPNET_ERR_ALIGN;
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = W; p.bias = bias; p.scale = scale; p.R = R; p.ldr = ldr;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  return launch_gemm<ALOAD_DENSE>(p, epilogue, (hipStream_t)stream);
}

extern "C" int pipnet_linear_rowscale_f32(const float* A, int64_t lda, const float* W, const float* bias,
                                          const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                                          int M, int N, int K, const float* row_scale, int rows_per_scale,
                                          void* stream) {
  if (M < 0 || N < 0 || K <= 0 || rows_per_scale <= 0) return PIPNET_ERR_ARG;
  if (M == 0 || N == 0) return PIPNET_OK;
  if ((K & 3) || (lda & 3) || lda < K || ldc < N || !R || ldr < N) return PIPNET_ERR_ARG;
  if (!A || !W || !C || !row_scale) return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(W)) return PIPNET_ERR_ALIGN;
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = W; p.bias = bias; p.scale = scale; p.R = R; p.ldr = ldr;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.row_scale = row_scale; p.rows_per_scale = rows_per_scale;
  return launch_gemm<ALOAD_DENSE>(p, PIPNET_EPI_RESID_ROWSCALE, (hipStream_t)stream);
}

extern "C" int pipnet_conv2x2_f32(const float* x, int B, int H, int W, int Cin, const float* w_packed,
                                  const float* bias, int Cout, int stride, float* y, void* stream) {
  if (B < 0 || H < 2 || W < 2 || Cin <= 0 || Cout <= 0) return PIPNET_ERR_ARG;
  if (stride != 1 && stride != 2) return PIPNET_ERR_ARG;
  if (Cin % 32) return PIPNET_ERR_ARG;       // a K tile never straddles (ky, kx)
  if (!x || !w_packed || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  GemmParams p{};
  p.OH = (H - 2) / stride + 1;
  p.OW = (W - 2) / stride + 1;
  p.A = x; p.lda = 0; p.W = w_packed; p.bias = bias; p.C = y; p.ldc = Cout;
  p.M = B * p.OH * p.OW; p.N = Cout; p.K = 4 * Cin;
  p.H = H; p.Wd = W; p.Cin = Cin; p.stride = stride;
  return launch_gemm<ALOAD_CONV2X2>(p, bias ? PIPNET_EPI_BIAS : PIPNET_EPI_NONE, (hipStream_t)stream);
}

extern "C" int pipnet_conv2d_nhwc_f32(const float* x, int B, int H, int W, int Cin, const float* w_packed,
                                      const float* bias, int Cout, int KH, int KW, int stride, int pad,
                                      const float* R, int epilogue, float* y, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || (Cin & 3) || Cout <= 0 || KH <= 0 || KW <= 0 || stride <= 0 ||
      pad < 0)
    return PIPNET_ERR_ARG;
  if (epilogue != PIPNET_EPI_NONE && epilogue != PIPNET_EPI_BIAS && epilogue != PIPNET_EPI_BIAS_RELU &&
      epilogue != PIPNET_EPI_BIAS_RESID_RELU)
    return PIPNET_ERR_ARG;
  if (epilogue == PIPNET_EPI_BIAS_RESID_RELU && !R) return PIPNET_ERR_ARG;
  if (!x || !w_packed || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed)) return PIPNET_ERR_ALIGN;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  if (OH <= 0 || OW <= 0) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  GemmParams p{};
  p.A = x; p.W = w_packed; p.bias = bias; p.R = R; p.ldr = Cout; p.C = y; p.ldc = Cout;
  p.M = B * OH * OW; p.N = Cout; p.K = KH * KW * Cin;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = OH; p.OW = OW; p.stride = stride; p.KW = KW; p.pad = pad;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {      // pointwise: plain GEMM over pixels
    p.lda = Cin;
    return launch_gemm<ALOAD_DENSE>(p, epilogue, (hipStream_t)stream);
  }
  return launch_gemm<ALOAD_CONV>(p, epilogue, (hipStream_t)stream);
}

extern "C" int pipnet_linear_pair_mul_f32(const float* A, int64_t lda, const float* Wpair, float* C, int64_t ldc, int M,
                                          int Nh, int K, int splits, float* workspace, void* stream) {
  if (M < 0 || Nh <= 0 || K <= 0 || (Nh & 3) || (K % 32) || (lda & 3) || lda < K || (ldc & 3) || ldc < Nh)
    return PIPNET_ERR_ARG;
  if (splits < 1 || splits > K / 32 || splits > 64 || !workspace || !A || !Wpair || !C) return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(Wpair) || !aligned16(C) || !aligned16(workspace)) return PIPNET_ERR_ALIGN;
  if (M == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = Wpair; p.C = workspace; p.ldc = 2 * Nh; p.M = M; p.N = 2 * Nh; p.K = K;
  p.nt = (p.N + BN - 1) / BN;
  p.mt = (M + 63) / 64;
  p.group_m = choose_group_m(p);
  p.vec_epi = 1;
  p.split_stride = (int64_t)M * p.N;
  const dim3 grid(p.mt * p.nt, splits);
  hipLaunchKernelGGL((gemm_f32_tn_kernel<32, 1, PIPNET_EPI_NONE, ALOAD_DENSE, 3, 2>), grid, dim3(NTHREADS), 0, s, p);
  PIPNET_CHECK_LAUNCH();
  const int64_t work = (int64_t)M * (Nh / 4);
  const int blocks = (int)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
  hipLaunchKernelGGL(splitk_pair_mul_kernel, dim3(blocks), dim3(256), 0, s, workspace, splits, p.split_stride, M, Nh, C,
                     ldc);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_linear_splitk_f32(const float* A, int64_t lda, const float* W, const float* bias,
                                        const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                                        int M, int N, int K, int epilogue, int splits, float* workspace,
                                        void* stream) {
  if (splits <= 1) return pipnet_linear_f32(A, lda, W, bias, scale, R, ldr, C, ldc, M, N, K, epilogue, stream);
  if (M < 0 || N <= 0 || K <= 0 || (N & 3) || (K % 32) || (lda & 3) || lda < K || (ldc & 3) || ldc < N)
    return PIPNET_ERR_ARG;
  if (splits > K / 32 || splits > 64 || !workspace || !A || !W || !C) return PIPNET_ERR_ARG;
  if (epilogue < PIPNET_EPI_NONE || epilogue > PIPNET_EPI_GELU_BWD || epilogue == PIPNET_EPI_RESID_ROWSCALE)
    return PIPNET_ERR_ARG;
  if ((epilogue == PIPNET_EPI_RESID || epilogue == PIPNET_EPI_MUL || epilogue == PIPNET_EPI_BIAS_RESID_RELU ||
       epilogue == PIPNET_EPI_GELU_BWD) &&
      (!R || ldr < N || (ldr & 3) || !aligned16(R)))
    return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(W) || !aligned16(C) || !aligned16(workspace) || (bias && !aligned16(bias)) ||
      (scale && !aligned16(scale)))
    return PIPNET_ERR_ALIGN;
  if (M == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = W; p.C = workspace; p.ldc = N; p.M = M; p.N = N; p.K = K;
  p.nt = (N + BN - 1) / BN;
  p.mt = (M + 63) / 64;
  p.group_m = choose_group_m(p);
  p.vec_epi = 1;
  p.split_stride = (int64_t)M * N;
  const dim3 grid(p.mt * p.nt, splits);
  hipLaunchKernelGGL((gemm_f32_tn_kernel<32, 1, PIPNET_EPI_NONE, ALOAD_DENSE, 3, 2>), grid, dim3(NTHREADS), 0, s, p);
  PIPNET_CHECK_LAUNCH();
  const int64_t work = (int64_t)M * (N / 4);
  const int blocks = (int)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
#define PIPNET_RED(E)                                                                                           \
  case E:                                                                                                      \
    hipLaunchKernelGGL((splitk_reduce_kernel<E>), dim3(blocks), dim3(256), 0, s, workspace, splits, p.split_stride, \
                       M, N, bias, scale, R, ldr, C, ldc);                                                     \
    break;
  switch (epilogue) {
    PIPNET_RED(PIPNET_EPI_NONE)
    PIPNET_RED(PIPNET_EPI_BIAS)
    PIPNET_RED(PIPNET_EPI_BIAS_GELU)
    PIPNET_RED(PIPNET_EPI_RESID)
    PIPNET_RED(PIPNET_EPI_MUL)
    PIPNET_RED(PIPNET_EPI_BIAS_RELU)
    PIPNET_RED(PIPNET_EPI_BIAS_RESID_RELU)
    PIPNET_RED(PIPNET_EPI_GELU_BWD)
    default: return PIPNET_ERR_ARG;
  }
#undef PIPNET_RED
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
