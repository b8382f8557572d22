// Product instantiation of the fp32 MFMA GEMM (templates + design notes: gemm_f32_impl.hpp).
#include "gemm_f32_impl.hpp"

#include <cstdlib>

#ifndef PIPNET_GEMM_PERSIST_DEFAULT
#define PIPNET_GEMM_PERSIST_DEFAULT 0
#endif

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
// 0 = register-staged K-tail kernel, 1 = BK16x128 rows x3 stages, 2 = BK32x64 rows,
// 3 = BK32x128 rows (mirrored by count_pipnet_amd/kernels.py:gemm_kernel_name)
int gemm_variant(int M, int N, int K, bool vec) {
  if (!vec) return 0;
  if (K % 16 == 0 && K <= 96 && N > 192 && M > 64) return 1;
  if (K % 32) return K % 16 == 0 && M > 64 ? 1 : 0;
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

// ======================================================================================
// Skinny GEMM (M <= 64 rows, e.g. C5's BilinearIntermediate at M = batch): the weights W
// [N][K] are read exactly once, so nothing is gained by staging them through LDS.  Every wave
// streams its own 64 columns of W and the (L1/L2-resident) A rows straight into registers
// with float4 loads and multiplies on v_mfma_f32_32x32x2_f32: with the k-slot permutation of
// gemm_f32_impl.hpp (lane (row|col, h = l >> 5) supplies k = 16 h + j in MFMA j of a 32-deep
// step) a lane's 16 k-values of a row are 64 contiguous bytes of that row, for A and W alike.
// A workgroup = 4 waves on the same 64 columns, each wave one quarter of the workgroup's K
// slab; the quarters are summed through LDS in wave order, and the slab partial goes to the
// split-K workspace, which splitk_reduce_kernel sums in slab order with the epilogue.  No
// barrier in the main loop; loads of step t+1 are in flight under the MFMAs of step t.
// At M = 64 an fp32 weight element feeds 2 x 64 flops: 32 flop / byte, above the fp32-MFMA
// ridge (157 TF/s / 8 TB/s = 20), so the bound is the MFMA pipe, not HBM.
// The per-row result depends on (N, K) only -- the slab split is chosen from them -- never
// on M (rows past M are clamped loads, never stored).
// ======================================================================================
template <int RB>
__global__ __launch_bounds__(256, 2) void skinny_gemm_kernel(const float* __restrict__ A, int64_t lda,
                                                           const float* __restrict__ W, int M, int N, int K,
                                                           int kslab, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) float red[3 * 64 * RB * 2 * 16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 64;
  const int kq = kslab / 4;                                   // per-wave K range (multiple of 32)
  const int kb = blockIdx.y * kslab + wid * kq;
  const int ke = min(kb + kq, K);
  const float* arow[RB];
  const float* wrow[2];
#pragma unroll
  for (int i = 0; i < RB; ++i) arow[i] = A + (int64_t)min(32 * i + r, M - 1) * lda + 16 * h;
#pragma unroll
  for (int j = 0; j < 2; ++j) wrow[j] = W + (int64_t)(n0 + 32 * j + r) * K + 16 * h;
  f32x16 acc[RB][2];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
  // One register set of operands: slice q (k = 16 h + 4 q .. + 3 of the step) is reloaded for
  // the next step right after its 4 x RB x 2 MFMAs, a whole step ahead of its use.  The loads
  // are inline asm with explicit waits: hipcc's own wait counting drains every load at the top
  // of the loop (vmcnt(0)), which would expose the full memory latency once per step.  Issue
  // order per step: [mma q, load q] for q = 0..3, so before mma q exactly 3 slices of loads
  // (3 (2 + RB) instructions) are younger than the ones it needs -- in every step, since the
  // last step re-loads its own operands (unused) to keep the pattern.  The wait names the
  // slice's registers as in/out operands, so no MFMA can be scheduled above it.
  constexpr int LPS = 2 + RB;                                 // loads per slice
  f32x4 a[RB][4], w[2][4];
  auto gload = [](f32x4& d, const float* p) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p) : "memory");
  };
  auto load_q = [&](int q, int k) {
#pragma unroll
    for (int j = 0; j < 2; ++j) gload(w[j][q], wrow[j] + k + 4 * q);
#pragma unroll
    for (int i = 0; i < RB; ++i) gload(a[i][q], arow[i] + k + 4 * q);
  };
  auto wait_q = [&](int q) {
    if constexpr (RB == 2)
      asm volatile("s_waitcnt vmcnt(%4)" : "+v"(w[0][q]), "+v"(w[1][q]), "+v"(a[0][q]), "+v"(a[1][q]) : "n"(3 * LPS));
    else
      asm volatile("s_waitcnt vmcnt(%3)" : "+v"(w[0][q]), "+v"(w[1][q]), "+v"(a[0][q]) : "n"(3 * LPS));
  };
  auto mma_q = [&](int q) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q][e], w[j][q][e], acc[i][j], 0, 0, 0);
  };
  if (kb < ke) {
#pragma unroll
    for (int q = 0; q < 4; ++q) load_q(q, kb);
    for (int k = kb; k < ke; k += 32) {
      const int kn = k + 32 < ke ? k + 32 : k;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        wait_q(q);
        mma_q(q);
        load_q(q, kn);
      }
    }
    // the trailing re-loads must land before their registers are reused
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (RB == 2)
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(w[0][q]), "+v"(w[1][q]), "+v"(a[0][q]), "+v"(a[1][q]));
      else
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(w[0][q]), "+v"(w[1][q]), "+v"(a[0][q]));
    }
  }
  // quarter sums in wave order: waves 1..3 park their accumulators, wave 0 adds them
  constexpr int PER = RB * 2 * 16;
  if (wid > 0) {
    float* dst = red + (wid - 1) * 64 * PER;
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) dst[((i * 2 + j) * 16 + v) * 64 + lane] = acc[i][j][v];
  }
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w) {
    const float* src = red + w * 64 * PER;
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc[i][j][v] += src[((i * 2 + j) * 16 + v) * 64 + lane];
  }
  float* out = ws + (int64_t)blockIdx.y * M * N;
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = 32 * i + (v & 3) + 8 * (v >> 2) + 4 * h;
        if (m < M) out[(int64_t)m * N + n0 + 32 * j + r] = acc[i][j][v];
      }
}

// compute units of the current device, queried once
int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n = v;
    else
      n = 256;
  }
  return n;
}

// PIPNET_GEMM_PERSIST=0/1 (read once): the persistent 128x128 tile for variant-3 dense GEMMs
// with N % 128 == 0 (A/B switch; the default is set from tools/gemm_bench.py runs).
int g_gemm_persist = -1;
bool gemm_persist() {
  if (g_gemm_persist < 0) {
    const char* e = getenv("PIPNET_GEMM_PERSIST");
    g_gemm_persist = e ? (e[0] == '1') : PIPNET_GEMM_PERSIST_DEFAULT;
  }
  return g_gemm_persist == 1;
}

// PIPNET_GEMM_STREAM=0/1 (read once; default 0 -- measured 3-5 % slower than the regular tile, profiles/r03/gemm_stream_ab.txt): the streaming persistent tile with deferred
// epilogues (gemm_f32_tn_stream_kernel) for variant-3 dense GEMMs with N % 128 == 0, K >= 256
// and at least two tiles per workgroup slot.
#ifndef PIPNET_GEMM_STREAM_DEFAULT
#define PIPNET_GEMM_STREAM_DEFAULT 0
#endif
int g_gemm_stream = -1;
bool gemm_stream() {
  if (g_gemm_stream < 0) {
    const char* e = getenv("PIPNET_GEMM_STREAM");
    g_gemm_stream = e ? (e[0] == '1') : PIPNET_GEMM_STREAM_DEFAULT;
  }
  return g_gemm_stream == 1;
}

template <int ALOAD>
int launch_gemm(GemmParams& p, int epi, hipStream_t s) {
  p.nt = (p.N + BN - 1) / BN;
  p.group_m = choose_group_m(p);
  p.vec_epi = (p.N % 4 == 0) && (p.ldc % 4 == 0) && aligned16(p.C) &&
              (!p.R || ((p.ldr % 4 == 0) && aligned16(p.R))) && (!p.bias || aligned16(p.bias)) &&
              (!p.scale || aligned16(p.scale));
  const bool vec = aligned16(p.A) && aligned16(p.W) && (ALOAD != ALOAD_DENSE || (p.lda & 3) == 0);
  const int v = gemm_variant(p.M, p.N, p.K, vec);
  p.mt = (p.M + (v == 2 ? 63 : 127)) / (v == 2 ? 64 : 128);
  const dim3 grid(p.mt * p.nt), block(NTHREADS);
  if (ALOAD == ALOAD_DENSE && v == 3 && p.vec_epi && p.N % BN == 0 && p.K % 32 == 0 && p.K >= 256 &&
      epi != PIPNET_EPI_RESID_ROWSCALE && p.mt * p.nt >= 4 * num_cus() && (int64_t)p.M * p.lda < (1LL << 31) &&
      (int64_t)p.N * p.K < (1LL << 31) && (int64_t)p.M * p.ldc < (1LL << 31) &&
      (!p.R || (int64_t)p.M * p.ldr < (1LL << 31)) && gemm_stream()) {
    const dim3 sgrid(2 * num_cus());
#define PIPNET_STREAM_CASE(E) \
  case E: hipLaunchKernelGGL((gemm_f32_tn_stream_kernel<E>), sgrid, block, 0, s, p); break;
    switch (epi) {
      PIPNET_STREAM_CASE(PIPNET_EPI_NONE)
      PIPNET_STREAM_CASE(PIPNET_EPI_BIAS)
      PIPNET_STREAM_CASE(PIPNET_EPI_BIAS_GELU)
      PIPNET_STREAM_CASE(PIPNET_EPI_RESID)
      PIPNET_STREAM_CASE(PIPNET_EPI_MUL)
      PIPNET_STREAM_CASE(PIPNET_EPI_BIAS_RELU)
      PIPNET_STREAM_CASE(PIPNET_EPI_BIAS_RESID_RELU)
      PIPNET_STREAM_CASE(PIPNET_EPI_GELU_BWD)
      default: return PIPNET_ERR_ARG;
    }
#undef PIPNET_STREAM_CASE
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
  if (ALOAD == ALOAD_DENSE && v == 3 && p.vec_epi && p.N % BN == 0 && gemm_persist()) {
    const int ntiles = p.mt * p.nt;
    const dim3 pgrid(ntiles < 2 * num_cus() ? ntiles : 2 * num_cus());
#define PIPNET_PERSIST_CASE(E) \
  case E: hipLaunchKernelGGL((gemm_f32_tn_persist_kernel<E>), pgrid, block, 0, s, p); break;
    switch (epi) {
      PIPNET_PERSIST_CASE(PIPNET_EPI_NONE)
      PIPNET_PERSIST_CASE(PIPNET_EPI_BIAS)
      PIPNET_PERSIST_CASE(PIPNET_EPI_BIAS_GELU)
      PIPNET_PERSIST_CASE(PIPNET_EPI_RESID)
      PIPNET_PERSIST_CASE(PIPNET_EPI_MUL)
      PIPNET_PERSIST_CASE(PIPNET_EPI_BIAS_RELU)
      PIPNET_PERSIST_CASE(PIPNET_EPI_BIAS_RESID_RELU)
      PIPNET_PERSIST_CASE(PIPNET_EPI_RESID_ROWSCALE)
      PIPNET_PERSIST_CASE(PIPNET_EPI_GELU_BWD)
      default: return PIPNET_ERR_ARG;
    }
#undef PIPNET_PERSIST_CASE
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
#define PIPNET_EPI_CASE(E)                                                                                 \
  case E:                                                                                                 \
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

extern "C" int pipnet_gemm_persist(int mode) {
  if (mode == 0 || mode == 1) g_gemm_persist = mode;
  else if (mode != -1) return PIPNET_ERR_ARG;
  return gemm_persist() ? 1 : 0;
}

extern "C" int pipnet_gemm_stream(int mode) {
  if (mode == 0 || mode == 1) g_gemm_stream = mode;
  else if (mode != -1) return PIPNET_ERR_ARG;
  return gemm_stream() ? 1 : 0;
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

// K slab per workgroup of the skinny GEMM (4 waves x a multiple of 32), from (N, K) only:
// about 2 workgroups per CU (each wave >= 2 K-steps).
static int skinny_kslab(int N, int K) {
  const int nb = N / 64;
  int slabs = (2 * num_cus() + nb - 1) / nb;
  int kslab = (K + slabs - 1) / slabs;
  kslab = (kslab + 127) / 128 * 128;
  return kslab < 256 ? 256 : kslab;
}

extern "C" int pipnet_skinny_splits(int N, int K) {
  if (N <= 0 || K <= 0) return PIPNET_ERR_ARG;
  const int ks = skinny_kslab(N, K);
  return (K + ks - 1) / ks;
}

extern "C" int pipnet_linear_skinny_f32(const float* A, int64_t lda, const float* W, const float* bias,
                                        const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                                        int M, int N, int K, int epilogue, float* workspace, void* stream) {
  if (M < 0 || M > 64 || N <= 0 || K <= 0 || (N % 64) || (K % 32) || (lda & 3) || lda < K || (ldc & 3) || ldc < N)
    return PIPNET_ERR_ARG;
  if (!workspace || !A || !W || !C) return PIPNET_ERR_ARG;
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
  const int kslab = skinny_kslab(N, K);
  const int splits = (K + kslab - 1) / kslab;
  const dim3 grid(N / 64, splits);
  if (M > 32) hipLaunchKernelGGL((skinny_gemm_kernel<2>), grid, dim3(256), 0, s, A, lda, W, M, N, K, kslab, workspace);
  else hipLaunchKernelGGL((skinny_gemm_kernel<1>), grid, dim3(256), 0, s, A, lda, W, M, N, K, kslab, workspace);
  PIPNET_CHECK_LAUNCH();
  const int64_t work = (int64_t)M * (N / 4);
  const int blocks = (int)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
  const int64_t slab = (int64_t)M * N;
#define PIPNET_RED(E)                                                                                      \
  case E:                                                                                                 \
    hipLaunchKernelGGL((splitk_reduce_kernel<E>), dim3(blocks), dim3(256), 0, s, workspace, splits, slab, M, N, \
                       bias, scale, R, ldr, C, ldc);                                                      \
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
