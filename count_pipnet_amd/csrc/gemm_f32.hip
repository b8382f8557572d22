// Product instantiation of the fp32 MFMA GEMM (templates + design notes: gemm_f32_impl.hpp).
#include "gemm_f32_impl.hpp"

using namespace pipnet_gemm;

namespace {

// Raster: consecutive tile ids walk group_m M-tiles before advancing N, sized so the A
// panels of one group (group_m x 128 rows x K) stay within ~2 MiB of an XCD's 4 MiB L2.
int choose_group_m(const GemmParams& p) {
  const double panel = 128.0 * p.K * 4.0;
  int g = (int)(2.0 * 1024 * 1024 / panel);
  return g < 1 ? 1 : (g > 16 ? 16 : g);
}

// K-tile depth (measured with tools/gemm_lab.py on the network's shapes, MI355X):
// BK=16 (32 KiB LDS, 4 workgroups/CU) wins +5..+28 % on short reductions (K <= 384) and
// on narrow outputs (N <= 192); BK=32 (64 KiB, 2 workgroups/CU) wins +2..+7 % on the
// long K=768..3072 reductions of stages 3-4.
template <int ALOAD>
int launch_gemm(GemmParams& p, int epi, hipStream_t s) {
  p.mt = (p.M + BM - 1) / BM;
  p.nt = (p.N + BN - 1) / BN;
  p.group_m = choose_group_m(p);
  const dim3 grid(p.mt * p.nt), block(NTHREADS);
  const bool vec = aligned16(p.A) && aligned16(p.W) && (ALOAD == ALOAD_CONV2X2 || (p.lda & 3) == 0);
  const bool bk32 = vec && (p.K % 32) == 0 && p.K > 384 && p.N > 192;
  const bool bk16 = vec && !bk32 && (p.K % 16) == 0;
#define PIPNET_EPI_CASE(E)                                                                          \
  case E:                                                                                          \
    if (bk32) hipLaunchKernelGGL((gemm_f32_tn_kernel<32, E, ALOAD, 2>), grid, block, 0, s, p);      \
    else if (bk16) hipLaunchKernelGGL((gemm_f32_tn_kernel<16, E, ALOAD, 4>), grid, block, 0, s, p); \
    else hipLaunchKernelGGL((gemm_f32_tn_ktail_kernel<E, ALOAD>), grid, block, 0, s, p);            \
    break;
  switch (epi) {
    PIPNET_EPI_CASE(PIPNET_EPI_NONE)
    PIPNET_EPI_CASE(PIPNET_EPI_BIAS)
    PIPNET_EPI_CASE(PIPNET_EPI_BIAS_GELU)
    PIPNET_EPI_CASE(PIPNET_EPI_RESID)
    PIPNET_EPI_CASE(PIPNET_EPI_MUL)
    default: return PIPNET_ERR_ARG;
  }
#undef PIPNET_EPI_CASE
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

}  // namespace

extern "C" int pipnet_linear_f32(const float* A, int64_t lda, const float* W, const float* bias,
                                 const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                                 int M, int N, int K, int epilogue, void* stream) {
  if (M < 0 || N < 0 || K <= 0) return PIPNET_ERR_ARG;
  if (M == 0 || N == 0) return PIPNET_OK;
  if (epilogue < PIPNET_EPI_NONE || epilogue > PIPNET_EPI_MUL) return PIPNET_ERR_ARG;
  if ((K & 3) || (lda & 3) || lda < K || ldc < N) return PIPNET_ERR_ARG;
  if (!A || !W || !C) return PIPNET_ERR_ARG;
  if ((epilogue == PIPNET_EPI_RESID || epilogue == PIPNET_EPI_MUL) && (!R || ldr < N)) return PIPNET_ERR_ARG;
  if (!aligned16(A) || !aligned16(W)) return PIPNET_ERR_ALIGN;
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = W; p.bias = bias; p.scale = scale; p.R = R; p.ldr = ldr;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  return launch_gemm<ALOAD_DENSE>(p, epilogue, (hipStream_t)stream);
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
