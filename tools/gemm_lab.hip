// Tuning lab for the fp32 MFMA GEMM (not part of the product ABI): every variant of
// count_pipnet_amd/csrc/gemm_f32_impl.hpp behind one entry point, for A/B timing in one process.
#include "../count_pipnet_amd/csrc/gemm_f32_impl.hpp"

using namespace pipnet_gemm;

template <int BK, int MINB>
static void launch(GemmParams& p, int epi, hipStream_t s) {
  const dim3 grid(p.mt * p.nt), block(NTHREADS);
  if (epi == PIPNET_EPI_BIAS_GELU)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, PIPNET_EPI_BIAS_GELU, ALOAD_DENSE, MINB>), grid, block, 0, s, p);
  else if (epi == PIPNET_EPI_RESID)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, PIPNET_EPI_RESID, ALOAD_DENSE, MINB>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, PIPNET_EPI_NONE, ALOAD_DENSE, MINB>), grid, block, 0, s, p);
}

extern "C" int lab_linear(int variant, int group_m, const float* A, int64_t lda, const float* W, const float* bias,
                          const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc, int M, int N, int K,
                          int epi, void* stream) {
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = W; p.bias = bias; p.scale = scale; p.R = R; p.ldr = ldr;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.mt = (M + BM - 1) / BM;
  p.nt = (N + BN - 1) / BN;
  p.group_m = group_m;
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: launch<32, 2>(p, epi, s); break;
    case 1: launch<16, 4>(p, epi, s); break;
    case 2: launch<16, 2>(p, epi, s); break;
    case 3: launch<32, 1>(p, epi, s); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
