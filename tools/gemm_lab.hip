// Tuning lab for the fp32 MFMA GEMM (not part of the product ABI): variants of
// count_pipnet_amd/csrc/gemm_f32_impl.hpp behind one entry point, for A/B timing in one process.
#include "gemm_variants_lab.hpp"

using namespace pipnet_gemm;

template <int BK, int TM, int MINB, int NS, int ABL = 0, int SH = 0>
static void launch(GemmParams& p, int epi, hipStream_t s) {
  if constexpr (SH == 1) {
    p.mt = (p.M + 64 * TM - 1) / (64 * TM);
    const dim3 grid(p.mt * p.nt), block(NTHREADS);
    if (epi == PIPNET_EPI_BIAS_GELU)
      hipLaunchKernelGGL((gemm_f32_tn16_kernel<BK, TM, PIPNET_EPI_BIAS_GELU, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
    else if (epi == PIPNET_EPI_BIAS)
      hipLaunchKernelGGL((gemm_f32_tn16_kernel<BK, TM, PIPNET_EPI_BIAS, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
    else if (epi == PIPNET_EPI_RESID)
      hipLaunchKernelGGL((gemm_f32_tn16_kernel<BK, TM, PIPNET_EPI_RESID, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
    else
      hipLaunchKernelGGL((gemm_f32_tn16_kernel<BK, TM, PIPNET_EPI_NONE, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
    return;
  }
  p.mt = (p.M + 64 * TM - 1) / (64 * TM);
  const dim3 grid(p.mt * p.nt), block(NTHREADS);
  if (epi == PIPNET_EPI_BIAS_GELU)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, PIPNET_EPI_BIAS_GELU, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else if (epi == EPI_LAB_GELU_PK)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, EPI_LAB_GELU_PK, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else if (epi == EPI_LAB_GELU_PK16)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, EPI_LAB_GELU_PK16, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else if (epi == EPI_LAB_GELU_SC16)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, EPI_LAB_GELU_SC16, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else if (epi == EPI_LAB_GELU_FAST)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, EPI_LAB_GELU_FAST, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else if (epi == PIPNET_EPI_BIAS)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, PIPNET_EPI_BIAS, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else if (epi == PIPNET_EPI_RESID)
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, PIPNET_EPI_RESID, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_tn_kernel<BK, TM, PIPNET_EPI_NONE, ALOAD_DENSE, MINB, NS, ABL>), grid, block, 0, s, p);
}

// round 6: the 8-wave workgroup (WGM = 4): (128 TM) x 128 tiles, one workgroup per CU
template <int BK, int TM, int MINB, int NS, int ABL = 0, int SH = 0>
static void launch8(GemmParams& p, int epi, hipStream_t s) {
  p.mt = (p.M + 128 * TM - 1) / (128 * TM);
  const dim3 grid(p.mt * p.nt), block(512);
  if (epi == PIPNET_EPI_BIAS_GELU)
    hipLaunchKernelGGL((gemm_f32_tn8_kernel<BK, TM, PIPNET_EPI_BIAS_GELU, ALOAD_DENSE, MINB, NS, ABL, SH>), grid, block, 0, s, p);
  else if (epi == PIPNET_EPI_BIAS)
    hipLaunchKernelGGL((gemm_f32_tn8_kernel<BK, TM, PIPNET_EPI_BIAS, ALOAD_DENSE, MINB, NS, ABL, SH>), grid, block, 0, s, p);
  else if (epi == PIPNET_EPI_RESID)
    hipLaunchKernelGGL((gemm_f32_tn8_kernel<BK, TM, PIPNET_EPI_RESID, ALOAD_DENSE, MINB, NS, ABL, SH>), grid, block, 0, s, p);
  else
    hipLaunchKernelGGL((gemm_f32_tn8_kernel<BK, TM, PIPNET_EPI_NONE, ALOAD_DENSE, MINB, NS, ABL, SH>), grid, block, 0, s, p);
}

static long long* g_stamps = nullptr;
extern "C" void lab_set_stamps(long long* p) { g_stamps = p; }

extern "C" int lab_linear(int variant, int group_m, const float* A, int64_t lda, const float* W, const float* bias,
                          const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc, int M, int N, int K,
                          int epi, void* stream) {
  GemmParams p{};
  p.A = A; p.lda = lda; p.W = W; p.bias = bias; p.scale = scale; p.R = R; p.ldr = ldr;
  p.C = C; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.nt = (N + BN - 1) / BN;
  p.group_m = group_m;
  const bool scalar_epi = variant >= 20 && variant < 30;   // 2x: variant x with the scalar epilogue
  p.vec_epi = scalar_epi ? 0 : 1;
  if (scalar_epi) variant -= 20;
  // group_m >= 100: stagger experiment, group_m = 100*s + g
  p.stagger = group_m / 100;
  p.group_m = group_m % 100;
  p.stagger_lo = 256;
  p.stagger_hi = 512;
  p.stamps = g_stamps;
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: launch<32, 2, 2, 2>(p, epi, s); break;
    case 1: launch<32, 1, 2, 2>(p, epi, s); break;
    case 2: launch<32, 1, 3, 2>(p, epi, s); break;
    case 3: launch<16, 2, 2, 3>(p, epi, s); break;
    case 4: launch<16, 1, 4, 3>(p, epi, s); break;
    case 5: launch<32, 1, 4, 2>(p, epi, s); break;
    case 6: launch<16, 1, 3, 4>(p, epi, s); break;
    case 7: launch<16, 2, 3, 3>(p, epi, s); break;    // 48 KiB LDS, <=168 VGPRs: 3 workgroups / CU
    case 8: launch<16, 2, 3, 2>(p, epi, s); break;    // 32 KiB LDS, 3 workgroups / CU
    // round 6: 8-wave workgroups -- 60/61: 256 x 128 tiles with 3 / 2 LDS stages; 62/63: 128 x 128 with 4 / 3
    case 60: launch8<32, 2, 1, 3>(p, epi, s); break;
    case 61: launch8<32, 2, 1, 2>(p, epi, s); break;
    case 62: launch8<32, 1, 1, 4>(p, epi, s); break;
    case 63: launch8<32, 1, 1, 3>(p, epi, s); break;
    case 64: launch8<32, 2, 1, 3, 0, 1>(p, epi, s); break;      // 60 on v_mfma_f32_16x16x4_f32
    // ablations of variant 0 (timing only; outputs are wrong)
    case 10: launch<32, 2, 2, 2, 1>(p, epi, s); break;
    case 11: launch<32, 2, 2, 2, 2>(p, epi, s); break;
    case 13: launch<32, 2, 2, 2, 7>(p, epi, s); break;
    // stamped (ABL 8) copies of variants 0 / 2 / 3: per-workgroup phase timing
    case 30: launch<32, 2, 2, 2, 8>(p, epi, s); break;
    case 32: launch<32, 1, 3, 2, 8>(p, epi, s); break;
    case 33: launch<16, 2, 2, 3, 8>(p, epi, s); break;
    // v_mfma_f32_16x16x4_f32 forms of variants 0 / 2 / 1, and a stamped copy of 40
    case 40: launch<32, 2, 2, 2, 0, 1>(p, epi, s); break;
    case 42: launch<32, 1, 3, 2, 0, 1>(p, epi, s); break;
    case 41: launch<32, 1, 2, 2, 0, 1>(p, epi, s); break;
    case 70: launch<32, 2, 2, 2, 8, 1>(p, epi, s); break;
    case 37: launch<16, 2, 3, 3, 8>(p, epi, s); break;    // v7 with stamps
    // persistent (50) and streaming persistent (51) 128x128 tiles, 2 workgroups per CU (N % 128 == 0)
    case 50:
    case 51: {
      int cus = 256, dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      p.mt = (p.M + 127) / 128;
      const int nt = p.mt * p.nt;
      const dim3 grid(nt < 2 * cus ? nt : 2 * cus), block(NTHREADS);
      if (variant == 50 && epi == PIPNET_EPI_BIAS_GELU) hipLaunchKernelGGL((gemm_f32_tn_persist_kernel<PIPNET_EPI_BIAS_GELU>), grid, block, 0, s, p);
      else if (variant == 50) hipLaunchKernelGGL((gemm_f32_tn_persist_kernel<PIPNET_EPI_RESID>), grid, block, 0, s, p);
      else if (epi == PIPNET_EPI_BIAS_GELU) hipLaunchKernelGGL((gemm_f32_tn_stream_kernel<PIPNET_EPI_BIAS_GELU>), grid, block, 0, s, p);
      else hipLaunchKernelGGL((gemm_f32_tn_stream_kernel<PIPNET_EPI_RESID>), grid, block, 0, s, p);
      break;
    }
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
