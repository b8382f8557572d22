// fp32 GEMM on gfx950 matrix cores: C = epi(A * W^T), exact fp32 (v_mfma_f32_32x32x2_f32).
//
// The ConvNeXt-tiny forward is 93 % Linear FLOPs: CNBlock Linear d->4d
// (+GELU) and 4d->d (*layer_scale + residual), the k2 downsample convs (implicit GEMM over
// an NHWC gather) and the 1x1 prototype add-on.  All of them are "TN" products whose two
// operands are K-contiguous in HBM (NHWC activations [M][K], torch Linear weights [N][K]),
// so one kernel serves them all; the A-tile loader is the only thing that differs.
//
// Tile: 128x128x32 per 256-thread workgroup, 4 waves in 2x2, each wave 64x64 = 2x2 MFMA
// 32x32 tiles (64 accumulator VGPRs).  For v_mfma_f32_32x32x2_f32 lane l supplies
// A[l&31][k] and B[k][l&31] with k = l>>5 of the 2-deep step; the k order inside a
// 32-deep LDS tile is free (both operands use the same map), so half-wave h walks
// k = 16h .. 16h+15 and reads its 16 operands with four conflict-free ds_read_b128
// (row stride 36 floats = 144 B: rows r*36 mod 64 dwords are distinct 16-B slots).
// Global -> registers -> LDS staging with 2 LDS buffers and one barrier per K-tile;
// the next tile's global loads are issued before the current tile's 64 MFMAs.
#include "common.hpp"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, LDK = BK + 4, NTHREADS = 256;
constexpr int GROUP_M = 8;

struct GemmParams {
  const float* A;
  int64_t lda;
  const float* W;
  const float* bias;
  const float* scale;
  const float* R;
  int64_t ldr;
  float* C;
  int64_t ldc;
  int M, N, K;
  // implicit conv2x2 A-loader
  int H, Wd, Cin, OH, OW, stride;
  int mt, nt;
};

enum { ALOAD_DENSE = 0, ALOAD_CONV2X2 = 1 };

template <int ALOAD>
PIPNET_DEV int64_t a_row_base(const GemmParams& p, int m) {
  if (ALOAD == ALOAD_DENSE) return (int64_t)m * p.lda;
  const int ohw = p.OH * p.OW;
  const int b = m / ohw;
  const int r = m - b * ohw;
  const int oy = r / p.OW;
  const int ox = r - oy * p.OW;
  return (((int64_t)b * p.H + oy * p.stride) * p.Wd + ox * p.stride) * p.Cin;
}

template <int ALOAD>
PIPNET_DEV int64_t a_col_off(const GemmParams& p, int k) {
  if (ALOAD == ALOAD_DENSE) return k;
  const int idx = k / p.Cin;                 // (ky, kx) = (idx >> 1, idx & 1)
  const int c = k - idx * p.Cin;
  return ((int64_t)(idx >> 1) * p.Wd + (idx & 1)) * p.Cin + c;
}

template <int EPI, int ALOAD>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_f32_tn_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDK];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;

  // ---- tile selection: XCD-contiguous ranges, GROUP_M-grouped raster for L2 reuse ----
  const int nwg = p.mt * p.nt;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int group = tile / (GROUP_M * p.nt);
  const int first_m = group * GROUP_M;
  const int gsz = min(p.mt - first_m, GROUP_M);
  const int in_group = tile - group * GROUP_M * p.nt;
  const int tm = first_m + in_group % gsz;
  const int tn = in_group / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread global staging coordinates: 4 rows of A, 4 rows of W, one float4 each ----
  const int srow = tid >> 3;          // 0..31
  const int sk = (tid & 7) * 4;       // 0..28
  int64_t abase[4];
  bool aval[4];
  const float* wrow[4];
  bool wval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + srow + 32 * i;
    aval[i] = m < p.M;
    abase[i] = a_row_base<ALOAD>(p, aval[i] ? m : 0);
    const int n = n0 + srow + 32 * i;
    wval[i] = n < p.N;
    wrow[i] = p.W + (int64_t)(wval[i] ? n : 0) * p.K;
  }

  f32x4 ra[4], rb[4];
  auto gload = [&](int kt) {
    const int k = kt * BK + sk;
    const bool kin = k < p.K;
    const int64_t aoff = a_col_off<ALOAD>(p, kin ? k : 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = (aval[i] && kin) ? ld4(p.A + abase[i] + aoff) : f32x4{0.f, 0.f, 0.f, 0.f};
      rb[i] = (wval[i] && kin) ? ld4(wrow[i] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * (BM + BN) * LDK;
    float* Bs = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st4(As + (srow + 32 * i) * LDK + sk, ra[i]);
      st4(Bs + (srow + 32 * i) * LDK + sk, rb[i]);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  const int nk = (p.K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);

    const float* As = smem + buf * (BM + BN) * LDK;
    const float* Bs = As + BM * LDK;
    f32x4 fa[2][4], fb[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float* pa = As + (wm * 64 + i * 32 + lr) * LDK + lh * 16;
      const float* pb = Bs + (wn * 64 + i * 32 + lr) * LDK + lh * 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        fa[i][q] = ld4(pa + 4 * q);
        fb[i][q] = ld4(pb + 4 * q);
      }
    }
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][kk >> 2][kk & 3], fb[j][kk >> 2][kk & 3],
                                                           acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane owns column n = ...+lr, rows (v&3) + 8(v>>2) + 4h of each 32x32 tile ----
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + lr;
    if (n >= p.N) continue;
    float bn = 0.f, sn = 1.f;
    if (EPI == PIPNET_EPI_BIAS || EPI == PIPNET_EPI_BIAS_GELU || EPI == PIPNET_EPI_RESID)
      bn = p.bias ? p.bias[n] : 0.f;
    if (EPI == PIPNET_EPI_RESID) sn = p.scale ? p.scale[n] : 1.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + wm * 64 + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * lh;
        if (m >= p.M) continue;
        float x = acc[i][j][v];
        if (EPI == PIPNET_EPI_BIAS) x = x + bn;
        if (EPI == PIPNET_EPI_BIAS_GELU) x = gelu_erf(x + bn);
        if (EPI == PIPNET_EPI_RESID) x = p.R[(int64_t)m * p.ldr + n] + sn * (x + bn);
        if (EPI == PIPNET_EPI_MUL) x = x * p.R[(int64_t)m * p.ldr + n];
        p.C[(int64_t)m * p.ldc + n] = x;
      }
    }
  }
}

template <int ALOAD>
int launch_gemm(GemmParams& p, int epi, hipStream_t s) {
  p.mt = (p.M + BM - 1) / BM;
  p.nt = (p.N + BN - 1) / BN;
  const dim3 grid(p.mt * p.nt), block(NTHREADS);
  switch (epi) {
    case PIPNET_EPI_NONE: hipLaunchKernelGGL((gemm_f32_tn_kernel<PIPNET_EPI_NONE, ALOAD>), grid, block, 0, s, p); break;
    case PIPNET_EPI_BIAS: hipLaunchKernelGGL((gemm_f32_tn_kernel<PIPNET_EPI_BIAS, ALOAD>), grid, block, 0, s, p); break;
    case PIPNET_EPI_BIAS_GELU: hipLaunchKernelGGL((gemm_f32_tn_kernel<PIPNET_EPI_BIAS_GELU, ALOAD>), grid, block, 0, s, p); break;
    case PIPNET_EPI_RESID: hipLaunchKernelGGL((gemm_f32_tn_kernel<PIPNET_EPI_RESID, ALOAD>), grid, block, 0, s, p); break;
    case PIPNET_EPI_MUL: hipLaunchKernelGGL((gemm_f32_tn_kernel<PIPNET_EPI_MUL, ALOAD>), grid, block, 0, s, p); break;
    default: return PIPNET_ERR_ARG;
  }
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
  if (Cin % BK) return PIPNET_ERR_ARG;       // a 32-deep K tile never straddles (ky, kx)
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
