// bf16 ResNet path (BASELINE C3): implicit-GEMM convolution (gemm_bf16_impl.hpp), NCHW fp32
// -> NHWC bf16 input relayout, NHWC bf16 max-pool.  Reference: features/resnet_features.py
// (conv / BatchNorm / ReLU / Bottleneck / MaxPool2d, :77-229).
#include "gemm_bf16_impl.hpp"

using namespace pipnet_bf16;

namespace {

int grid_for(int64_t n) { return (int)((n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192); }

// compute units of the current device (one persistent workgroup each), queried per launch
int num_cus() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
      v > 0)
    return v;
  return 256;
}

// Raster group (tile_coords): group_m M-tiles are walked before N advances; budget in bytes of
// 128-row A panels (build-time knob for tools/ab_build.py experiments)
#ifndef PIPNET_BF16_GROUP_BUDGET
#define PIPNET_BF16_GROUP_BUDGET (2.0 * 1024 * 1024)
#endif
int choose_group_m(int K) {
  const double panel = 128.0 * K * 2.0;
  int g = (int)(PIPNET_BF16_GROUP_BUDGET / panel);
  return g < 1 ? 1 : (g > 16 ? 16 : g);
}

using CfgS = Cfg<2, 2, 1, 2, 32, 4>;  //  64 x 128, BK 32 x 4 stages, 48 KiB LDS, 3 workgroups / CU
using CfgM = Cfg<2, 2, 2, 2>;          // 128 x 128, 256 threads, 64 KiB LDS, 2 workgroups / CU
using CfgL = Cfg<2, 4, 4, 2>;          // 256 x 256, 512 threads, 128 KiB LDS, 1 workgroup / CU
using CfgL4 = Cfg<2, 4, 4, 2, 32, 4>;  // 256 x 256, BK 32 x 4 stages (3 tiles in flight), 128 KiB
using CfgM4 = Cfg<2, 2, 2, 2, 32, 4>;  // 128 x 128, BK 32 x 4 stages, 64 KiB, 2 workgroups / CU
using CfgN64 = Cfg<4, 1, 2, 2, 32, 4>; // 256 x 64 (N = 64 layers), BK 32 x 4 stages, 80 KiB, 2 workgroups / CU

// Tile choice: the largest tile that still gives every CU at least one workgroup (larger
// tiles halve the L2 -> LDS bytes per MFMA: 128x128 needs ~64 B/clk/CU at the MFMA rate,
// the L2's whole bandwidth; 256x256 needs 32), with 32-deep K tiles in 4 stages (+1..+30 %
// over 64-deep x 2 on the ResNet50 shapes, profiles/r01/conv_bf16_tiles.log).  Every tile the
// automatic choice can pick walks K in the same 32-deep steps, so the MFMA accumulation order
// -- and therefore every bf16 rounding -- of a pixel does not depend on the batch it is in.
// Mirrored by kernels.py:bf16_conv_tile.
// N >= 256 layers run the ping-pong 16x16x32 kernel (tile 5) at every batch size -- the
// choice depends on the layer only, never on M, so per-pixel results stay batch-invariant.
int conv_variant(int M, int N, bool pp_ok, bool s3 = false, int Kv = 0) {
  if (s3) {  // split GEMMs (tools/s3_tiles.py, profiles/r01/s3_tiles.txt); tiles 0 / 4 / 5 / 7 only
    const int m128 = ((M + 127) / 128) * ((N + 127) / 128) >= 512 ? 4 : 0;
    if (!pp_ok) return m128;
    if (N == 192) return 7;                          // one 192-wide tile instead of a 256-wide one
    if (N == 384) return Kv >= 3 * 1024 ? 7 : m128;  // stage-3 Linear2: 192-wide; short K: 128x128
    return N >= 256 ? 5 : m128;
  }
  const int64_t tm = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  // K <= 64 (layer1 conv3: 64 -> 256 + identity): one K-tile pair per tile, all epilogue -- the
  // 2-workgroup 128 x 128 tile overlaps one workgroup's epilogue with the other's MFMAs
  // (41 vs 47 us per half batch, profiles/r03/conv_bf16_b64.log).  A per-layer rule (K, N).
  if (N >= 256 && pp_ok && Kv > 64) return 5;
  if (N <= 64 && !s3) return 6;   // 256 x 64: a 128-wide tile would compute half padding columns
  const int64_t tl = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
  if (N >= 256 && tl >= 256 && Kv > 64) return 3;
  // 128 x 128 once the grid covers each CU once (layer2 conv2 at 64 images: 392 tiles, 31-34 vs
  // 42-44 us on 64 x 128); tiles 0 / 3 / 4 walk K identically, so this M-dependent choice keeps
  // every pixel's result bitwise batch-invariant
  if (tm >= 256) return 4;
  return 0;
}

bool is_s3_epi(int epi) {
  return epi == PIPNET_EPI_S3_GELU || epi == PIPNET_EPI_F32_BIAS || epi == PIPNET_EPI_F32_RESID;
}

// 3x3 / stride 1 / pad 1 convs with N >= 256 whose halo fits the kernel's 320 LDS rows
// (256 + 2W + 2): the LDS-halo ping-pong kernel (tile 8) replaces tile 5 -- a per-layer
// choice, never M.
// 3x3 / stride 1 / pad 1 convs with Cin = N = 64 (layer1 conv2, W <= 63) or Cin = N = 128
// (layer2 conv2, W <= 31): the small-N LDS-halo tile (11) -- a per-layer choice, never M.
bool halo64_ok(const ConvParams& p, int epi) {
  const bool shape = (p.Cin == 64 && p.N == 64 && p.Wd <= hsm::Shape<64>::MAX_W) ||
                     (p.Cin == 128 && p.N == 128 && p.Wd <= hsm::Shape<128>::MAX_W);
  return p.KW == 3 && p.Kv == 9 * p.Cin && p.stride == 1 && p.pad == 1 && p.OH == p.H && p.OW == p.Wd &&
         p.seg == 0 && shape && !is_s3_epi(epi);
}

bool halo_ok(const ConvParams& p, int epi) {
  return p.KW == 3 && p.Kv == 9 * p.Cin && p.stride == 1 && p.pad == 1 && p.OH == p.H && p.OW == p.Wd &&
         p.seg == 0 && p.Cin % 64 == 0 && p.Wd <= 31 && p.N >= 256 && !is_s3_epi(epi) &&
         (int64_t)p.M * p.Cin < ((int64_t)1 << 31);        // 32-bit halo source offsets
}
// B fragments of 16 columns per wave.  Only the 256-wide tile is dispatched: the 64 / 128-wide
// instantiations (4 / 8 MFMAs per phase) measured slower than tile 6 on layer1 conv2 (125 vs
// 88 us) and +5 % on layer2 conv2 (profiles/r02/conv_bf16_halo_narrow.log).
// the N = 64 halo tile (11), bitwise tile 6: layer1 conv2 52 -> 28 us at 64 images, 88 -> 46 us at 128
// (profiles/r03/conv_bf16_n64.log)
#ifndef H64_AUTO
#define H64_AUTO 1
#endif
int halo_nb(int N) { return N >= 256 ? 4 : (N >= 128 ? 2 : 1); }

// Row blocks per wave group of the 256-wide ping-pong tiles (halo 8, persistent 9): 8 -> 256-row
// tiles.  (224-row tiles, RB = 7, gave the single-stream C3 +2 % on the layers whose 256-row grid
// leaves a short last round, but lost under the two-stream default, which already fills those
// rounds: 6.00 vs 6.11 ms, profiles/r04/ab_c3_rb224.txt; the template keeps RB for the lab.)
constexpr int PP_RB = 8;

// The tile a launch takes (requested tile v >= 0 validated, v < 0 = the automatic choice), or -1
// when the requested tile cannot run this conv.  The ONE tile rule: launch_conv dispatches on it
// and pipnet_conv2d_nhwc_bf16_plan exports it, so profiling labels never mirror it in Python.
template <int ALOAD>
int plan_conv(const ConvParams& p, int epi, int v) {
  const bool pp_ok = (ALOAD == ALOAD_DENSE || p.Cin % 32 == 0) && p.K % 32 == 0;
  const bool hk = ALOAD == ALOAD_CONV && halo_ok(p, epi);
  const bool h64 = ALOAD == ALOAD_CONV && halo64_ok(p, epi);
  // 1x1 convs with N % 256 == 0: the persistent ping-pong tile (9), same K order as tile 5
  const bool pk = ALOAD == ALOAD_DENSE && pp_ok && p.N % 256 == 0 && !is_s3_epi(epi);
  if (v < 0) {
    v = conv_variant(p.M, p.N, pp_ok, is_s3_epi(epi), p.Kv > 0 ? p.Kv : p.K);
    if (hk) v = 8;
    else if (h64 && H64_AUTO) v = 11;
    else if (v == 5 && pk) v = 9;
  }
  if (v > 11 || v == 10 || (v == 11 && !h64) || ((v == 5 || v == 7) && !pp_ok) || (v == 8 && !hk) || (v == 9 && !pk)) return -1;
  return v;
}

template <int ALOAD>
int launch_conv(ConvParams& p, int epi, int v, hipStream_t s) {
  v = plan_conv<ALOAD>(p, epi, v);
  if (v < 0) return PIPNET_ERR_ARG;
  if (v == 11) {                                 // Cin = N = 64 / 128 3x3 on the LDS input halo
    const int bm = p.N == 64 ? hsm::Shape<64>::BM : hsm::Shape<128>::BM;
    p.nt = 1;
    p.mt = (p.M + bm - 1) / bm;
    const dim3 grid(p.mt);
#define PIPNET_HSM(CIN)                                                                                  \
    switch (epi) {                                                                                       \
      case PIPNET_EPI_NONE: hipLaunchKernelGGL((conv3x3_bf16_hsmall_kernel<CIN, PIPNET_EPI_NONE>), grid, dim3(256), 0, s, p); break; \
      case PIPNET_EPI_BIAS: hipLaunchKernelGGL((conv3x3_bf16_hsmall_kernel<CIN, PIPNET_EPI_BIAS>), grid, dim3(256), 0, s, p); break; \
      case PIPNET_EPI_BIAS_RELU:                                                                         \
        hipLaunchKernelGGL((conv3x3_bf16_hsmall_kernel<CIN, PIPNET_EPI_BIAS_RELU>), grid, dim3(256), 0, s, p); \
        break;                                                                                           \
      case PIPNET_EPI_BIAS_RESID_RELU:                                                                   \
        hipLaunchKernelGGL((conv3x3_bf16_hsmall_kernel<CIN, PIPNET_EPI_BIAS_RESID_RELU>), grid, dim3(256), 0, s, p); \
        break;                                                                                           \
      default: return PIPNET_ERR_ARG;                                                                    \
    }
    if (p.N == 64) {
      PIPNET_HSM(64)
    } else {
      PIPNET_HSM(128)
    }
#undef PIPNET_HSM
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
  if (v == 9) {                                  // persistent 256 x 256 ping-pong (1x1, N % 256 == 0)
    p.nt = p.N / 256;
    p.mt = (p.M + 32 * PP_RB - 1) / (32 * PP_RB);
    p.group_m = choose_group_m(p.K);
    const int ntiles = p.mt * p.nt;
    const dim3 grid(ntiles < num_cus() ? ntiles : num_cus());
#define PIPNET_PPP(E)                                                                                  \
  case E:                                                                                               \
    hipLaunchKernelGGL((conv_bf16_ppp_kernel<E, PP_RB>), grid, dim3(512), 0, s, p);                   \
    break;
    switch (epi) {
      PIPNET_PPP(PIPNET_EPI_NONE)
      PIPNET_PPP(PIPNET_EPI_BIAS)
      PIPNET_PPP(PIPNET_EPI_BIAS_RELU)
      PIPNET_PPP(PIPNET_EPI_BIAS_RESID_RELU)
      PIPNET_PPP(PIPNET_EPI_DUAL_BIAS_RELU)
      default: return PIPNET_ERR_ARG;
    }
#undef PIPNET_PPP
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
  if (epi == PIPNET_EPI_DUAL_BIAS_RELU) return PIPNET_ERR_ARG;   // persistent 1x1 tile only
  if (v == 8) {                                  // ping-pong with the LDS input halo, 256 x 64 NB
    const int nb = halo_nb(p.N);
    p.nt = (p.N + 64 * nb - 1) / (64 * nb);
    p.mt = (p.M + 32 * PP_RB - 1) / (32 * PP_RB);
    p.group_m = choose_group_m(p.K);
    const dim3 grid(p.mt * p.nt);
#define PIPNET_HALO(E)                                                                                \
  case E:                                                                                              \
    if (nb == 4) hipLaunchKernelGGL((conv3x3_bf16_halo_kernel<E, 4, PP_RB>), grid, dim3(512), 0, s, p); \
    else return PIPNET_ERR_ARG;                                                                        \
    break;
    switch (epi) {
      PIPNET_HALO(PIPNET_EPI_NONE)
      PIPNET_HALO(PIPNET_EPI_BIAS)
      PIPNET_HALO(PIPNET_EPI_BIAS_RELU)
      PIPNET_HALO(PIPNET_EPI_BIAS_RESID_RELU)
      default: return PIPNET_ERR_ARG;
    }
#undef PIPNET_HALO
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
  if (v == 7) {                                  // 256 x 192 ping-pong (split epilogues only)
    p.nt = (p.N + 191) / 192;
    p.mt = (p.M + 255) / 256;
    p.group_m = choose_group_m(p.K);
    const dim3 grid(p.mt * p.nt);
    switch (epi) {
      case PIPNET_EPI_S3_GELU:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_S3_GELU, ALOAD, 3>), grid, dim3(512), 0, s, p);
        break;
      case PIPNET_EPI_F32_BIAS:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_F32_BIAS, ALOAD, 3>), grid, dim3(512), 0, s, p);
        break;
      case PIPNET_EPI_F32_RESID:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_F32_RESID, ALOAD, 3>), grid, dim3(512), 0, s, p);
        break;
      default: return PIPNET_ERR_ARG;
    }
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
  if (v == 5) {
    p.nt = (p.N + 255) / 256;
    p.mt = (p.M + 255) / 256;
    p.group_m = choose_group_m(p.K);
    const dim3 grid(p.mt * p.nt);
    switch (epi) {
      case PIPNET_EPI_NONE: hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_NONE, ALOAD>), grid, dim3(512), 0, s, p); break;
      case PIPNET_EPI_BIAS: hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_BIAS, ALOAD>), grid, dim3(512), 0, s, p); break;
      case PIPNET_EPI_BIAS_RELU:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_BIAS_RELU, ALOAD>), grid, dim3(512), 0, s, p);
        break;
      case PIPNET_EPI_BIAS_RESID_RELU:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_BIAS_RESID_RELU, ALOAD>), grid, dim3(512), 0, s, p);
        break;
      case PIPNET_EPI_S3_GELU:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_S3_GELU, ALOAD>), grid, dim3(512), 0, s, p);
        break;
      case PIPNET_EPI_F32_BIAS:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_F32_BIAS, ALOAD>), grid, dim3(512), 0, s, p);
        break;
      case PIPNET_EPI_F32_RESID:
        hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_F32_RESID, ALOAD>), grid, dim3(512), 0, s, p);
        break;
      default: return PIPNET_ERR_ARG;
    }
    PIPNET_CHECK_LAUNCH();
    return PIPNET_OK;
  }
  const int bm = (v == 2 || v == 3 || v == 6) ? 256 : (v == 0 ? 64 : 128),
            bn = (v == 2 || v == 3) ? 256 : (v == 6 ? 64 : 128);
  p.nt = (p.N + bn - 1) / bn;
  p.mt = (p.M + bm - 1) / bm;
  p.group_m = choose_group_m(p.K);
  const dim3 grid(p.mt * p.nt);
#define PIPNET_BF_CASE(E)                                                                            \
  case E:                                                                                           \
    if (v == 2) hipLaunchKernelGGL((conv_bf16_kernel<CfgL, E, ALOAD, 1>), grid, dim3(512), 0, s, p);  \
    else if (v == 3) hipLaunchKernelGGL((conv_bf16_kernel<CfgL4, E, ALOAD, 1>), grid, dim3(512), 0, s, p); \
    else if (v == 4) hipLaunchKernelGGL((conv_bf16_kernel<CfgM4, E, ALOAD, 2>), grid, dim3(256), 0, s, p); \
    else if (v == 6) hipLaunchKernelGGL((conv_bf16_kernel<CfgN64, E, ALOAD, 2>), grid, dim3(256), 0, s, p); \
    else if (v == 1) hipLaunchKernelGGL((conv_bf16_kernel<CfgM, E, ALOAD, 2>), grid, dim3(256), 0, s, p); \
    else hipLaunchKernelGGL((conv_bf16_kernel<CfgS, E, ALOAD, 3>), grid, dim3(256), 0, s, p);        \
    break;
  // split-bf16 epilogues: only the tiles the automatic choice picks for N < 256 (0 and 4)
#define PIPNET_S3_CASE(E)                                                                            \
  case E:                                                                                           \
    if (v == 4 && p.N % 128) hipLaunchKernelGGL((conv_bf16_kernel<CfgM4, E, ALOAD, 2, true>), grid, dim3(256), 0, s, p); \
    else if (v == 4) hipLaunchKernelGGL((conv_bf16_kernel<CfgM4, E, ALOAD, 2>), grid, dim3(256), 0, s, p); \
    else if (v == 0) hipLaunchKernelGGL((conv_bf16_kernel<CfgS, E, ALOAD, 3>), grid, dim3(256), 0, s, p); \
    else return PIPNET_ERR_ARG;                                                                     \
    break;
  switch (epi) {
    PIPNET_S3_CASE(PIPNET_EPI_S3_GELU)
    PIPNET_S3_CASE(PIPNET_EPI_F32_BIAS)
    PIPNET_S3_CASE(PIPNET_EPI_F32_RESID)
    PIPNET_BF_CASE(PIPNET_EPI_NONE)
    PIPNET_BF_CASE(PIPNET_EPI_BIAS)
    PIPNET_BF_CASE(PIPNET_EPI_BIAS_RELU)
    PIPNET_BF_CASE(PIPNET_EPI_BIAS_RESID_RELU)
    default: return PIPNET_ERR_ARG;
  }
#undef PIPNET_BF_CASE
#undef PIPNET_S3_CASE
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// [B,C,H,W] fp32 -> [B,H,W,Cpad] bf16 (RNE, channels >= C zero); Cpad % 8 == 0, one
// thread per pixel writes one or more 16-B chunks.
__global__ __launch_bounds__(256) void nchw_to_nhwc_bf16_kernel(const float* __restrict__ x, int B, int C, int H,
                                                                int W, int Cpad, bf16* __restrict__ y) {
  const int64_t hw = (int64_t)H * W;
  const int64_t n = (int64_t)B * hw;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / hw;
    const int64_t pix = i - b * hw;
    for (int c0 = 0; c0 < Cpad; c0 += 8) {
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)(c0 + e < C ? x[(b * C + c0 + e) * hw + pix] : 0.f);
      *reinterpret_cast<bf16x8*>(y + i * Cpad + c0) = o;
    }
  }
}

// The ResNet stem (Conv2d 3 -> 64, k7 s2 p3) as a 4x4 / stride-1 / pad-0 conv over a 2x2
// space-to-depth image: S[b][i][j][q], q = (2 bi + bj) * 4 + c, holds x[b][c][2(i-2)+bi][2(j-2)+bj]
// (zero outside the image and in the c = 3 slots), SH = OH + 3, SW = OW + 3.  With the weights
// re-laid as W'[o][a][a'][q] = w[o][c][2a+bi-1][2a'+bj-1] (zero where the tap index is -1) the
// conv has K = 4*4*16 = 256 instead of 7*7*8 = 392 -> 448 padded: 1.75x fewer MFMAs and A-operand
// bytes for the same outputs (every product of the 7x7 conv appears once; the extra ones are
// exact zeros).  One thread per S pixel: 12 reads, two 16-B stores.
__global__ __launch_bounds__(256) void nchw_to_s2d_bf16_kernel(const float* __restrict__ x, int B, int H, int W,
                                                               int SH, int SW, bf16* __restrict__ y) {
  const int64_t n = (int64_t)B * SH * SW;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / ((int64_t)SH * SW);
    const int rem = (int)(i - b * SH * SW);
    const int si = rem / SW, sj = rem - (rem / SW) * SW;
    bf16x8 o[2];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int bi = q >> 3, bj = (q >> 2) & 1, c = q & 3;
      const int r = 2 * (si - 2) + bi, cc = 2 * (sj - 2) + bj;
      float v = 0.f;
      if (c < 3 && (unsigned)r < (unsigned)H && (unsigned)cc < (unsigned)W) v = x[((b * 3 + c) * H + r) * W + cc];
      o[q >> 3][q & 7] = (bf16)v;
    }
    *reinterpret_cast<bf16x8*>(y + i * 16) = o[0];
    *reinterpret_cast<bf16x8*>(y + i * 16 + 8) = o[1];
  }
}

// MaxPool2d on NHWC bf16, 8 channels (16 B) per thread; max is exact in bf16 and padding
// never wins (torch pads max-pool with -inf).
__global__ __launch_bounds__(256) void maxpool_nhwc_bf16_kernel(const bf16* __restrict__ x, int B, int H, int W,
                                                                int C, int k, int stride, int pad, int OH, int OW,
                                                                bf16* __restrict__ y) {
  const int QC = C / 8;
  const int64_t n = (int64_t)B * OH * OW * QC;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int q = (int)(i % QC);
    const int64_t pix = i / QC;
    const int ox = (int)(pix % OW);
    const int oy = (int)((pix / OW) % OH);
    const int64_t b = pix / ((int64_t)OW * OH);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * stride - pad + ky;
      if (iy < 0 || iy >= H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * stride - pad + kx;
        if (ix < 0 || ix >= W) continue;
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + (((b * H + iy) * W + ix) * C) + 8 * q);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], (float)v[e]);
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)m[e];   // exact: every m[e] is a bf16 value
    *reinterpret_cast<bf16x8*>(y + pix * C + 8 * q) = o;
  }
}

// Shape part of a bf16 conv's ConvParams (no pointers) -- shared by the launch and the plan query.
// Returns PIPNET_OK or PIPNET_ERR_ARG; `dense` = the 1x1 stride-1 pad-0 plain-GEMM form.
int conv_bf16_shape(ConvParams& p, bool& dense, int B, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                    int pad, int epilogue) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || (Cin & 7) || Cout <= 0 || (Cout & 7) || KH <= 0 || KW <= 0 ||
      stride <= 0 || pad < 0)
    return PIPNET_ERR_ARG;
  if (epilogue != PIPNET_EPI_NONE && epilogue != PIPNET_EPI_BIAS && epilogue != PIPNET_EPI_BIAS_RELU &&
      epilogue != PIPNET_EPI_BIAS_RESID_RELU)
    return PIPNET_ERR_ARG;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  if (OH <= 0 || OW <= 0) return PIPNET_ERR_ARG;
  if ((int64_t)B * OH * OW >= (int64_t)1 << 31) return PIPNET_ERR_ARG;
  p.ldr = Cout;
  p.ldc = Cout;
  p.M = B * OH * OW; p.N = Cout;
  p.Kv = KH * KW * Cin;
  p.K = (p.Kv + KPAD - 1) / KPAD * KPAD;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = OH; p.OW = OW; p.stride = stride; p.KW = KW; p.pad = pad;
  p.Cinp = Cin;
  p.seg = 0;
  dense = KH == 1 && KW == 1 && stride == 1 && pad == 0;     // pointwise: plain GEMM over pixels
  if (dense) p.lda = Cin;
  return PIPNET_OK;
}

}  // namespace

extern "C" int pipnet_conv2d_nhwc_bf16_tile(const void* x, int B, int H, int W, int Cin, const void* w_packed,
                                            const float* bias, int Cout, int KH, int KW, int stride, int pad,
                                            const void* R, int epilogue, void* y, int tile, void* stream) {
  ConvParams p{};
  bool dense = false;
  if (const int st = conv_bf16_shape(p, dense, B, H, W, Cin, Cout, KH, KW, stride, pad, epilogue)) return st;
  if (epilogue == PIPNET_EPI_BIAS_RESID_RELU && !R) return PIPNET_ERR_ARG;
  if (!x || !w_packed || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(y) || (R && !aligned16(R)) || (bias && !aligned16(bias)))
    return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  p.A = reinterpret_cast<const bf16*>(x);
  p.W = reinterpret_cast<const bf16*>(w_packed);
  p.bias = bias;
  p.R = reinterpret_cast<const bf16*>(R);
  p.C = reinterpret_cast<bf16*>(y);
  return dense ? launch_conv<ALOAD_DENSE>(p, epilogue, tile, (hipStream_t)stream)
               : launch_conv<ALOAD_CONV>(p, epilogue, tile, (hipStream_t)stream);
}

extern "C" int pipnet_conv2d_nhwc_bf16_plan(int B, int H, int W, int Cin, int Cout, int KH, int KW, int stride,
                                            int pad, int epilogue, int tile) {
  ConvParams p{};
  bool dense = false;
  if (conv_bf16_shape(p, dense, B, H, W, Cin, Cout, KH, KW, stride, pad, epilogue)) return -PIPNET_ERR_ARG;
  const int v = dense ? plan_conv<ALOAD_DENSE>(p, epilogue, tile) : plan_conv<ALOAD_CONV>(p, epilogue, tile);
  return v < 0 ? -PIPNET_ERR_ARG : v;
}

extern "C" int pipnet_conv2d_nhwc_bf16(const void* x, int B, int H, int W, int Cin, const void* w_packed,
                                       const float* bias, int Cout, int KH, int KW, int stride, int pad,
                                       const void* R, int epilogue, void* y, void* stream) {
  return pipnet_conv2d_nhwc_bf16_tile(x, B, H, W, Cin, w_packed, bias, Cout, KH, KW, stride, pad, R, epilogue, y, -1,
                                      stream);
}

extern "C" int pipnet_conv1x1_bf16_dual(const void* x, int64_t M, int Cin, const void* w_packed, const float* bias,
                                        int N1, void* y1, int N2, void* y2, void* stream) {
  if (M < 0 || M >= ((int64_t)1 << 31) || Cin <= 0 || (Cin & 7) || N1 <= 0 || N2 <= 0 || (N1 % 256) || (N2 % 256) ||
      !x || !w_packed || !y1 || !y2)
    return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(y1) || !aligned16(y2) || (bias && !aligned16(bias)))
    return PIPNET_ERR_ALIGN;
  if (M == 0) return PIPNET_OK;
  ConvParams p{};
  p.A = reinterpret_cast<const bf16*>(x);
  p.lda = Cin;
  p.W = reinterpret_cast<const bf16*>(w_packed);
  p.bias = bias;
  p.C = reinterpret_cast<bf16*>(y1);
  p.ldc = N1;
  p.C2 = reinterpret_cast<bf16*>(y2);
  p.ldc2 = N2;
  p.nsplit = N1;
  p.M = (int)M; p.N = N1 + N2;
  p.Kv = Cin;
  p.K = (Cin + KPAD - 1) / KPAD * KPAD;
  p.H = (int)M; p.Wd = 1; p.Cin = Cin; p.OH = (int)M; p.OW = 1; p.stride = 1; p.KW = 1; p.pad = 0;
  p.Cinp = Cin;
  return launch_conv<ALOAD_DENSE>(p, PIPNET_EPI_DUAL_BIAS_RELU, 9, (hipStream_t)stream);
}

extern "C" int pipnet_nchw_to_nhwc_bf16(const float* x, int B, int C, int H, int W, int Cpad, void* y,
                                        void* stream) {
  if (B < 0 || C <= 0 || H <= 0 || W <= 0 || Cpad < C || (Cpad & 7) || !x || !y) return PIPNET_ERR_ARG;
  if (!aligned16(y)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  hipLaunchKernelGGL(nchw_to_nhwc_bf16_kernel, dim3(grid_for((int64_t)B * H * W)), dim3(256), 0,
                     (hipStream_t)stream, x, B, C, H, W, Cpad, reinterpret_cast<bf16*>(y));
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_nchw_to_s2d_bf16(const float* x, int B, int H, int W, void* y, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || !x || !y) return PIPNET_ERR_ARG;
  if (!aligned16(y)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int SH = (H - 1) / 2 + 4, SW = (W - 1) / 2 + 4;
  hipLaunchKernelGGL(nchw_to_s2d_bf16_kernel, dim3(grid_for((int64_t)B * SH * SW)), dim3(256), 0, (hipStream_t)stream,
                     x, B, H, W, SH, SW, reinterpret_cast<bf16*>(y));
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// ResNet stem (4x4 stride-1 conv over the s2d image, 16 -> 64, + bias + ReLU) fused with
// MaxPool2d(3, 2, 1): s2d [B][SH][SW][16] bf16 (pipnet_nchw_to_s2d_bf16), w packed [64][256]
// (pipnet_pack_conv_weight_bf16 of the regrouped 4x4x16 stem weight), y [B][PH][PW][64] bf16
// with PH = (SH - 4) / 2 + 1.  Bitwise the unfused conv (tile 6) + pipnet_maxpool2d_nhwc_bf16.
extern "C" int pipnet_stem_pool_bf16(const void* s2d, int B, int SH, int SW, const void* w, const float* bias,
                                     void* y, void* stream) {
  if (B < 0 || SH < 4 || SW < 4 || SW - 3 > spool::MAX_OW || !s2d || !w || !bias || !y) return PIPNET_ERR_ARG;
  if (!aligned16(s2d) || !aligned16(w) || !aligned16(y)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int PH = (SH - 3 - 1) / 2 + 1, PW = (SW - 3 - 1) / 2 + 1;
  const int npr = (PH + spool::PR - 1) / spool::PR;
  hipLaunchKernelGGL(stem_pool_bf16_kernel, dim3((unsigned)(B * npr)), dim3(spool::NT), 0, (hipStream_t)stream,
                     reinterpret_cast<const bf16*>(s2d), SH, SW, reinterpret_cast<const bf16*>(w), bias,
                     reinterpret_cast<bf16*>(y), PH, PW);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_maxpool2d_nhwc_bf16(const void* x, int B, int H, int W, int C, int k, int stride, int pad,
                                          void* y, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || C <= 0 || (C & 7) || k <= 0 || stride <= 0 || pad < 0 || 2 * pad > k)
    return PIPNET_ERR_ARG;
  if (!x || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(y)) return PIPNET_ERR_ALIGN;
  const int OH = (H + 2 * pad - k) / stride + 1, OW = (W + 2 * pad - k) / stride + 1;
  if (OH <= 0 || OW <= 0) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  hipLaunchKernelGGL(maxpool_nhwc_bf16_kernel, dim3(grid_for((int64_t)B * OH * OW * (C / 8))), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const bf16*>(x), B, H, W, C, k, stride, pad, OH, OW,
                     reinterpret_cast<bf16*>(y));
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// Split-bf16 ("bf16x3") conv / linear of the ConvNeXt backbone (include/pipnet_amd.h): x holds
// split planes [hi | lo] (2 Cin channels per pixel), read as the virtual 3 Cin channels
// [hi | lo | hi] of each tap (seg_remap), against weights [hi | hi | lo] per tap.
extern "C" int pipnet_conv2d_nhwc_s3(const void* x, int B, int H, int W, int Cin, const void* w_packed,
                                     const float* bias, const float* scale, const float* R, int Cout, int KH, int KW,
                                     int stride, int pad, int epilogue, void* y, int tile, void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || Cin <= 0 || (Cin % 32) || Cout <= 0 || (Cout & 7) || KH <= 0 || KW <= 0 ||
      stride <= 0 || pad < 0)
    return PIPNET_ERR_ARG;
  if (!is_s3_epi(epilogue)) return PIPNET_ERR_ARG;
  if (epilogue == PIPNET_EPI_F32_RESID && (!R || !scale)) return PIPNET_ERR_ARG;
  if (tile != -1 && tile != 0 && tile != 4 && tile != 5 && tile != 7) return PIPNET_ERR_ARG;
  if (!x || !w_packed || !y) return PIPNET_ERR_ARG;
  if (!aligned16(x) || !aligned16(w_packed) || !aligned16(y) || (R && !aligned16(R)) || (bias && !aligned16(bias)) ||
      (scale && !aligned16(scale)))
    return PIPNET_ERR_ALIGN;
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  if (OH <= 0 || OW <= 0) return PIPNET_ERR_ARG;
  if ((int64_t)B * OH * OW >= (int64_t)1 << 31) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  ConvParams p{};
  p.A = reinterpret_cast<const bf16*>(x);
  p.W = reinterpret_cast<const bf16*>(w_packed);
  p.bias = bias;
  p.scale = scale;
  p.R32 = R;
  p.ldr = Cout;
  if (epilogue == PIPNET_EPI_S3_GELU) {
    p.C = reinterpret_cast<bf16*>(y);
    p.ldc = 2 * (int64_t)Cout;
  } else {
    p.Cf = reinterpret_cast<float*>(y);
    p.ldc = Cout;
  }
  p.M = B * OH * OW; p.N = Cout;
  p.Kv = KH * KW * 3 * Cin;
  p.K = (p.Kv + 31) / 32 * 32;                 // the split tiles (0, 4, 5) all walk K in 32-deep steps
  p.H = H; p.Wd = W; p.Cin = 3 * Cin; p.OH = OH; p.OW = OW; p.stride = stride; p.KW = KW; p.pad = pad;
  p.Cinp = 2 * Cin;
  p.seg = Cin;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) {
    p.lda = 2 * Cin;
    return launch_conv<ALOAD_DENSE>(p, epilogue, tile, (hipStream_t)stream);
  }
  return launch_conv<ALOAD_CONV>(p, epilogue, tile, (hipStream_t)stream);
}
