// fp32 GEMM on gfx950 matrix cores: C = epi(A * W^T), exact fp32 (v_mfma_f32_32x32x2_f32).
// Kernel templates shared by the product library (gemm_f32.hip) and the tuning lab
// (tools/gemm_lab.hip).
//
// The ConvNeXt-tiny forward is 93 % Linear FLOPs: CNBlock Linear d->4d
// (+GELU) and 4d->d (*layer_scale + residual), the k2 downsample convs (implicit GEMM over
// an NHWC gather) and the 1x1 prototype add-on.  All of them are "TN" products whose two
// operands are K-contiguous in HBM (NHWC activations [M][K], torch Linear weights [N][K]),
// so one kernel serves them all; the A-tile loader is the only thing that differs.
//
// Tile: (64*TM)x128xBK per 256-thread workgroup, 4 waves in 2x2, each wave (32*TM)x64 =
// TMx2 MFMA 32x32 tiles.  For v_mfma_f32_32x32x2_f32 lane l supplies A[l&31][k] and
// B[k][l&31] with k = l>>5 of the 2-deep step; the k order inside a BK-deep LDS tile is
// free (both operands use the same map), so half-wave h walks k = h*BK/2 .. (h+1)*BK/2-1
// and reads its operands 4 k-steps at a time (ds_read_b128).  TM=1 (64-row tiles) halves
// the tail of grids that are only ~2-3 workgroups deep per CU.
//
// Main path (K % BK == 0): global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave instruction), NS LDS stages, one barrier per K-tile.  LDS rows are BK*4 bytes with
// the 16-B chunk index XOR-swizzled by a row-dependent mask: the DMA writes lane-linear,
// so the swizzle is applied to each lane's SOURCE address and undone on the read
// (cdna_hip_programming.md rule 21); every ds_read_b128 lane group then hits 16 distinct
// 16-B bank slots.  Operand fragments are software-pipelined in two named register sets,
// and the first fragment group of tile k+1 is read right after the barrier, under the last
// MFMA group of tile k.
// General path (any K % 4): register staging with zero-fill of the K tail.
#pragma once
#include <type_traits>

#include "common.hpp"

namespace pipnet_gemm {

constexpr int BN = 128, NTHREADS = 256, NWAVES = 4;

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
  // implicit-GEMM convolution A-loaders (NHWC input [B][H][Wd][Cin])
  int H, Wd, Cin, OH, OW, stride, KW, pad;
  int mt, nt, group_m;
  int vec_epi;     // 1: float4 epilogue through LDS (N, ldc, ldr % 4 == 0, C / R 16-B aligned)
  int stagger;     // lab: workgroups [stagger_lo, stagger_hi) sleep stagger x s_sleep(127) first
  int stagger_lo, stagger_hi;
  int64_t split_stride;   // split-K (gridDim.y > 1): slab y of C starts at C + y * split_stride
  long long* stamps;      // lab (ABL & 8): per-workgroup s_memtime stamps + hardware ids
  const float* row_scale; // PIPNET_EPI_RESID_ROWSCALE: per row-group factor (stochastic depth)
  int rows_per_scale;
};

// Lab instrumentation (ABL & 8, tools/gemm_stamps.py): thread 0 of each workgroup records 16
// int64: start, first K-tile landed, main loop done, epilogue done (s_memtime), HW_ID,
// XCC_ID, s_memrealtime at start and end; 8.. = epilogue sub-phases (vector epilogue: per
// 32-row slab, accumulators re-laid through LDS / its stores issued).
template <int ABL>
PIPNET_DEV void lab_stamp(const GemmParams& p, int slot) {
  if constexpr ((ABL & 8) != 0) {
    if (threadIdx.x == 0) {
      long long* s = p.stamps + ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 16;
      s[slot] = (long long)__builtin_amdgcn_s_memtime();
      if (slot == 0) {
        s[4] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
        s[5] = (long long)__builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
        s[6] = (long long)__builtin_amdgcn_s_memrealtime();
      }
      if (slot == 3) s[7] = (long long)__builtin_amdgcn_s_memrealtime();
    }
  }
}

enum { ALOAD_DENSE = 0, ALOAD_CONV2X2 = 1, ALOAD_CONV = 2 };

// 16 zero bytes: the LDS-DMA / float4 source for implicit-GEMM taps that fall in the
// zero padding of a convolution (the DMA cannot zero-fill, but its source is per lane).
static __device__ const __attribute__((aligned(16))) float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};

// One A row (= one output pixel of a convolution, or one matrix row).
struct ARow {
  int64_t base;    // dense: m*lda; conv: offset of image b (and, for conv2x2, of the pixel)
  int iy0, ix0;    // generic conv: top-left input coordinate of the receptive field
};

template <int ALOAD>
PIPNET_DEV ARow a_row(const GemmParams& p, int m) {
  ARow r{0, 0, 0};
  if (ALOAD == ALOAD_DENSE) {
    r.base = (int64_t)m * p.lda;
    return r;
  }
  const int ohw = p.OH * p.OW;
  const int b = m / ohw;
  const int rr = m - b * ohw;
  const int oy = rr / p.OW;
  const int ox = rr - oy * p.OW;
  if (ALOAD == ALOAD_CONV2X2) {
    r.base = (((int64_t)b * p.H + oy * p.stride) * p.Wd + ox * p.stride) * p.Cin;
  } else {
    r.base = (int64_t)b * p.H * p.Wd * p.Cin;
    r.iy0 = oy * p.stride - p.pad;
    r.ix0 = ox * p.stride - p.pad;
  }
  return r;
}

// Address of A[m][k .. k+3] (k % 4 == 0, the 4 channels of one tap), or of g_zero4.
template <int ALOAD>
PIPNET_DEV const float* a_ptr(const GemmParams& p, const ARow& r, int k) {
  if (ALOAD == ALOAD_DENSE) return p.A + r.base + k;
  const int tap = k / p.Cin;
  const int c = k - tap * p.Cin;
  if (ALOAD == ALOAD_CONV2X2)          // (ky, kx) = (tap >> 1, tap & 1), never out of bounds
    return p.A + r.base + ((int64_t)(tap >> 1) * p.Wd + (tap & 1)) * p.Cin + c;
  const int ky = tap / p.KW;
  const int iy = r.iy0 + ky;
  const int ix = r.ix0 + tap - ky * p.KW;
  if ((unsigned)iy >= (unsigned)p.H || (unsigned)ix >= (unsigned)p.Wd) return g_zero4;
  return p.A + r.base + ((int64_t)iy * p.Wd + ix) * p.Cin + c;
}

// exact-enough GELU: x * Phi(x), Phi from erfc(|x|/sqrt2) by the Chebyshev fit of
// Numerical Recipes (erfcc, fractional error < 1.2e-7 everywhere).  Max |error| vs the
// erf-GELU of torch: 1.4e-8 absolute, 1.2e-7 relative for |x| < 6 (~18 VALU ops instead
// of ~58 for ocml erff; the GELU epilogue is VALU work the MFMA pipe cannot hide).
PIPNET_DEV float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float q = fmaf(t, 0.17087277f, -0.82215223f);
  q = fmaf(t, q, 1.48851587f);
  q = fmaf(t, q, -1.13520398f);
  q = fmaf(t, q, 0.27886807f);
  q = fmaf(t, q, -0.18628806f);
  q = fmaf(t, q, 0.09678418f);
  q = fmaf(t, q, 0.37409196f);
  q = fmaf(t, q, 1.00002368f);
  q = fmaf(t, q, -1.26551223f);
  const float half_erfc = 0.5f * t * __expf(fmaf(-z, z, q));
  return x * (x < 0.f ? half_erfc : 1.0f - half_erfc);
}

// d gelu_erf(x) / dx = Phi(x) + x phi(x)  (training backward, EPI_GELU_BWD)
PIPNET_DEV float gelu_grad(float x) {
  const float cdf = 0.5f * erfcf(-x * 0.70710678118654752440f);
  const float pdf = 0.39894228040143267794f * expf(-0.5f * x * x);
  return fmaf(x, pdf, cdf);
}

// GELU by Abramowitz & Stegun 7.1.26 (|erf error| < 1.5e-7, GELU error < 2.2e-7 absolute, checked on [-8, 8])
// on packed fp32 pairs: the polynomial, scaling and select run as v_pk_{fma,mul,add}_f32
// (two lanes' worth per instruction), only rcp / exp2 are per element: ~8 VALU issues per
// element instead of ~19 for gelu_fast.  u = |x|/sqrt2, s = u*sqrt(log2 e):
// Phi(-|x|) = 0.5 * poly(t) * exp(-u^2) = poly'(t) * exp2(-s^2), t = 1 / (1 + p u).
typedef float f32x2 __attribute__((ext_vector_type(2)));
PIPNET_DEV f32x2 gelu_pk(f32x2 x) {
  const f32x2 ax = {fabsf(x[0]), fabsf(x[1])};
  const f32x2 s = ax * 0.84932180028801904272f;                       // sqrt(log2(e) / 2)
  const f32x2 d = __builtin_elementwise_fma(s, (f32x2)0.27273748088f, (f32x2)1.0f);   // p / sqrt(log2 e)
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 q = __builtin_elementwise_fma(t, (f32x2)0.5307027145f, (f32x2)-0.7265760135f);
  q = __builtin_elementwise_fma(t, q, (f32x2)0.7107068705f);
  q = __builtin_elementwise_fma(t, q, (f32x2)-0.142248368f);
  q = __builtin_elementwise_fma(t, q, (f32x2)0.127414796f);
  q = q * t;
  const f32x2 s2 = s * s;
  const f32x2 e = {__builtin_amdgcn_exp2f(-s2[0]), __builtin_amdgcn_exp2f(-s2[1])};
  const f32x2 h = q * e;                                               // Phi(-|x|)
  const f32x2 om = (f32x2)1.0f - h;
  const f32x2 ph = {x[0] < 0.f ? h[0] : om[0], x[1] < 0.f ? h[1] : om[1]};
  return x * ph;
}

// gelu_pk16 (A&S 7.1.28, packed): common.hpp

constexpr int EPI_LAB_GELU_PK = 100;     // tuning lab only: BIAS_GELU through gelu_pk
constexpr int EPI_LAB_GELU_PK16 = 101;   // tuning lab only: BIAS_GELU through gelu_pk16
constexpr int EPI_LAB_GELU_SC16 = 102;   // tuning lab only: gelu_pk16's math on unpacked scalars
constexpr int EPI_LAB_GELU_FAST = 103;   // tuning lab only: gelu_fast (scalar erfc fit, 1 rcp + 1 exp)

// gelu_pk16's A&S 7.1.28 arithmetic with scalar (unpacked) fp32 instructions: packed VALU beside
// another wave's MFMAs costs more than two scalar ops (MI355X_MICROARCH.md cycle constants).
// Not bitwise gelu_pk16 (the packed and scalar fmas round alike, but hipcc may contract differently).
PIPNET_DEV float gelu_sc16(float x) {
  const float hx = x * 0.5f, ahx = fabsf(hx);
  float p = fmaf(ahx, 0.00034451040f, 0.0015645004f);
  p = fmaf(ahx, p, 0.00060805720f);
  p = fmaf(ahx, p, 0.026221010f);
  p = fmaf(ahx, p, 0.084564020f);
  p = fmaf(ahx, p, 0.099734694f);
  p = fmaf(ahx, p, 1.0f);
  p = p * p;
  p = p * p;
  p = p * p;
  p = p * p;
  return fmaf(-ahx, __builtin_amdgcn_rcpf(p), hx + ahx);
}

// accumulators of a (32 TM) x 64 wave tile: acc[i][j] = 32 x 32 block (rows i*32.., cols j*32..);
// TM <= 2 keep the [2][2] shape (TM 1 leaves row 1 unused), TM 3 = the wide tile's 96-row waves
template <int TM>
using AccM = f32x16[TM < 2 ? 2 : TM][2];
using Acc = AccM<2>;

// scalar epilogue (any N / ldc): lane owns column n, rows (v&3) + 8(v>>2) + 4h per tile
template <int EPI, int TM, int R>
PIPNET_DEV void epilogue(const GemmParams& p, const f32x16 (&acc)[R][2], int m0, int n0, int wm, int wn, int lr,
                         int lh) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + lr;
    if (n >= p.N) continue;
    float bn = 0.f, sn = 1.f;
    if (EPI != PIPNET_EPI_NONE && EPI != PIPNET_EPI_MUL && EPI != PIPNET_EPI_GELU_BWD) bn = p.bias ? p.bias[n] : 0.f;
    if (EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_RESID_ROWSCALE) sn = p.scale ? p.scale[n] : 1.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + wm * 32 * TM + i * 32 + (v & 3) + 8 * (v >> 2) + 4 * lh;
        if (m >= p.M) continue;
        float x = acc[i][j][v];
        if (EPI == PIPNET_EPI_BIAS) x = x + bn;
        if (EPI == PIPNET_EPI_BIAS_GELU) x = gelu_fast(x + bn);
        if (EPI == PIPNET_EPI_RESID) x = fmaf(sn, x + bn, p.R[(int64_t)m * p.ldr + n]);
        if (EPI == PIPNET_EPI_RESID_ROWSCALE)
          x = p.R[(int64_t)m * p.ldr + n] + p.row_scale[m / p.rows_per_scale] * (sn * (x + bn));
        if (EPI == PIPNET_EPI_GELU_BWD) x = x * gelu_grad(p.R[(int64_t)m * p.ldr + n]);
        if (EPI == PIPNET_EPI_MUL) x = x * p.R[(int64_t)m * p.ldr + n];
        if (EPI == PIPNET_EPI_BIAS_RELU) x = fmaxf(x + bn, 0.f);
        if (EPI == PIPNET_EPI_BIAS_RESID_RELU) x = fmaxf(x + bn + p.R[(int64_t)m * p.ldr + n], 0.f);
        p.C[(int64_t)m * p.ldc + n] = x;
      }
    }
  }
}

// 16x16x4 accumulator set of a (32*TM)x64 wave tile: acc[ib][jb] is the 16x16 block at rows
// ib*16.., columns jb*16..; register e of lane l holds row 4*(l>>4) + e, column l & 15.
using Acc16 = f32x4[4][4];

template <int EPI, int TM>
PIPNET_DEV void epilogue(const GemmParams& p, const Acc16& acc, int m0, int n0, int wm, int wn, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int n = n0 + wn * 64 + jb * 16 + r16;
    if (n >= p.N) continue;
    float bn = 0.f, sn = 1.f;
    if (EPI != PIPNET_EPI_NONE && EPI != PIPNET_EPI_MUL && EPI != PIPNET_EPI_GELU_BWD) bn = p.bias ? p.bias[n] : 0.f;
    if (EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_RESID_ROWSCALE) sn = p.scale ? p.scale[n] : 1.f;
#pragma unroll
    for (int ib = 0; ib < 2 * TM; ++ib) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 * TM + ib * 16 + 4 * g + e;
        if (m >= p.M) continue;
        float x = acc[ib][jb][e];
        if (EPI == PIPNET_EPI_BIAS) x = x + bn;
        if (EPI == PIPNET_EPI_BIAS_GELU) x = gelu_fast(x + bn);
        if (EPI == PIPNET_EPI_RESID) x = fmaf(sn, x + bn, p.R[(int64_t)m * p.ldr + n]);
        if (EPI == PIPNET_EPI_RESID_ROWSCALE)
          x = p.R[(int64_t)m * p.ldr + n] + p.row_scale[m / p.rows_per_scale] * (sn * (x + bn));
        if (EPI == PIPNET_EPI_GELU_BWD) x = x * gelu_grad(p.R[(int64_t)m * p.ldr + n]);
        if (EPI == PIPNET_EPI_MUL) x = x * p.R[(int64_t)m * p.ldr + n];
        if (EPI == PIPNET_EPI_BIAS_RELU) x = fmaxf(x + bn, 0.f);
        if (EPI == PIPNET_EPI_BIAS_RESID_RELU) x = fmaxf(x + bn + p.R[(int64_t)m * p.ldr + n], 0.f);
        p.C[(int64_t)m * p.ldc + n] = x;
      }
    }
  }
}

// 32-row slab i of a wave's accumulators -> its 32 x 64 LDS image (row-major), per MFMA layout
template <int R>
PIPNET_DEV void slab_write(float* wt, const f32x16 (&acc)[R][2], int i, int lane) {
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int v = 0; v < 16; ++v) wt[((v & 3) + 8 * (v >> 2) + 4 * lh) * 64 + j * 32 + lr] = acc[i][j][v];
}
PIPNET_DEV void slab_write(float* wt, const Acc16& acc, int i, int lane) {
  const int r16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
      for (int e = 0; e < 4; ++e) wt[(h * 16 + 4 * g + e) * 64 + jb * 16 + r16] = acc[2 * i + h][jb][e];
}

template <int EPI>
PIPNET_DEV f32x4 epi_math(f32x4 x, const f32x4& bn, const f32x4& sn, const f32x4& r, float rs = 1.f) {
  if (EPI == PIPNET_EPI_BIAS) x = x + bn;
  if (EPI == PIPNET_EPI_BIAS_GELU) {      // packed A&S 7.1.28 (lab: +2..+8 % over gelu_fast)
    x = x + bn;
    const f32x2 lo = gelu_pk16(f32x2{x[0], x[1]}), hi = gelu_pk16(f32x2{x[2], x[3]});
    x = f32x4{lo[0], lo[1], hi[0], hi[1]};
  }
  if (EPI == EPI_LAB_GELU_SC16 || EPI == EPI_LAB_GELU_FAST) {
    x = x + bn;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = EPI == EPI_LAB_GELU_SC16 ? gelu_sc16(x[e]) : gelu_fast(x[e]);
  }
  if (EPI == EPI_LAB_GELU_PK || EPI == EPI_LAB_GELU_PK16) {
    x = x + bn;
    f32x2 lo, hi;
    if (EPI == EPI_LAB_GELU_PK) lo = gelu_pk(f32x2{x[0], x[1]}), hi = gelu_pk(f32x2{x[2], x[3]});
    else lo = gelu_pk16(f32x2{x[0], x[1]}), hi = gelu_pk16(f32x2{x[2], x[3]});
    x = f32x4{lo[0], lo[1], hi[0], hi[1]};
  }
  // explicit fma: the streaming kernel's scalar epilogue (epi_scalar) must round identically
  if (EPI == PIPNET_EPI_RESID) x = __builtin_elementwise_fma(sn, x + bn, r);
  if (EPI == PIPNET_EPI_RESID_ROWSCALE) x = r + rs * (sn * (x + bn));   // (ls * y) * (mask / keep) + x
  if (EPI == PIPNET_EPI_GELU_BWD) {
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = x[e] * gelu_grad(r[e]);
  }
  if (EPI == PIPNET_EPI_MUL) x = x * r;
  if (EPI == PIPNET_EPI_BIAS_RELU) {
    x = x + bn;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
  }
  if (EPI == PIPNET_EPI_BIAS_RESID_RELU) {
    x = x + bn + r;
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
  }
  return x;
}

// Output-tile store: non-temporal, so the streaming C tiles do not evict the A / W panels
// other workgroups of the XCD still read (s384 fc1: 338 -> 184 MiB fetched per launch at
// equal time, profiles/r02/gemm_raster_store_ab.txt).
PIPNET_DEV void st4_c(float* p, f32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p)); }

// Vectorised epilogue: each wave re-lays its accumulator tile through LDS (32 rows at a
// time, 8 KiB per wave) so every global store / residual load is a float4 and one wave
// instruction covers 4 rows x 256 B -- the lane-per-column MFMA layout would otherwise
// cost 64 scattered dword stores (and loads) per lane, which measured as long as the
// whole main loop on the K=96 GEMMs.  All residual float4 loads of a lane are issued
// before the first store (one latency, not sixteen).  Needs N % 4 == 0, ldc / ldr % 4 ==
// 0, 16-B aligned C / R, and 32 KiB of the kernel's LDS (free after the main loop).
template <int EPI, int TM, class AccT, int ABL = 0>
PIPNET_DEV void epilogue_vec(const GemmParams& p, const AccT& acc, float* smem, int m0, int n0, int wm, int wn,
                             int lane, int wid) {
  constexpr bool HAS_R = EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_MUL || EPI == PIPNET_EPI_BIAS_RESID_RELU ||
                         EPI == PIPNET_EPI_RESID_ROWSCALE || EPI == PIPNET_EPI_GELU_BWD;
  float* wt = smem + wid * 32 * 64;
  const int c4 = lane & 15;
  const int n = n0 + wn * 64 + 4 * c4;
  const bool nok = n < p.N;
  f32x4 bn = {0.f, 0.f, 0.f, 0.f}, sn = {1.f, 1.f, 1.f, 1.f};
  if (EPI != PIPNET_EPI_NONE && EPI != PIPNET_EPI_MUL && EPI != PIPNET_EPI_GELU_BWD && p.bias && nok)
    bn = ld4(p.bias + n);   // (incl. lab GELU)
  if ((EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_RESID_ROWSCALE) && p.scale && nok) sn = ld4(p.scale + n);
  // Row addresses as running pointers (+4 rows per step; the residual's clamped rows by a
  // select): a per-access (int64) m * ld is three quarter-rate integer multiplies per store.
  const int mrow0 = m0 + wm * 32 * TM + (lane >> 4);
  // TM <= 2: every residual float4 of the lane loaded before the first slab (one latency);
  // TM 3 (96-row waves beside 96 accumulators): one slab's 8 at a time, issued once that slab's
  // accumulators are in LDS (before the barrier)
  constexpr bool PRE = TM <= 2;
  f32x4 r[PRE ? TM : 1][8];
  if (HAS_R && PRE) {
    const float* rp = p.R + (int64_t)mrow0 * p.ldr + n;
    const float* const rlast = p.R + (int64_t)(p.M - 1) * p.ldr + n;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const float* src = mrow0 + i * 32 + it * 4 < p.M ? rp : rlast;
        r[i][it] = nok ? ld4(src) : f32x4{0.f, 0.f, 0.f, 0.f};
        rp += 4 * p.ldr;
      }
  }
  float* op = p.C + (int64_t)mrow0 * p.ldc + n;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    __syncthreads();
    slab_write(wt, acc, i, lane);
    if (HAS_R && !PRE) {                  // after the slab's accumulators are dead
      const float* rp = p.R + (int64_t)(mrow0 + i * 32) * p.ldr + n;
      const float* const rlast = p.R + (int64_t)(p.M - 1) * p.ldr + n;
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const float* src = mrow0 + i * 32 + it * 4 < p.M ? rp : rlast;
        r[0][it] = nok ? ld4(src) : f32x4{0.f, 0.f, 0.f, 0.f};
        rp += 4 * p.ldr;
      }
    }
    __syncthreads();
    lab_stamp<ABL>(p, 8 + 2 * i);
    if (i == 0 || !PRE) vm_drain();       // bias / residual preloads landed (common.hpp)
    // the slab's 8 LDS reads issued together, outside the row-guarded stores (one latency)
    f32x4 sv[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) sv[it] = ld4(wt + (it * 4 + (lane >> 4)) * 64 + 4 * c4);
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = it * 4 + (lane >> 4);
      const int m = m0 + wm * 32 * TM + i * 32 + row;
      float rs = 1.f;
      if constexpr (EPI == PIPNET_EPI_RESID_ROWSCALE) rs = p.row_scale[min(m, p.M - 1) / p.rows_per_scale];
      const f32x4 x = epi_math<EPI>(sv[it], bn, sn, HAS_R ? r[PRE ? i : 0][it] : bn, rs);
      if (m < p.M && nok) st4_c(op, x);
      op += 4 * p.ldc;
      if constexpr ((ABL & 8) != 0) {     // lab: per-iteration timing of the first slab
        if (i == 0 && it == 0) lab_stamp<ABL>(p, 12);
        if (i == 0 && it == 1) lab_stamp<ABL>(p, 13);
        if (i == 0 && it == 3) lab_stamp<ABL>(p, 14);
        if (i == 0 && it == 5) lab_stamp<ABL>(p, 15);
      }
    }
    lab_stamp<ABL>(p, 9 + 2 * i);
  }
}

// XCD-contiguous tile ranges, group_m-grouped raster (m fastest inside a group).  (An
// XCD-slab raster -- each XCD owning an N slab so its W panels stay L2-resident -- measured no
// faster, profiles/r02/gemm_raster_store_ab.txt.)
PIPNET_DEV void tile_coords(const GemmParams& p, int bm, int& m0, int& n0, int bn = BN) {
  const int nwg = p.mt * p.nt;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int gm = p.group_m;
  const int group = tile / (gm * p.nt);
  const int first_m = group * gm;
  const int gsz = min(p.mt - first_m, gm);
  const int in_group = tile - group * gm * p.nt;
  m0 = (first_m + in_group % gsz) * bm;
  n0 = (in_group / gsz) * bn;
}

PIPNET_DEV void zero_acc(Acc16& acc) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

template <int R>
PIPNET_DEV void zero_acc(f32x16 (&acc)[R][2]) {
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
}

// ======================================================================================
// main path: LDS-DMA staging, swizzled rows, pipelined fragments (K % BK == 0)
// ======================================================================================
// WGM = waves along M (2: the product's 4-wave 2x2 workgroup; 4: an 8-wave 4x2 workgroup -- same wave
// tile, same K order -- lab only: +4-8 % on the stage-4 GEMMs standalone, nothing inside C2)
// WGN = waves along N (2: 128 columns; 6: the wide tile's 384 columns, gemm_f32_tnw_kernel)
template <int BK, int TM, int WGM = 2, int WGN = 2>
struct Geo {
  static constexpr int NW = WGM * WGN;                    // waves per workgroup
  static constexpr int BMT = 32 * TM * WGM;               // tile rows of A
  static constexpr int BNT = 64 * WGN;                    // tile rows of W (output columns)
  static constexpr int CHUNKS = BK / 4;                   // 16-B chunks per LDS row
  static constexpr int ROWS_PER_DMA = 64 / CHUNKS;        // rows one 1-KiB DMA fills
  static constexpr int A_DMA = BMT / ROWS_PER_DMA / NW;
  static constexpr int B_DMA = BNT / ROWS_PER_DMA / NW;
  static constexpr int TILE_FLOATS = (BMT + BNT) * BK;    // one buffer: A rows then B rows
  static_assert(A_DMA * ROWS_PER_DMA * NW == BMT && B_DMA * ROWS_PER_DMA * NW == BNT, "DMA rows per wave");
  static constexpr int NGROUPS = BK / 8;                  // 4-deep fragment groups per half-wave
  // chunk swizzle: the 16 lanes of a ds_read_b128 group read 16 distinct bank slots
  static PIPNET_DEV int swz(int row, int c) {
    return BK == 32 ? (c ^ ((row >> 1) & 7)) : (c ^ ((row >> 2) & 3));
  }
};

template <int TM>
struct FragM {
  f32x4 a[TM < 2 ? 2 : TM], b[2];
};
using Frag = FragM<2>;

template <int BK, int TM, int WGM = 2, int WGN = 2, class F>
PIPNET_DEV void read_frag(F& f, const float* buf, int wm, int wn, int lr, int lh, int q) {
  using G = Geo<BK, TM, WGM, WGN>;
  const int c = lh * (G::CHUNKS / 2) + q;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int ra = wm * 32 * TM + i * 32 + lr;
    f.a[i] = ld4(buf + ra * BK + 4 * G::swz(ra, c));
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rb = wn * 64 + j * 32 + lr;
    f.b[j] = ld4(buf + G::BMT * BK + rb * BK + 4 * G::swz(rb, c));
  }
}

// JL = how many of the wave's two 32-column blocks take part (2 everywhere except NPAD
// waves whose blocks lie past N); a compile-time count, so the MFMA stream stays branch-free.
template <int TM, int JL = 2, int R, class F>
PIPNET_DEV void mfma_frag(f32x16 (&acc)[R][2], const F& f) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < JL; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[i][e], f.b[j][e], acc[i][j], 0, 0, 0);
}

// v_mfma_f32_16x16x4_f32 operands (cdna_hip_programming.md section 3: lane l supplies
// A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]).  Group q of a BK-deep LDS tile: lane group
// g = l >> 4 reads logical chunk 4q + g (4 consecutive k) of row (l & 15) of every 16-row
// block, so MFMA e of the group multiplies k = 4 (4q + g) + e in lane group g -- the same map
// for both operands, so every k of the tile is summed once.  With the swz() XOR above every
// ds_read_b128 lane group ({0-3,12-15,20-27}, ...) hits 16 distinct 16-B bank slots (BK 32).
struct Frag16 {
  f32x4 a[4], b[4];
};

template <int BK, int TM, int WGM = 2>
PIPNET_DEV void read_frag16(Frag16& f, const float* buf, int wm, int wn, int lane, int q) {
  using G = Geo<BK, TM, WGM>;
  const int r16 = lane & 15, c = 4 * q + (lane >> 4);
#pragma unroll
  for (int ib = 0; ib < 2 * TM; ++ib) {
    const int ra = wm * 32 * TM + ib * 16 + r16;
    f.a[ib] = ld4(buf + ra * BK + 4 * G::swz(ra, c));
  }
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    const int rb = wn * 64 + jb * 16 + r16;
    f.b[jb] = ld4(buf + G::BMT * BK + rb * BK + 4 * G::swz(rb, c));
  }
}

// JL = active 32-column blocks of the wave (NPAD), i.e. 2 * JL 16-column blocks
template <int TM, int JL = 2>
PIPNET_DEV void mfma_frag16(Acc16& acc, const Frag16& f) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int ib = 0; ib < 2 * TM; ++ib)
#pragma unroll
      for (int jb = 0; jb < 2 * JL; ++jb)
        acc[ib][jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(f.a[ib][e], f.b[jb][e], acc[ib][jb], 0, 0, 0);
}

template <int V>
struct IntC {
  static constexpr int value = V;
};

PIPNET_DEV void dma16(const float* src, float* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Retire all but the NPEND youngest vector-memory ops of this wave (LDS-DMA counts as VMEM),
// drain this wave's LDS reads, then the workgroup barrier -- one asm block, so hipcc cannot
// widen it to vmcnt(0) (cdna_hip_programming.md 5, "Pipelining across barriers").
template <int NPEND>
PIPNET_DEV void wait_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NPEND) : "memory");
}

// ABL (tuning-lab ablations only, 0 in the product): 1 = no DMA (stale LDS), 2 = no
// epilogue (one store per lane keeps the accumulators live), 4 = no barrier, 8 = stamps.
// NS = LDS stages: tile k+NS-1 is in flight while tile k is multiplied.
// NPAD (grids whose N % 128 != 0): MFMA blocks of columns >= N are skipped, and the wave ->
// column-half map flips with the workgroup parity, so the lighter waves of co-resident
// workgroups land on different SIMDs (a relabelling: every output is computed identically).
// SH = MFMA shape: 0 = v_mfma_f32_32x32x2_f32, 1 = v_mfma_f32_16x16x4_f32 (same tile, LDS image,
// DMA and fragment bytes; a different k order inside each K-tile, so a different rounding).
template <int SH, int BK, int TM, int EPI, int ALOAD, int NS, int ABL, bool NPAD, int WGM = 2, int WGN = 2>
PIPNET_DEV void gemm_tn_body(GemmParams p, float* smem) {
  using G = Geo<BK, TM, WGM, WGN>;
  static_assert(!NPAD || WGN == 2, "NPAD column flip: two waves along N");
  static_assert(SH == 0 || TM <= 2, "16x16x4 accumulators: TM <= 2");
  constexpr int NWAVES = G::NW;
  static_assert(SH == 0 || BK == 32, "16x16x4 fragments: BK 32 (the swizzle is conflict-free there)");
  // split-K: workgroup row y reduces K-tiles [y*nk/S, (y+1)*nk/S) into its own C slab
  const int nk_all = p.K / BK;
  const int kt_begin = (int)((int64_t)nk_all * blockIdx.y / gridDim.y);
  const int nk = (int)((int64_t)nk_all * (blockIdx.y + 1) / gridDim.y) - kt_begin;
  p.C += (int64_t)blockIdx.y * p.split_stride;
  constexpr int DMA_PER_TILE = G::A_DMA + G::B_DMA;     // per wave
  static_assert(NS * G::TILE_FLOATS >= NWAVES * 32 * 64, "vector epilogue needs 8 KiB of LDS per wave");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WGN, wn = NPAD ? ((wid & 1) ^ (int)(blockIdx.x & 1)) : wid % WGN;
  const int lr = lane & 31, lh = lane >> 5;
  int m0, n0;
  tile_coords(p, G::BMT, m0, n0, G::BNT);
  const int jl = NPAD ? __builtin_amdgcn_readfirstlane(min(2, max(0, (p.N - n0 - wn * 64 + 31) >> 5))) : 2;
  if (p.stagger && (int)blockIdx.x >= p.stagger_lo && (int)blockIdx.x < p.stagger_hi)
    for (int i = 0; i < p.stagger; ++i) __builtin_amdgcn_s_sleep(127);

  // DMA sources: instruction i of this wave fills tile rows (i*NWAVES+wid)*ROWS_PER_DMA + ..;
  // lane writes row +lane/CHUNKS, physical chunk lane%CHUNKS -> fetches chunk c = swz(row, phys).
  const int drow = lane / G::CHUNKS;
  ARow arow[G::A_DMA];
  int achunk[G::A_DMA];
  const float* wsrc[G::B_DMA];
#pragma unroll
  for (int i = 0; i < G::A_DMA; ++i) {
    const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + drow;
    const int c = G::swz(row, lane % G::CHUNKS);
    achunk[i] = 4 * c;
    arow[i] = a_row<ALOAD>(p, min(m0 + row, p.M - 1));   // rows past M: valid, never stored
  }
#pragma unroll
  for (int i = 0; i < G::B_DMA; ++i) {
    const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + drow;
    const int c = G::swz(row, lane % G::CHUNKS);
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + 4 * c;
  }
  // Implicit-GEMM convolutions with Cin % BK == 0: a K-tile never straddles two taps, so the
  // (channel, kx, ky) of the next K-tile the DMA fetches is tracked incrementally (stage() is
  // called for consecutive K-tiles) -- wave-uniform, no per-lane division in the loop.
  const bool tap_walk = ALOAD != ALOAD_DENSE && p.Cin % BK == 0;
  int t_c = 0, t_kx = 0, t_ky = 0;
  if (ALOAD != ALOAD_DENSE && tap_walk) {
    const int k = kt_begin * BK, tap = k / p.Cin;
    t_c = k - tap * p.Cin;
    t_ky = ALOAD == ALOAD_CONV2X2 ? tap >> 1 : tap / p.KW;
    t_kx = ALOAD == ALOAD_CONV2X2 ? tap & 1 : tap - t_ky * p.KW;
  }
  auto a_src = [&](const ARow& r, int k0, int chunk) -> const float* {
    if (ALOAD == ALOAD_DENSE || !tap_walk) return a_ptr<ALOAD>(p, r, k0 + chunk);
    if (ALOAD == ALOAD_CONV2X2) return p.A + r.base + ((int64_t)t_ky * p.Wd + t_kx) * p.Cin + t_c + chunk;
    const int iy = r.iy0 + t_ky, ix = r.ix0 + t_kx;
    if ((unsigned)iy >= (unsigned)p.H || (unsigned)ix >= (unsigned)p.Wd) return g_zero4;
    return p.A + r.base + ((int64_t)iy * p.Wd + ix) * p.Cin + t_c + chunk;
  };
  auto stage = [&](int kt, int buf) {
    if (ABL & 1) return;
    float* base = smem + buf * G::TILE_FLOATS;
    const int k0 = (kt_begin + kt) * BK;
#pragma unroll
    for (int i = 0; i < G::A_DMA; ++i)
      dma16(a_src(arow[i], k0, achunk[i]), base + (i * NWAVES + wid) * G::ROWS_PER_DMA * BK);
    if (ALOAD != ALOAD_DENSE && tap_walk) {
      t_c += BK;
      if (t_c == p.Cin) {
        t_c = 0;
        if (++t_kx == (ALOAD == ALOAD_CONV2X2 ? 2 : p.KW)) t_kx = 0, ++t_ky;
      }
    }
#pragma unroll
    for (int i = 0; i < G::B_DMA; ++i)
      dma16(wsrc[i] + k0, base + G::BMT * BK + (i * NWAVES + wid) * G::ROWS_PER_DMA * BK);
  };
  // barrier once tile `need` has landed, `last` = youngest tile in flight
  auto wait_tile = [&](int need, int last) {
    if constexpr (NS == 2) {
      __syncthreads();
    } else {
      const int pend = last - need;
      if (NS >= 4 && pend >= 2) wait_dma_barrier<(NS >= 4 ? 2 : 0) * DMA_PER_TILE>();
      else if (pend >= 1) wait_dma_barrier<DMA_PER_TILE>();
      else wait_dma_barrier<0>();
    }
  };

  using AccT = typename std::conditional<SH == 0, AccM<TM>, Acc16>::type;
  AccT acc;
  zero_acc(acc);
  lab_stamp<ABL>(p, 0);

  int issued = -1;                                  // youngest tile whose DMA is in flight
  for (int s0 = 0; s0 < NS - 1 && s0 < nk; ++s0) stage(s0, s0), issued = s0;
  wait_tile(0, issued);
  lab_stamp<ABL>(p, 1);
  // main loop, instantiated per JL (the wave's active 32-column blocks): one wave-uniform
  // branch here instead of one per MFMA group
  auto main_loop = [&](auto jlc) {
    constexpr int JL = decltype(jlc)::value;
    if constexpr (SH == 1) {
      // 2 fragment groups of 64 MFMAs (2048 cycles per wave) per 32-deep K-tile
      Frag16 fa, fb;
      read_frag16<BK, TM, WGM>(fa, smem, wm, wn, lane, 0);
      int cur = 0;
      for (int kt = 0; kt < nk; ++kt) {
        const float* buf = smem + cur * G::TILE_FLOATS;
        if (kt + NS - 1 < nk) {
          int nb = cur + NS - 1;
          if (nb >= NS) nb -= NS;
          stage(kt + NS - 1, nb);
          issued = kt + NS - 1;
        }
        read_frag16<BK, TM, WGM>(fb, buf, wm, wn, lane, 1);
        mfma_frag16<TM, JL>(acc, fa);
        const int nxt = (cur + 1 == NS) ? 0 : cur + 1;
        if (!(ABL & 4)) wait_tile(kt + 1 < nk ? kt + 1 : issued, issued);
        if (kt + 1 < nk) read_frag16<BK, TM, WGM>(fa, smem + nxt * G::TILE_FLOATS, wm, wn, lane, 0);
        mfma_frag16<TM, JL>(acc, fb);
        cur = nxt;
      }
      return;
    } else {
    FragM<TM> fa, fb;
    read_frag<BK, TM, WGM, WGN>(fa, smem, wm, wn, lr, lh, 0);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const float* buf = smem + cur * G::TILE_FLOATS;
      if (kt + NS - 1 < nk) {
        int nb = cur + NS - 1;
        if (nb >= NS) nb -= NS;
        stage(kt + NS - 1, nb);
        issued = kt + NS - 1;
      }
      if constexpr (G::NGROUPS == 4) {
        read_frag<BK, TM, WGM, WGN>(fb, buf, wm, wn, lr, lh, 1);
        mfma_frag<TM, JL>(acc, fa);
        read_frag<BK, TM, WGM, WGN>(fa, buf, wm, wn, lr, lh, 2);
        mfma_frag<TM, JL>(acc, fb);
        read_frag<BK, TM, WGM, WGN>(fb, buf, wm, wn, lr, lh, 3);
        mfma_frag<TM, JL>(acc, fa);
      } else {
        read_frag<BK, TM, WGM, WGN>(fb, buf, wm, wn, lr, lh, 1);
        mfma_frag<TM, JL>(acc, fa);
      }
      const int nxt = (cur + 1 == NS) ? 0 : cur + 1;
      if (!(ABL & 4)) wait_tile(kt + 1 < nk ? kt + 1 : issued, issued);   // tile kt+1 landed, tile kt read
      if (kt + 1 < nk) read_frag<BK, TM, WGM, WGN>(fa, smem + nxt * G::TILE_FLOATS, wm, wn, lr, lh, 0);
      mfma_frag<TM, JL>(acc, fb);
      cur = nxt;
    }
    }
  };
  if constexpr (NPAD) {
    if (jl >= 2) main_loop(IntC<2>{});
    else if (jl == 1) main_loop(IntC<1>{});
    else main_loop(IntC<0>{});
  } else {
    main_loop(IntC<2>{});
  }
  lab_stamp<ABL>(p, 2);
  if (ABL & 2) {
    const float* av = reinterpret_cast<const float*>(&acc);
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < (int)(sizeof(AccT) / sizeof(float)); ++v) t += av[v];
    p.C[(int64_t)blockIdx.x * 64 * NWAVES + tid] = t;
    return;
  }
  if (WGN != 2 || p.vec_epi)            // the wide tile is launched for float4 epilogues only
    epilogue_vec<EPI, TM, AccT, ABL>(p, acc, smem, m0, n0, wm, wn, lane, wid);
  else if constexpr (WGN != 2)
    return;
  else if constexpr (SH == 0)
    epilogue<EPI, TM>(p, acc, m0, n0, wm, wn, lr, lh);
  else
    epilogue<EPI, TM>(p, acc, m0, n0, wm, wn, lane);
  if constexpr ((ABL & 8) != 0) {
    __syncthreads();
    lab_stamp<ABL>(p, 3);
  }
}

template <int BK, int TM, int EPI, int ALOAD, int MINB, int NS = 2, int ABL = 0, bool NPAD = false>
__global__ __launch_bounds__(NTHREADS, MINB) void gemm_f32_tn_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[NS * Geo<BK, TM>::TILE_FLOATS];
  gemm_tn_body<0, BK, TM, EPI, ALOAD, NS, ABL, NPAD>(p, smem);
}

// 8-wave form (WGM = 4): a (128 TM) x 128 tile, waves 4 (M) x 2 (N) of the same (32 TM) x 64 wave
// tile (tuning lab tools/gemm_lab.hip variants 60+; not dispatched by the product)
template <int BK, int TM, int EPI, int ALOAD, int MINB, int NS, int ABL = 0, int SH = 0>
__global__ __launch_bounds__(512, MINB) void gemm_f32_tn8_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[NS * Geo<BK, TM, 4>::TILE_FLOATS];
  gemm_tn_body<SH, BK, TM, EPI, ALOAD, NS, ABL, false, 4>(p, smem);
}

// Wide form: a 192 x 384 tile on 12 waves, 2 (M) x 6 (N) of a 96 x 64 wave tile (TM 3) -- the whole
// N of a 384-column product in one workgroup, so each A panel is fetched once, and 243 tiles of
// C2's stage-3 fc2 (M = 46,656) fill the 256 CUs in one round.  Per 32-deep K-tile: 73.7 KB of
// LDS-DMA for 4.7 MFLOP (64 flop per staged byte, 2x the 128 x 128 tile).  One workgroup per CU
// (2 x 72 KiB stages), 3 waves per SIMD.
template <int EPI, int ALOAD, int ABL = 0>
__global__ __launch_bounds__(768, 1) void gemm_f32_tnw_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * Geo<32, 3, 2, 6>::TILE_FLOATS];
  gemm_tn_body<0, 32, 3, EPI, ALOAD, 2, ABL, false, 2, 6>(p, smem);
}

// the same tile on v_mfma_f32_16x16x4_f32
template <int BK, int TM, int EPI, int ALOAD, int MINB, int NS = 2, int ABL = 0, bool NPAD = false>
__global__ __launch_bounds__(NTHREADS, MINB) void gemm_f32_tn16_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[NS * Geo<BK, TM>::TILE_FLOATS];
  gemm_tn_body<1, BK, TM, EPI, ALOAD, NS, ABL, NPAD>(p, smem);
}

// ======================================================================================
// general path: register staging, zero-filled K tail (K % 4 == 0), 128x128x32 tiles
// ======================================================================================
constexpr int TBM = 128, TBK = 32, LDK = TBK + 4;   // padded rows (144 B): conflict-free ds_read_b128

template <int EPI, int ALOAD>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_f32_tn_ktail_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (TBM + BN) * LDK];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  int m0, n0;
  tile_coords(p, TBM, m0, n0);

  const int srow = tid >> 3;
  const int sk = (tid & 7) * 4;
  ARow arow[4];
  bool aval[4];
  const float* wrow[4];
  bool wval[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + srow + 32 * i;
    aval[i] = m < p.M;
    arow[i] = a_row<ALOAD>(p, aval[i] ? m : 0);
    const int n = n0 + srow + 32 * i;
    wval[i] = n < p.N;
    wrow[i] = p.W + (int64_t)(wval[i] ? n : 0) * p.K;
  }
  f32x4 ra[4], rb[4];
  auto gload = [&](int kt) {
    const int k = kt * TBK + sk;
    const bool kin = k < p.K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = (aval[i] && kin) ? ld4(a_ptr<ALOAD>(p, arow[i], k)) : f32x4{0.f, 0.f, 0.f, 0.f};
      rb[i] = (wval[i] && kin) ? ld4(wrow[i] + k) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto sstore = [&](int buf) {
    float* As = smem + buf * (TBM + BN) * LDK;
    float* Bs = As + TBM * LDK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st4(As + (srow + 32 * i) * LDK + sk, ra[i]);
      st4(Bs + (srow + 32 * i) * LDK + sk, rb[i]);
    }
  };

  Acc acc;
  zero_acc(acc);
  const int nk = (p.K + TBK - 1) / TBK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
    const float* As = smem + buf * (TBM + BN) * LDK;
    const float* Bs = As + TBM * LDK;
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
    for (int kk = 0; kk < 16; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][kk >> 2][kk & 3], fb[j][kk >> 2][kk & 3],
                                                           acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
  epilogue<EPI, 2>(p, acc, m0, n0, wm, wn, lr, lh);
}

}  // namespace pipnet_gemm
