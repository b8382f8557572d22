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
// Tile: 128x128xBK per 256-thread workgroup, 4 waves in 2x2, each wave 64x64 = 2x2 MFMA
// 32x32 tiles (64 accumulator VGPRs).  For v_mfma_f32_32x32x2_f32 lane l supplies
// A[l&31][k] and B[k][l&31] with k = l>>5 of the 2-deep step; the k order inside a
// BK-deep LDS tile is free (both operands use the same map), so half-wave h walks
// k = h*BK/2 .. (h+1)*BK/2-1 and reads its operands 4 k-steps at a time (ds_read_b128).
//
// Main path (K % BK == 0): global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave instruction), two LDS buffers, one barrier per K-tile.  LDS rows are BK*4 bytes
// with the 16-B chunk index XOR-swizzled by a row-dependent mask: the DMA writes
// lane-linear, so the swizzle is applied to each lane's SOURCE address and undone on the
// read (cdna_hip_programming.md rule 21); every ds_read_b128 lane group then hits 16
// distinct 16-B bank slots.  Operand fragments are software-pipelined in two named
// register sets, and the first fragment group of tile k+1 is read right after the
// barrier, under the last MFMA group of tile k.  BK=16 keeps a workgroup at 32 KiB of
// LDS and 128 VGPRs so four workgroups (16 waves) share a CU and hide the DMA latency.
// General path (any K % 4): register staging with zero-fill of the K tail.
#pragma once
#include "common.hpp"

namespace pipnet_gemm {

constexpr int BM = 128, BN = 128, NTHREADS = 256, NWAVES = 4;

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
  int mt, nt, group_m;
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

template <int EPI>
PIPNET_DEV void epilogue(const GemmParams& p, const f32x16 (&acc)[2][2], int m0, int n0, int wm, int wn, int lr,
                         int lh) {
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
        if (EPI == PIPNET_EPI_BIAS_GELU) x = gelu_fast(x + bn);
        if (EPI == PIPNET_EPI_RESID) x = p.R[(int64_t)m * p.ldr + n] + sn * (x + bn);
        if (EPI == PIPNET_EPI_MUL) x = x * p.R[(int64_t)m * p.ldr + n];
        p.C[(int64_t)m * p.ldc + n] = x;
      }
    }
  }
}

// XCD-contiguous tile ranges, group_m-grouped raster (m fastest inside a group).
PIPNET_DEV void tile_coords(const GemmParams& p, int& m0, int& n0) {
  const int nwg = p.mt * p.nt;
  const int tile = xcd_remap(blockIdx.x, nwg);
  const int gm = p.group_m;
  const int group = tile / (gm * p.nt);
  const int first_m = group * gm;
  const int gsz = min(p.mt - first_m, gm);
  const int in_group = tile - group * gm * p.nt;
  m0 = (first_m + in_group % gsz) * BM;
  n0 = (in_group / gsz) * BN;
}

PIPNET_DEV void zero_acc(f32x16 (&acc)[2][2]) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
}

// ======================================================================================
// main path: LDS-DMA staging, swizzled rows, pipelined fragments (K % BK == 0)
// ======================================================================================
template <int BK>
struct Geo {
  static constexpr int CHUNKS = BK / 4;                   // 16-B chunks per LDS row
  static constexpr int ROWS_PER_DMA = 64 / CHUNKS;        // rows one 1-KiB DMA fills
  static constexpr int DMA_PER_WAVE = BM / ROWS_PER_DMA / NWAVES;
  static constexpr int TILE_FLOATS = (BM + BN) * BK;      // one buffer: A rows then B rows
  static constexpr int NGROUPS = BK / 8;                  // 4-deep fragment groups per half-wave
  // chunk swizzle: the 16 lanes of a ds_read_b128 group read 16 distinct bank slots
  static PIPNET_DEV int swz(int row, int c) {
    return BK == 32 ? (c ^ ((row >> 1) & 7)) : (c ^ ((row >> 2) & 3));
  }
};

struct Frag {
  f32x4 a[2], b[2];
};

template <int BK>
PIPNET_DEV void read_frag(Frag& f, const float* buf, int wm, int wn, int lr, int lh, int q) {
  using G = Geo<BK>;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int ra = wm * 64 + i * 32 + lr;
    const int rb = wn * 64 + i * 32 + lr;
    const int c = lh * (G::CHUNKS / 2) + q;
    f.a[i] = ld4(buf + ra * BK + 4 * G::swz(ra, c));
    f.b[i] = ld4(buf + BM * BK + rb * BK + 4 * G::swz(rb, c));
  }
}

PIPNET_DEV void mfma_frag(f32x16 (&acc)[2][2], const Frag& f) {
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.a[i][e], f.b[j][e], acc[i][j], 0, 0, 0);
}

PIPNET_DEV void dma16(const float* src, float* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

template <int BK, int EPI, int ALOAD, int MINB>
__global__ __launch_bounds__(NTHREADS, MINB) void gemm_f32_tn_kernel(GemmParams p) {
  using G = Geo<BK>;
  __shared__ __attribute__((aligned(16))) float smem[2 * G::TILE_FLOATS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  int m0, n0;
  tile_coords(p, m0, n0);

  // DMA sources: instruction i of this wave fills tile rows (i*NWAVES+wid)*ROWS_PER_DMA + ..;
  // lane writes row +lane/CHUNKS, physical chunk lane%CHUNKS -> fetches chunk c = swz(row, phys).
  int64_t asrc[G::DMA_PER_WAVE];
  const float* wsrc[G::DMA_PER_WAVE];
  int achunk[G::DMA_PER_WAVE];
#pragma unroll
  for (int i = 0; i < G::DMA_PER_WAVE; ++i) {
    const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + lane / G::CHUNKS;
    const int c = G::swz(row, lane % G::CHUNKS);
    achunk[i] = 4 * c;
    const int m = min(m0 + row, p.M - 1);           // out-of-range rows: any valid row, never stored
    const int n = min(n0 + row, p.N - 1);
    asrc[i] = a_row_base<ALOAD>(p, m);
    wsrc[i] = p.W + (int64_t)n * p.K + 4 * c;
  }
  auto stage = [&](int kt, int buf) {
    float* base = smem + buf * G::TILE_FLOATS;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < G::DMA_PER_WAVE; ++i) {
      const int rb = (i * NWAVES + wid) * G::ROWS_PER_DMA;
      dma16(p.A + asrc[i] + a_col_off<ALOAD>(p, k0 + achunk[i]), base + rb * BK);
      dma16(wsrc[i] + k0, base + BM * BK + rb * BK);
    }
  };

  f32x16 acc[2][2];
  zero_acc(acc);
  const int nk = p.K / BK;

  stage(0, 0);
  __syncthreads();
  Frag fa, fb;
  read_frag<BK>(fa, smem, wm, wn, lr, lh, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const float* buf = smem + cur * G::TILE_FLOATS;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    if constexpr (G::NGROUPS == 4) {
      read_frag<BK>(fb, buf, wm, wn, lr, lh, 1);
      mfma_frag(acc, fa);
      read_frag<BK>(fa, buf, wm, wn, lr, lh, 2);
      mfma_frag(acc, fb);
      read_frag<BK>(fb, buf, wm, wn, lr, lh, 3);
      mfma_frag(acc, fa);
    } else {
      read_frag<BK>(fb, buf, wm, wn, lr, lh, 1);
      mfma_frag(acc, fa);
    }
    __syncthreads();                                  // tile kt+1 landed, tile kt fully read
    if (kt + 1 < nk) read_frag<BK>(fa, smem + (cur ^ 1) * G::TILE_FLOATS, wm, wn, lr, lh, 0);
    mfma_frag(acc, fb);
  }
  epilogue<EPI>(p, acc, m0, n0, wm, wn, lr, lh);
}

// ======================================================================================
// general path: register staging, zero-filled K tail (K % 4 == 0)
// ======================================================================================
constexpr int TBK = 32, LDK = TBK + 4;   // padded rows (144 B): conflict-free ds_read_b128

template <int EPI, int ALOAD>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_f32_tn_ktail_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDK];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  int m0, n0;
  tile_coords(p, m0, n0);

  const int srow = tid >> 3;
  const int sk = (tid & 7) * 4;
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
    const int k = kt * TBK + sk;
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
  zero_acc(acc);
  const int nk = (p.K + TBK - 1) / TBK;
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
  epilogue<EPI>(p, acc, m0, n0, wm, wn, lr, lh);
}

}  // namespace pipnet_gemm
