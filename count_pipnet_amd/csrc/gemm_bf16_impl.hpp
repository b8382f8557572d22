// bf16 implicit-GEMM convolution on gfx950 matrix cores (v_mfma_f32_32x32x16_bf16), fp32
// accumulation, bf16 NHWC activations in and out.  Serves the ResNet backbones in the
// BASELINE C3 configuration ("PIP-Net ResNet50 ... bf16 inference"; SURVEY.md 8a a7:
// "FP32 ref; build bf16"): every conv + folded BatchNorm (+ReLU, + identity-add+ReLU) of
// features/resnet_features.py:77-229 is one launch of this kernel.
//
// Same "TN" product and tile machinery as the fp32 kernel (gemm_f32_impl.hpp), byte for
// byte: an LDS row is 128 B (BK = 64 bf16 = 8 16-B chunks, chunk index XOR-swizzled by
// (row>>1)&7 at the DMA source, undone on the read), global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, 16 B = 8 channels per lane).  For 32x32x16 bf16 lane l supplies
// A[l&31][k = 8(l>>5) + j] and B[k][l&31], j = 0..7 -- one ds_read_b128 per operand; the
// k order inside a tile is free, so half-wave h reads chunks 4h .. 4h+3 (one MFMA k-step
// per chunk pair), exactly the fp32 kernel's access pattern.
//
// K is padded to a multiple of 64 at pack time (zero weight rows); the A loader returns
// the zero chunk for k >= Kv (the valid K) and for taps in the convolution's padding, so
// one kernel covers the 7x7x8 stem (K 392 -> 448) as well as 1x1 and 3x3 convs.
// Requires Cin % 8 == 0 (a 16-B chunk never straddles two taps).
#pragma once
#include "common.hpp"

namespace pipnet_bf16 {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Epilogue element math shared by the bf16 tiles (bitwise the element-wise forms they replace):
// * add_bf16x8: the residual's 8 bf16 widened exactly to fp32 (a shift / mask per element) as two
//   float4, so the adds issue as v_pk_add_f32 (one per 2 elements) instead of per-element v_add_f32;
// * to_bf16x8: RNE to bf16 (v_cvt_pk_bf16_f32), then ReLU as v_pk_max_i16 against 0 on the packed
//   pairs -- a bf16's bits order like an int16 (sign first), so max(bits, 0) zeroes exactly the
//   negative values (-0 included) and keeps the rest: RNE(max(x, 0)) for every non-NaN x in one
//   instruction per 2 elements instead of a v_max_f32 per element.  NaNs: a positive-sign NaN stays
//   NaN (as torch.relu keeps it), a NEGATIVE-sign NaN (e.g. 0xFFC0) is a negative int16 and becomes
//   +0 -- the one input class where this differs from torch.relu.
PIPNET_DEV void add_bf16x8(f32x4& x0, f32x4& x1, const bf16x8& r) {
  const u32x4 u = __builtin_bit_cast(u32x4, r);
  const u32x4 ev = u << 16, od = u & 0xffff0000u;   // elements 2j (low half) / 2j + 1 (high half)
  x0 += f32x4{__uint_as_float(ev[0]), __uint_as_float(od[0]), __uint_as_float(ev[1]), __uint_as_float(od[1])};
  x1 += f32x4{__uint_as_float(ev[2]), __uint_as_float(od[2]), __uint_as_float(ev[3]), __uint_as_float(od[3])};
}
template <bool RELU>
PIPNET_DEV unsigned bf16_pair(float a, float b) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  typedef short i16x2 __attribute__((ext_vector_type(2)));
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  i16x2 v = __builtin_bit_cast(i16x2, __builtin_convertvector((f32x2){a, b}, bf16x2));
  if constexpr (RELU) v = __builtin_elementwise_max(v, (i16x2)0);
  return __builtin_bit_cast(unsigned, v);
}
template <bool RELU>
PIPNET_DEV bf16x8 to_bf16x8(const f32x4& x0, const f32x4& x1) {
  return __builtin_bit_cast(bf16x8, u32x4{bf16_pair<RELU>(x0[0], x0[1]), bf16_pair<RELU>(x0[2], x0[3]),
                                          bf16_pair<RELU>(x1[0], x1[1]), bf16_pair<RELU>(x1[2], x1[3])});
}

constexpr int KPAD = 64;                      // packed weights: K rounded up to this

struct ConvParams {
  const bf16* A;
  int64_t lda;         // dense rows (1x1 stride-1 convs): row pitch in elements
  const bf16* W;       // [N][K] (K padded to 64, zero beyond Kv)
  const float* bias;   // [N] fp32 (folded BatchNorm shift), may be null
  const bf16* R;       // residual [M][ldr] bf16 (EPI_BIAS_RESID_RELU)
  int64_t ldr;
  bf16* C;
  int64_t ldc;
  const float* scale;  // [N] layer scale (EPI_F32_RESID)
  const float* R32;    // fp32 residual [M][ldr] (EPI_F32_RESID), may alias Cf
  float* Cf;           // fp32 output [M][ldc] (EPI_F32_BIAS / EPI_F32_RESID)
  bf16* C2;            // EPI_DUAL_BIAS_RELU: columns >= nsplit go here (relu), [M][ldc2]
  int64_t ldc2;
  int nsplit;
  int M, N, K, Kv;
  int H, Wd, Cin, OH, OW, stride, KW, pad;
  int Cinp;            // physical channels per pixel of A (= Cin, or 2 seg for split planes)
  int seg;             // split planes [hi | lo] of seg channels read as K' = [hi | lo | hi]: a
                       // (virtual) channel c >= 2 seg is read at c - 2 seg; 0 = no remap
  int mt, nt, group_m;
};

enum { ALOAD_DENSE = 0, ALOAD_CONV = 2 };

// virtual split-plane channel -> physical (K-tiles never straddle a segment: seg % 32 == 0)
PIPNET_DEV int seg_remap(const ConvParams& p, int c) { return (p.seg && c >= 2 * p.seg) ? c - 2 * p.seg : c; }

static __device__ const __attribute__((aligned(16))) float g_zero_bf[4] = {0.f, 0.f, 0.f, 0.f};

struct ARow {
  int64_t base;
  int iy0, ix0;
};

template <int ALOAD>
PIPNET_DEV ARow a_row(const ConvParams& p, int m) {
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
  r.base = (int64_t)b * p.H * p.Wd * p.Cinp;
  r.iy0 = oy * p.stride - p.pad;
  r.ix0 = ox * p.stride - p.pad;
  return r;
}

// Address of A[m][k .. k+7] (8 channels of one tap), or of the zero chunk.
template <int ALOAD>
PIPNET_DEV const void* a_ptr(const ConvParams& p, const ARow& r, int k) {
  if (k >= p.Kv) return g_zero_bf;   // K padding (packed weights are zero there too)
  if (ALOAD == ALOAD_DENSE) return p.A + r.base + seg_remap(p, k);
  const int tap = k / p.Cin;
  const int c = k - tap * p.Cin;
  const int ky = tap / p.KW;
  const int iy = r.iy0 + ky;
  const int ix = r.ix0 + tap - ky * p.KW;
  if ((unsigned)iy >= (unsigned)p.H || (unsigned)ix >= (unsigned)p.Wd) return g_zero_bf;
  return p.A + r.base + ((int64_t)iy * p.Wd + ix) * p.Cinp + seg_remap(p, c);
}

// Workgroup tile: WGM x WGN waves, each wave TM x TN MFMA 32x32 tiles, BK-deep K tiles in NS
// LDS stages.  BK = 64: 128-B rows, 8 chunks, chunk ^= (row>>1)&7; BK = 32: 64-B rows, 4
// chunks, chunk ^= (row>>2)&3 -- either way the 16 lanes of a ds_read_b128 group hit 16
// distinct 16-B bank slots.
//   <2,2,2,2,64,2> 128x128, <2,2,1,2,64,2> 64x128, <2,4,4,2,64,2> 256x256 (512 threads),
//   <2,4,4,2,32,4> 256x256 with 3 K-tiles in flight across the barriers.
template <int WGM_, int WGN_, int TM_, int TN_, int BK_ = 64, int NS_ = 2>
struct Cfg {
  static constexpr int WGM = WGM_, WGN = WGN_, TM = TM_, TN = TN_, BK = BK_, NS = NS_;
  static constexpr int NWAVES = WGM * WGN, NTHREADS = 64 * NWAVES;
  static constexpr int BMT = WGM * 32 * TM, BNT = WGN * 32 * TN;
  static constexpr int CHUNKS = BK / 8, ROWS_PER_DMA = 64 / CHUNKS;
  static constexpr int NGROUPS = CHUNKS / 2;            // chunk groups per half-wave per tile
  static constexpr int A_DMA = BMT / ROWS_PER_DMA / NWAVES;
  static constexpr int B_DMA = BNT / ROWS_PER_DMA / NWAVES;
  static constexpr int TILE_ELEMS = (BMT + BNT) * BK;   // bf16 elements of one stage
  static_assert(BK == 32 || BK == 64, "BK");
  static_assert(KPAD % BK == 0, "packed K must be a multiple of BK");
  static_assert(A_DMA * ROWS_PER_DMA * NWAVES == BMT && B_DMA * ROWS_PER_DMA * NWAVES == BNT, "DMA split");
  static PIPNET_DEV int swz(int row, int c) { return BK == 64 ? (c ^ ((row >> 1) & 7)) : (c ^ ((row >> 2) & 3)); }
};

template <class C>
struct Frag {
  bf16x8 a[C::TM], b[C::TN];
};
template <class C>
using Acc = f32x16[C::TM][C::TN];

template <class C>
PIPNET_DEV void read_frag(Frag<C>& f, const bf16* buf, int wm, int wn, int lr, int lh, int q) {
  constexpr int BK = C::BK;
  const int c = lh * C::NGROUPS + q;
#pragma unroll
  for (int i = 0; i < C::TM; ++i) {
    const int ra = wm * 32 * C::TM + i * 32 + lr;
    f.a[i] = *reinterpret_cast<const bf16x8*>(buf + ra * BK + 8 * C::swz(ra, c));
  }
#pragma unroll
  for (int j = 0; j < C::TN; ++j) {
    const int rb = wn * 32 * C::TN + j * 32 + lr;
    f.b[j] = *reinterpret_cast<const bf16x8*>(buf + C::BMT * BK + rb * BK + 8 * C::swz(rb, c));
  }
}

// JL = the wave's active 32-column blocks (TN except NPAD waves whose blocks lie past N),
// a compile-time count so the MFMA stream stays branch-free.
template <class C, int JL = C::TN>
PIPNET_DEV void mfma_frag(Acc<C>& acc, const Frag<C>& f) {
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < JL; ++j)
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
}

template <int V>
struct IntC {
  static constexpr int value = V;
};

PIPNET_DEV void dma16(const void* src, bf16* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// Retire all but the NPEND youngest vector-memory ops of this wave (LDS-DMA counts as VMEM),
// drain this wave's LDS reads, then the workgroup barrier -- one asm block, so the LDS-DMA of
// later tiles stays in flight across it (a __syncthreads() would emit vmcnt(0)).
template <int NPEND>
PIPNET_DEV void wait_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(NPEND) : "memory");
}

PIPNET_DEV void tile_coords(const ConvParams& p, int bm, int bn, int& m0, int& n0) {
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

PIPNET_DEV u32x4 as_u32x4(const bf16x8& v) { return __builtin_bit_cast(u32x4, v); }

// Epilogues of the split-bf16 ConvNeXt path (include/pipnet_amd.h, pipnet_conv2d_nhwc_s3):
// x0 / x1 = accumulator + bias of channels n .. n+7 of row m.  S3_GELU writes GELU's output
// as the next GEMM's A operand, split planes [hi | lo] (row pitch ldc = 2N); F32_BIAS /
// F32_RESID write fp32 (the residual stream and the downsample outputs stay fp32).
template <int EPI>
PIPNET_DEV void finish_s3(const ConvParams& p, int m, int n, f32x4 x0, f32x4 x1, f32x4 s0, f32x4 s1) {
  if constexpr (EPI == PIPNET_EPI_S3_GELU) {
    const f32x2 g0 = gelu_pk16(f32x2{x0[0], x0[1]}), g1 = gelu_pk16(f32x2{x0[2], x0[3]});
    const f32x2 g2 = gelu_pk16(f32x2{x1[0], x1[1]}), g3 = gelu_pk16(f32x2{x1[2], x1[3]});
    const float g[8] = {g0[0], g0[1], g1[0], g1[1], g2[0], g2[1], g3[0], g3[1]};
    bf16x8 hi, lo;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bf16 h, l;
      split_bf16(g[e], h, l);
      hi[e] = h;
      lo[e] = l;
    }
    bf16* dst = p.C + (int64_t)m * p.ldc + n;
    *reinterpret_cast<bf16x8*>(dst) = hi;
    *reinterpret_cast<bf16x8*>(dst + p.N) = lo;
  } else {
    if constexpr (EPI == PIPNET_EPI_F32_RESID) {
      const float* r = p.R32 + (int64_t)m * p.ldr + n;
      x0 = ld4(r) + s0 * x0;
      x1 = ld4(r + 4) + s1 * x1;
    }
    float* dst = p.Cf + (int64_t)m * p.ldc + n;
    st4(dst, x0);
    st4(dst + 4, x1);
  }
}

// Epilogue: each wave re-lays its 32 x (TN*32) fp32 accumulator slice through LDS (rows
// padded by 4 floats: the 16-B reads of one row's lanes then cover all 64 banks), then every
// lane finishes 8 consecutive channels of one pixel -- bias, residual (one 16-B bf16
// load, all issued before the first store), ReLU, round-to-nearest-even to bf16
// (v_cvt_pk_bf16_f32), one 16-B store.  Needs N % 8 == 0 and 16-B aligned C / R rows.
template <int EPI, class C>
PIPNET_DEV void epilogue(const ConvParams& p, const Acc<C>& acc, float* smem, int m0, int n0, int wm, int wn,
                         int lane, int wid) {
  constexpr int TM = C::TM, TN = C::TN, LD = TN * 32 + 4;
  constexpr bool HAS_R = EPI == PIPNET_EPI_BIAS_RESID_RELU;
  // a lane finishes 8 channels; CPR lanes cover one row of the wave's TN*32 columns
  constexpr int CPR = TN * 4, RPI = 64 / CPR, NIT = 32 / RPI;
  float* wt = smem + wid * 32 * LD;
  const int lr = lane & 31, lh = lane >> 5;
  const int c8 = lane % CPR;
  const int n = n0 + wn * 32 * TN + 8 * c8;
  const bool nok = n < p.N;
  f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0, s0 = b0, s1 = b0;
  if (EPI != PIPNET_EPI_NONE && p.bias && nok) {
    b0 = ld4(p.bias + n);
    b1 = ld4(p.bias + n + 4);
  }
  if (EPI == PIPNET_EPI_F32_RESID && nok) {
    s0 = ld4(p.scale + n);
    s1 = ld4(p.scale + n + 4);
  }
  bf16x8 r[TM][NIT];
  if (HAS_R) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int m = min(m0 + wm * 32 * TM + i * 32 + it * RPI + lane / CPR, p.M - 1);
        if (nok) r[i][it] = *reinterpret_cast<const bf16x8*>(p.R + (int64_t)m * p.ldr + n);
      }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) wt[((v & 3) + 8 * (v >> 2) + 4 * lh) * LD + j * 32 + lr] = acc[i][j][v];
    __syncthreads();
    if (i == 0) vm_drain();                      // bias / residual preloads landed (common.hpp)
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int row = it * RPI + lane / CPR;
      const int m = m0 + wm * 32 * TM + i * 32 + row;
      f32x4 x0 = ld4(wt + row * LD + 8 * c8), x1 = ld4(wt + row * LD + 8 * c8 + 4);
      x0 += b0;
      x1 += b1;
      if constexpr (EPI >= PIPNET_EPI_S3_GELU) {
        if (m < p.M && nok) finish_s3<EPI>(p, m, n, x0, x1, s0, s1);
        continue;
      }
      if (HAS_R) add_bf16x8(x0, x1, r[i][it]);
      const bf16x8 o = to_bf16x8<EPI == PIPNET_EPI_BIAS_RELU || EPI == PIPNET_EPI_BIAS_RESID_RELU>(x0, x1);
      if (m < p.M && nok) *reinterpret_cast<bf16x8*>(p.C + (int64_t)m * p.ldc + n) = o;
    }
  }
}

// NS LDS stages (tile k+NS-1 in flight while tile k is multiplied), one barrier per K tile,
// fragments software-pipelined over the tile's chunk groups (group q of half-wave h = chunk
// h*NGROUPS + q = k 8(h*NGROUPS + q) .. +7 of the tile).  NS = 2 waits with vmcnt(0); NS >= 3
// with a counted vmcnt and a raw s_barrier so younger tiles' DMA spans the barrier.
// NPAD (N % BNT != 0, two wave columns): MFMA blocks of columns >= N are skipped and the
// wave -> column-half map flips with the workgroup parity (as the fp32 GEMM's NPAD tiles).
template <class C, int EPI, int ALOAD, int MINB, bool NPAD = false>
__global__ __launch_bounds__(C::NTHREADS, MINB) void conv_bf16_kernel(ConvParams p) {
  constexpr int NS = C::NS, BK = C::BK;
  constexpr int NWAVES = C::NWAVES;
  constexpr int DMA_PER_TILE = C::A_DMA + C::B_DMA;    // per wave
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * C::TILE_ELEMS];
  static_assert(NS * C::TILE_ELEMS * 2 >= NWAVES * 32 * (C::TN * 32 + 4) * 4, "epilogue LDS");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  static_assert(!NPAD || C::WGN == 2, "NPAD flips between two wave columns");
  const int wm = wid / C::WGN, wn = NPAD ? ((wid % C::WGN) ^ (int)(blockIdx.x & 1)) : wid % C::WGN;
  const int lr = lane & 31, lh = lane >> 5;
  int m0, n0;
  tile_coords(p, C::BMT, C::BNT, m0, n0);
  const int nk = p.K / BK;
  const int jl = NPAD ? __builtin_amdgcn_readfirstlane(min(C::TN, max(0, (p.N - n0 - wn * 32 * C::TN + 31) >> 5)))
                      : C::TN;

  const int drow = lane / C::CHUNKS;
  ARow arow[C::A_DMA];
  int achunk[C::A_DMA];
  const bf16* wsrc[C::B_DMA];
#pragma unroll
  for (int i = 0; i < C::A_DMA; ++i) {
    const int row = (i * NWAVES + wid) * C::ROWS_PER_DMA + drow;
    achunk[i] = 8 * C::swz(row, lane % C::CHUNKS);
    arow[i] = a_row<ALOAD>(p, min(m0 + row, p.M - 1));
  }
#pragma unroll
  for (int i = 0; i < C::B_DMA; ++i) {
    const int row = (i * NWAVES + wid) * C::ROWS_PER_DMA + drow;
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + 8 * C::swz(row, lane % C::CHUNKS);
  }
  auto stage = [&](int kt, int buf) {
    bf16* base = smem + buf * C::TILE_ELEMS;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < C::A_DMA; ++i)
      dma16(a_ptr<ALOAD>(p, arow[i], k0 + achunk[i]), base + (i * NWAVES + wid) * C::ROWS_PER_DMA * BK);
#pragma unroll
    for (int i = 0; i < C::B_DMA; ++i)
      dma16(wsrc[i] + k0, base + C::BMT * BK + (i * NWAVES + wid) * C::ROWS_PER_DMA * BK);
  };
  // barrier once tile `need` has landed; `last` = youngest tile whose DMA is in flight
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

  Acc<C> acc;
#pragma unroll
  for (int i = 0; i < C::TM; ++i)
#pragma unroll
    for (int j = 0; j < C::TN; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  int issued = -1;
  for (int s0 = 0; s0 < NS - 1 && s0 < nk; ++s0) stage(s0, s0), issued = s0;
  wait_tile(0, issued);
  auto main_loop = [&](auto jlc) {
    constexpr int JL = decltype(jlc)::value;
    Frag<C> fa, fb;
    read_frag<C>(fa, smem, wm, wn, lr, lh, 0);
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bf16* buf = smem + cur * C::TILE_ELEMS;
      if (kt + NS - 1 < nk) {
        int nb = cur + NS - 1;
        if (nb >= NS) nb -= NS;
        stage(kt + NS - 1, nb);
        issued = kt + NS - 1;
      }
      if constexpr (C::NGROUPS == 4) {
        read_frag<C>(fb, buf, wm, wn, lr, lh, 1);
        mfma_frag<C, JL>(acc, fa);
        read_frag<C>(fa, buf, wm, wn, lr, lh, 2);
        mfma_frag<C, JL>(acc, fb);
        read_frag<C>(fb, buf, wm, wn, lr, lh, 3);
        mfma_frag<C, JL>(acc, fa);
      } else {
        read_frag<C>(fb, buf, wm, wn, lr, lh, 1);
        mfma_frag<C, JL>(acc, fa);
      }
      const int nxt = (cur + 1 == NS) ? 0 : cur + 1;
      wait_tile(kt + 1 < nk ? kt + 1 : issued, issued);     // tile kt+1 landed, tile kt read
      if (kt + 1 < nk) read_frag<C>(fa, smem + nxt * C::TILE_ELEMS, wm, wn, lr, lh, 0);
      mfma_frag<C, JL>(acc, fb);
      cur = nxt;
    }
  };
  if constexpr (NPAD) {
    static_assert(C::TN == 2, "NPAD dispatch covers TN = 2");
    if (jl >= 2) main_loop(IntC<2>{});
    else if (jl == 1) main_loop(IntC<1>{});
    else main_loop(IntC<0>{});
  } else {
    main_loop(IntC<C::TN>{});
  }
  epilogue<EPI, C>(p, acc, reinterpret_cast<float*>(smem), m0, n0, wm, wn, lane, wid);
}

// ======================================================================================
// Ping-pong 256x256 tile on v_mfma_f32_16x16x32_bf16 (cdna_hip_programming.md "256^2
// 8-phase template" structure, re-derived for 32-deep K tiles in 4 LDS stages).
//
// 8 waves = 2 groups (wr = wid >> 2) x 4 column blocks (wc); wave (wr, wc) owns the 128x64
// output block rows wr*128.., cols wc*64.. as 8 x 4 MFMA 16x16 tiles.  A K-tile (32 deep, one
// MFMA k-step) is two PHASES of 16 MFMAs (row half 0 / 1 of the wave's block), each phase
//     [ds_read fragments of this phase] [LDS-DMA] s_barrier | MFMA x16 (prio 1) | s_barrier
// and group 1 runs one barrier behind group 0 (one extra s_barrier before the loop), so on
// every SIMD one wave's MFMA segment coincides with its partner's read / DMA / barrier
// segment and the matrix pipe alternates between the two instead of both stalling together.
//
// LDS: 4 stages x (256 A rows + 256 B rows) x 64 B.  Each phase issues 2 x 1 KiB LDS-DMA
// pieces per wave: B of K-tile t+2 in phase 0 of K-tile t (into the stage of t-2, read by
// everyone long before), A of K-tile t+3 in phase 1 (into the stage of t-1: every wave
// retired its reads of t-1 -- compiler lgkmcnt before the MFMAs of the phase that read
// them -- before the barrier this DMA issue follows, for both groups).  Each wave waits for
// its own pieces of K-tile t+1 (vmcnt counting the 6 / 4 / 0 younger pieces) before the
// first barrier of phase 1 of K-tile t; group 0 reads t+1 after its next barrier, group 1
// one barrier later -- both after every wave's wait.
//
// Rows are 64 B (4 x 16-B chunks); chunk c of row r lives at physical chunk c ^ g(r),
// g(r) = (-(r >> 2)) & 3: with the 16x16x32 operand map (lane l reads row l & 15, chunk
// l >> 4) every ds_read_b128 lane group of 16 hits 16 distinct 16-B bank slots.  The DMA
// writes lane-linear, so the swizzle is applied to its source address.
// Requirements: Cin % 32 == 0 (a K-tile never straddles two taps), N % 8 == 0, K % 32 == 0.
// ======================================================================================
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));


namespace pp {
constexpr int BM = 256, BN = 256, BK = 32, NT = 512;
constexpr int ROWB = BK * 2;                          // 64 B per LDS row
constexpr int STAGE_BYTES = (BM + BN) * ROWB;         // 32 KiB
constexpr int EPI_LD = 68;                            // fp32 epilogue rows: 64 + 4 pad
constexpr int EPI_BYTES = 8 * 64 * EPI_LD * 4;        // 8 waves x 64 rows
// DB = prefetch distance of B in K-tiles (A: DB + 1), NS = DB + 2 LDS stages of 32 KiB
template <int DB>
constexpr int smem_bytes() { return (DB + 2) * STAGE_BYTES > EPI_BYTES ? (DB + 2) * STAGE_BYTES : EPI_BYTES; }
PIPNET_DEV int g(int r) { return (-(r >> 2)) & 3; }
}  // namespace pp

template <int NPEND>
PIPNET_DEV void pp_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPEND) : "memory");
}
// runtime (wave-uniform) count -> immediate: the counts are <= 4 DB - 2 (odd ones from the
// one-A-piece waves of 224-row persistent tiles)
PIPNET_DEV void pp_wait_vm_dyn(int n) {
  switch (n) {
    case 0: pp_wait_vm<0>(); break;
    case 1: pp_wait_vm<1>(); break;
    case 3: pp_wait_vm<3>(); break;
    case 5: pp_wait_vm<5>(); break;
    case 2: pp_wait_vm<2>(); break;
    case 4: pp_wait_vm<4>(); break;
    case 6: pp_wait_vm<6>(); break;
    case 8: pp_wait_vm<8>(); break;
    case 10: pp_wait_vm<10>(); break;
    default: pp_wait_vm<0>(); break;
  }
}
PIPNET_DEV void pp_barrier() {
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// ds_read_b128 the compiler does not track (its waitcnt pass sees the value as ready at issue):
// the caller waits with lgkm_wait_dyn before the first use
PIPNET_DEV bf16x8v ds_read_b128_asm(const unsigned char* p) {
  bf16x8v v;
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int N>
PIPNET_DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
PIPNET_DEV void lgkm_wait_dyn(int n) {        // n compile-time after unrolling
  switch (n) {
    case 0: lgkm_wait<0>(); break;
    case 1: lgkm_wait<1>(); break;
    case 2: lgkm_wait<2>(); break;
    default: lgkm_wait<3>(); break;
  }
}

// MFMA-segment schedule of the 256-row ping-pong tiles (halo 8, pp 5, persistent 9): 2 = two
// 16-MFMA phases per 32-deep K-tile, each between a barrier pair (rounds 2-5); 3 = ONE 32-MFMA
// segment per K-tile with the row-half-1 A reads interleaved as untracked (inline-asm) reads and
// per-row lgkmcnt waits (round 6; profiles/r06/halo_seg_lab.txt).  Bitwise the same results: every
// accumulator sees the same MFMA chain.  Build-time knobs for tools/ab_build.py A/B arms.
#ifndef PIPNET_HALO_SEG
#define PIPNET_HALO_SEG 3
#endif
#ifndef PIPNET_PP_SEG
#define PIPNET_PP_SEG 3
#endif
#ifndef PIPNET_PPP_SEG
#define PIPNET_PPP_SEG 3
#endif
// Matrix-segment priority of the SEG 3 schedules: 1 = s_setprio 1 around every M segment (the
// product), 0 = none, 2 = one static s_setprio 1 for the younger half (waves 4-7) before the loop
#ifndef PIPNET_BF16_PRIO
#define PIPNET_BF16_PRIO 1
#endif
PIPNET_DEV void seg_prio(int on) {
  if constexpr (PIPNET_BF16_PRIO == 1) {
    if (on) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
  }
}
PIPNET_DEV void static_prio() {
  if constexpr (PIPNET_BF16_PRIO == 2) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
}

// The SEG = 3 M segment: half 0's 4 x NB MFMAs, each row followed by the untracked read of the
// half-1 fragment that reuses its registers, then half 1's (RB - 4) x NB MFMAs, each row after a
// wait for its own read (LDS returns in order).  `rd(r)` returns half-1 row r's fragment through
// ds_read_b128_asm.
template <int RB, int NB, typename RD>
PIPNET_DEV void pp_mseg3(f32x4v (&acc)[8][NB], bf16x8v (&fa)[4], const bf16x8v* fb, RD&& rd) {
  seg_prio(1);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
    if (r < RB - 4) {
      __builtin_amdgcn_sched_barrier(0);
      fa[r] = rd(r);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int r = 0; r < RB - 4; ++r) {
    __builtin_amdgcn_sched_barrier(0);
    lgkm_wait_dyn(RB - 5 - r);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NB; ++n)
      acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
  }
  seg_prio(0);
}

// Epilogue of the 256-row ping-pong tiles: per row half, the wave's fp32 accumulators are
// re-laid through its own LDS rows (64 x 68 floats), then every lane finishes 8 consecutive
// channels of one pixel (bias, residual, ReLU or the split-bf16 forms) with 16-B accesses.
// The stage buffers must be free (all waves past the main loop's last barrier).
// RB = 16-row blocks per wave group (8: 256-row tiles; 7: 224-row tiles, see conv_bf16.hip
// pick_rb): half 0 holds blocks 0..3, half 1 blocks 4..RB-1.
template <int EPI, int NB, int RB = 8>
PIPNET_DEV void pp_epilogue(const ConvParams& p, const f32x4v (&acc)[8][NB], unsigned char* smem, int m0, int n0,
                            int wr, int wc, int lane, int wid) {
  using namespace pp;
  static_assert(RB == 7 || RB == 8, "RB");
  constexpr int WCOLS = 16 * NB;
  const int mw = m0 + wr * 16 * RB;              // first row of this wave group
  const int fr = lane & 15;
  constexpr bool HAS_R = EPI == PIPNET_EPI_BIAS_RESID_RELU;
  float* wt = reinterpret_cast<float*>(smem) + wid * 64 * EPI_LD;
  const int c8 = lane & 7;
  const int n = n0 + wc * WCOLS + 8 * c8;
  const bool nok = c8 < 2 * NB && n < p.N;
  f32x4v b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0, s0 = b0, s1 = b0;
  if (EPI != PIPNET_EPI_NONE && p.bias && nok) {
    b0 = *reinterpret_cast<const f32x4v*>(p.bias + n);
    b1 = *reinterpret_cast<const f32x4v*>(p.bias + n + 4);
  }
  if (EPI == PIPNET_EPI_F32_RESID && nok) {
    s0 = *reinterpret_cast<const f32x4v*>(p.scale + n);
    s1 = *reinterpret_cast<const f32x4v*>(p.scale + n + 4);
  }
  // residual rows of both halves requested up front: one HBM latency per tile, not two
  // running row pointers (+8 rows per step): no per-access 64-bit multiply (ppp epilogue note)
  const int mrow0 = mw + (lane >> 3);
  bf16x8v rrs[2][8];
  if (HAS_R) {
    const bf16* rp = p.R + (int64_t)mrow0 * p.ldr + n;
    const bf16* const rlast = p.R + (int64_t)(p.M - 1) * p.ldr + n;
#pragma unroll
    for (int half = 0; half < 2; ++half)
#pragma unroll
      for (int it = 0; it < 2 * (half ? RB - 4 : 4); ++it) {
        const bf16* src = mrow0 + half * 64 + it * 8 < p.M ? rp : rlast;
        if (nok) rrs[half][it] = *reinterpret_cast<const bf16x8v*>(src);
        rp += 8 * p.ldr;
      }
  }
  bf16* op = p.C + (int64_t)mrow0 * p.ldc + n;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const int nr = half ? RB - 4 : 4;            // row blocks of this half (compile-time after unrolling)
    bf16x8v (&rr)[8] = rrs[half];
#pragma unroll
    for (int r = 0; r < nr; ++r)
#pragma unroll
      for (int nn = 0; nn < NB; ++nn)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          wt[(r * 16 + 4 * (lane >> 4) + i) * EPI_LD + nn * 16 + fr] = acc[half * 4 + r][nn][i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (half == 0) vm_drain();                   // bias / residual preloads landed (common.hpp)
#pragma unroll
    for (int it = 0; it < 2 * nr; ++it) {
      const int row = it * 8 + (lane >> 3);
      const int m = mw + half * 64 + row;
      f32x4v x0 = *reinterpret_cast<const f32x4v*>(wt + row * EPI_LD + 8 * c8);
      f32x4v x1 = *reinterpret_cast<const f32x4v*>(wt + row * EPI_LD + 8 * c8 + 4);
      x0 += b0;
      x1 += b1;
      if constexpr (EPI >= PIPNET_EPI_S3_GELU) {
        if (m < p.M && nok) finish_s3<EPI>(p, m, n, x0, x1, s0, s1);
        continue;
      }
      if (HAS_R) add_bf16x8(x0, x1, rr[it]);
      const bf16x8v o = to_bf16x8<EPI == PIPNET_EPI_BIAS_RELU || EPI == PIPNET_EPI_BIAS_RESID_RELU>(x0, x1);
      if (m < p.M && nok) *reinterpret_cast<bf16x8v*>(op) = o;
      op += 8 * p.ldc;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // reads done before the next half's writes
  }
}

// NB = B fragments (16 columns each) per wave: 4 -> 256-wide tiles, 3 -> 192-wide (N = 384 /
// 192 layers: two 192-wide tiles instead of a full and a half-empty 256-wide one).  The DMA
// and LDS layout stay those of the 256-wide tile (rows 192..255 are fetched and unused), so
// the vmcnt accounting is identical.
// ABL (tuning lab only, tools/bf16_lab.hip; 0 in the product): 1 = no LDS-DMA (stale LDS, no
// vmcnt waits), 2 = no epilogue (one store per lane keeps the accumulators live), 4 = no
// barriers, 8 = no fragment reads after the first (stale registers).
template <int EPI, int ALOAD, int NB = 4, int ABL = 0, int DB = 2>
__global__ __launch_bounds__(pp::NT, 1) void conv_bf16_pp_kernel(ConvParams p) {
  using namespace pp;
  constexpr int NS = DB + 2;
  static_assert(DB >= 2 && DB <= 3, "DB");
  __shared__ __attribute__((aligned(16))) unsigned char smem[smem_bytes<DB>()];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  static_assert(NB == 3 || NB == 4, "NB");
  constexpr int WCOLS = 16 * NB;                               // output columns per wave
  tile_coords(p, BM, 4 * WCOLS, m0, n0);
  const int nk = p.K / BK;

  // ---- DMA sources: pieces wid and wid + 8 of A and of B (16 rows x 64 B each) ----
  const int drow = lane >> 2;                                  // row within a piece
  const int dchunk = 8 * ((lane & 3) ^ g(drow));               // logical chunk (elements)
  ARow ar[2];
  const bf16* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (wid + 8 * i) + drow;
    ar[i] = a_row<ALOAD>(p, min(m0 + row, p.M - 1));
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + dchunk;
  }
  // (tap, channel) of the K-tile the DMA fetches next, advanced incrementally (a 32-deep
  // K-tile never straddles a tap: Cin % 32 == 0), so no division in the loop.
  int d_c = 0, d_kx = 0, d_ky = 0;
  // K-tiles past the valid K (K padded to 64) re-read the last valid one: the packed weights
  // are zero there, so the products are exact zeros (finite activations) and no per-K-tile
  // branch to a zero source is needed.
  auto a_src = [&](const ARow& r, int k0) -> const void* {
    if (ALOAD == ALOAD_DENSE) return p.A + r.base + seg_remap(p, min(k0, p.Kv - BK)) + dchunk;
    const int iy = r.iy0 + d_ky, ix = r.ix0 + d_kx;
    if ((unsigned)iy >= (unsigned)p.H || (unsigned)ix >= (unsigned)p.Wd) return g_zero_bf;
    return p.A + r.base + ((int64_t)iy * p.Wd + ix) * p.Cinp + seg_remap(p, d_c) + dchunk;
  };
  auto advance = [&]() {
    if (ALOAD != ALOAD_DENSE) {
      d_c += BK;
      if (d_c == p.Cin) {
        d_c = 0;
        if (++d_kx == p.KW) d_kx = 0, ++d_ky;
      }
    }
  };
  auto stage_a = [&](int kt) {                                 // 2 x 1 KiB A pieces of this wave
    if constexpr ((ABL & 1) != 0) return;
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)a_src(ar[i], kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + (wid + 8 * i) * 1024), 16,
                                       0, 0);
    advance();
  };
  auto stage_b = [&](int kt) {                                 // 2 x 1 KiB B pieces of this wave
    if constexpr ((ABL & 1) != 0) return;
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + BM * ROWB +
                                                                                 (wid + 8 * i) * 1024),
                                       16, 0, 0);
  };
  // ---- fragment reads: lane reads row (l & 15) of a 16-row block, logical chunk l >> 4 ----
  const int fr = lane & 15;
  const int fofs = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));     // byte offset inside a 16-row block
  auto read_a = [&](bf16x8v (&fa)[4], const unsigned char* st, int half) {
    if constexpr ((ABL & 8) != 0) {
      if (st != smem || half != 0) return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      fa[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 128 + half * 64 + r * 16) * ROWB + fofs);
  };
  auto read_b = [&](bf16x8v (&fb)[4], const unsigned char* st) {
    if constexpr ((ABL & 8) != 0) {
      if (st != smem) return;
    }
#pragma unroll
    for (int n = 0; n < NB; ++n)
      fb[n] = *reinterpret_cast<const bf16x8v*>(st + BM * ROWB + (wc * WCOLS + n * 16) * ROWB + fofs);
  };

  f32x4v acc[8][NB];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};

  // SEG 3 (one 32-MFMA segment per K-tile) fetches A and B of K-tile kt+2 in the R segment of kt;
  // only with the 4-stage ring (DB = 2): the stage of kt+2 was last read in group 1's M segment
  // of kt-2, two segments before group 0's R segment of kt
  constexpr int SEG = (DB == 2 && ABL == 0) ? PIPNET_PP_SEG : 2;
  if constexpr (SEG == 3) {
    stage_a(0), stage_b(0);
    if (1 < nk) stage_a(1), stage_b(1);
    pp_wait_vm_dyn(1 < nk ? 4 : 0);
    pp_barrier();
    if (wr == 1) pp_barrier();                                 // group 1 runs one barrier behind
    static_prio();
    bf16x8v fa[4], fb[4];
    for (int kt = 0; kt < nk; ++kt) {
      const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
      const bool pre = kt + 2 < nk;
      if (pre) stage_a(kt + 2), stage_b(kt + 2);               // DMA before the reads (M0 write)
      read_b(fb, st);
      read_a(fa, st, 0);
      if (pre) pp_wait_vm<4>();                                // A(kt+1), B(kt+1) landed
      else pp_wait_vm<0>();
      pp_barrier();
      pp_mseg3<8, NB>(acc, fa, fb, [&](int r) {
        return ds_read_b128_asm(st + (wr * 128 + 64 + r * 16) * ROWB + fofs);
      });
      pp_barrier();
    }
  } else {
  // pieces (2 per operand tile per wave) issued after B(kt + 1) by the end of phase 1 of K-tile kt:
  // A(j), B(j) for j = kt+2 .. kt+DB and A(kt+DB+1), those that exist
  auto younger_than_b = [&](int kt) {
    int n = 0;
#pragma unroll
    for (int j = 2; j <= DB; ++j) n += (kt + j < nk) ? 4 : 0;
    return n + ((kt + DB + 1 < nk) ? 2 : 0);
  };
  // prologue: A(0) B(0) .. A(DB-1) B(DB-1) A(DB) in flight (B(kt+DB) is fetched in phase 0 of
  // K-tile kt, A(kt+DB+1) in phase 1: two pieces per phase), wait for tile 0
#pragma unroll
  for (int i = 0; i < DB; ++i)
    if (i < nk) stage_a(i), stage_b(i);
  if (DB < nk) stage_a(DB);
  pp_wait_vm_dyn(younger_than_b(-1));
  pp_barrier();
  if (wr == 1) pp_barrier();                                   // group 1 runs one barrier behind

  auto bar = [&]() {
    if constexpr ((ABL & 4) == 0) pp_barrier();
  };
  bf16x8v fa[4], fb[4];
  // One K-tile.  STEADY (every K-tile but the last DB + 1): both DMA pieces exist and the wait
  // count is the constant 4 (DB - 1) + 2 -- no per-K-tile count arithmetic or wait-count
  // switch (that scalar bookkeeping and its branches lengthened every read segment).
  auto ktile = [&](int kt, auto steady) {
    constexpr bool STEADY = decltype(steady)::value;
    const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
    // ---- phase 0: rows 0..63 of the wave's block ----
    if (STEADY || kt + DB < nk) stage_b(kt + DB);              // DMA before the reads (M0 write)
    read_b(fb, st);
    read_a(fa, st, 0);
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
    // ---- phase 1: rows 64..127; fetch A of K-tile kt+3 (DMA first: an M0 write for the DMA
    // would otherwise wait for this phase's fragment reads); wait for K-tile kt+1 ----
    if (STEADY || kt + DB + 1 < nk) stage_a(kt + DB + 1);
    read_a(fa, st, 1);
    // wait for this wave's pieces of K-tile kt+1 (B(kt+1) is its last)
    if constexpr ((ABL & 1) == 0) {
      if constexpr (STEADY) pp_wait_vm<4 * (DB - 1) + 2>();
      else pp_wait_vm_dyn(younger_than_b(kt));
    }
    bar();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar();
  };
  int kt = 0;
  for (; kt < nk - DB - 1; ++kt) ktile(kt, IntC<1>{});
  for (; kt < nk; ++kt) ktile(kt, IntC<0>{});
  }
  if (wr == 0) pp_barrier();                                   // re-align the groups
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pp_barrier();                                                // stage buffers free for the epilogue
  if constexpr ((ABL & 2) != 0) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) t += acc[r][n][i];
    reinterpret_cast<float*>(p.C)[(int64_t)blockIdx.x * pp::NT + tid] = t;
    return;
  }

  pp_epilogue<EPI, NB>(p, acc, smem, m0, n0, wr, wc, lane, wid);
}

// ======================================================================================
// Persistent ping-pong tile for 1x1 (dense) convolutions with N % 256 == 0.
//
// One workgroup per CU walks tiles blockIdx.x, +gridDim.x, ... (the same XCD-grouped raster:
// gridDim.x % 8 == 0 keeps a workgroup's tiles on its XCD's slice).  Between two tiles it
// issues the next tile's first K-tiles (A0 B0 A1 B1 A2, the pp prologue) into the stage
// buffers BEFORE the current tile's epilogue, and the epilogue re-lays the accumulators
// through a separate 32 KiB region (per wave 16 rows x 64 fp32 at a time, XOR-swizzled rows:
// physical column = c ^ (((r >> 2) & 3) << 4 | (r & 1) << 2), conflict-free for the MFMA-layout
// writes and the 8-channel reads).  So the next tile's operand latency, the workgroup launch
// and the store drain of the previous one overlap instead of idling the CU (the pp tile holds
// 139 KiB of LDS: one workgroup per CU, nothing else covers those gaps; short-K layers such
// as the bottleneck conv3 + residual spend a large share of each tile there).
// Counting: every lane issues the same number of epilogue loads / stores (rows past M are
// clamped to row M-1 -- they recompute row M-1's values from the clamped A row, so the
// duplicate store writes identical bits; N % 256 == 0 so every column is valid), which keeps
// the vmcnt waits exact: the next tile's K-tile 0 is retired with vmcnt(6 + stores), and
// its first in-loop wait excludes the epilogue stores as well.
// ======================================================================================
namespace ppp {
constexpr int OFF_EPI = 4 * pp::STAGE_BYTES;          // 128 KiB of stages (DB = 2), then 8 x 4 KiB
constexpr int SMEM = OFF_EPI + 8 * 16 * 64 * 4;
PIPNET_DEV int swz(int r) { return (((r >> 2) & 3) << 4) | ((r & 1) << 2); }
}  // namespace ppp

PIPNET_DEV void tile_coords_id(const ConvParams& p, int id, int bm, int bn, int& m0, int& n0) {
  const int nwg = p.mt * p.nt;
  const int tile = xcd_remap(id, nwg);
  const int gm = p.group_m;
  const int group = tile / (gm * p.nt);
  const int first_m = group * gm;
  const int gsz = min(p.mt - first_m, gm);
  const int in_group = tile - group * gm * p.nt;
  m0 = (first_m + in_group % gsz) * bm;
  n0 = (in_group / gsz) * bn;
}

// RB = 16-row blocks per wave group: 8 -> 256-row tiles, 7 -> 224-row tiles (conv_bf16.hip
// pick_rb: fewer idle CUs in the last round; bitwise the same outputs).  With RB = 7 the A tile
// is 14 DMA pieces of 16 rows: waves 0-5 issue two per K-tile, waves 6-7 one (na), and every
// counted wait uses the wave's own count.
template <int EPI, int RB = 8>
__global__ __launch_bounds__(pp::NT, 1) void conv_bf16_ppp_kernel(ConvParams p) {
  using namespace pp;
  constexpr int DB = 2, NS = 4;
  constexpr int SEG = PIPNET_PPP_SEG;      // 3: A and B of K-tile kt+2 both fetched in kt's R segment
  static_assert(RB == 7 || RB == 8, "RB");
  constexpr int BMR = 32 * RB;                         // tile rows
  constexpr int NSTORE = 2 * RB;                       // epilogue 16-B stores per lane per tile
  constexpr bool HAS_R = EPI == PIPNET_EPI_BIAS_RESID_RELU;
  __shared__ __attribute__((aligned(16))) unsigned char smem[ppp::SMEM];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int nk = p.K / BK;
  const int ntiles = p.mt * p.nt;

  const int drow = lane >> 2;
  const int dchunk = 8 * ((lane & 3) ^ g(drow));
  // A pieces of this wave (wave-uniform): 2, or 1 for waves 6-7 of a 224-row tile
  const int na = __builtin_amdgcn_readfirstlane(wid + 8 < 2 * RB ? 2 : 1);
  int64_t abase[2];
  const bf16* wsrc[2];
  auto setup = [&](int id, int& m0, int& n0) {
    tile_coords_id(p, id, BMR, BN, m0, n0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = 16 * (wid + 8 * i) + drow;
      abase[i] = (int64_t)min(m0 + min(row, BMR - 1), p.M - 1) * p.lda + dchunk;
      wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + dchunk;
    }
  };
  auto stage_a = [&](int kt) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
    const int k0 = seg_remap(p, min(kt * BK, p.Kv - BK));
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p.A + abase[0] + k0),
                                     (__attribute__((address_space(3))) void*)(base + wid * 1024), 16, 0, 0);
    if (RB == 8 || na == 2)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p.A + abase[1] + k0),
                                       (__attribute__((address_space(3))) void*)(base + (wid + 8) * 1024), 16, 0, 0);
  };
  auto stage_b = [&](int kt) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + BM * ROWB +
                                                                                 (wid + 8 * i) * 1024),
                                       16, 0, 0);
  };
  auto prologue_dma = [&]() {
    stage_a(0), stage_b(0);
    if (1 < nk) stage_a(1), stage_b(1);
    if (SEG == 2 && 2 < nk) stage_a(2);
  };
  const int fr = lane & 15;
  const int fofs = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));
  auto read_a = [&](bf16x8v (&fa)[4], const unsigned char* st, int half) {
#pragma unroll
    for (int r = 0; r < (half ? RB - 4 : 4); ++r)
      fa[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 16 * RB + half * 64 + r * 16) * ROWB + fofs);
  };
  auto read_b = [&](bf16x8v (&fb)[4], const unsigned char* st) {
#pragma unroll
    for (int n = 0; n < 4; ++n) fb[n] = *reinterpret_cast<const bf16x8v*>(st + BM * ROWB + (wc * 64 + n * 16) * ROWB + fofs);
  };
  // this wave's pieces issued after its B(kt + 1): A(kt+2), B(kt+2), A(kt+3), those that exist
  // (SEG 3: A(kt+2), B(kt+2) only)
  auto younger_than_b = [&](int kt) {
    return ((kt + 2 < nk) ? 2 + na : 0) + ((SEG == 2 && kt + 3 < nk) ? na : 0);
  };
  // the steady-state wait (2 + 2 na pieces younger than B(kt + 1); SEG 3: 2 + na), as an immediate
  auto wait_steady = [&](auto extra) {
    constexpr int X = decltype(extra)::value;
    if constexpr (SEG == 3) {
      if (RB == 8 || na == 2) pp_wait_vm<4 + X>();
      else pp_wait_vm<3 + X>();
    } else {
      if (RB == 8 || na == 2) pp_wait_vm<6 + X>();
      else pp_wait_vm<4 + X>();
    }
  };

  int m0, n0;
  int id = blockIdx.x;
  setup(id, m0, n0);
  prologue_dma();
  pp_wait_vm_dyn(younger_than_b(-1));
  pp_barrier();
  int extra = 0;                       // epilogue stores younger than this tile's first B(1)
  if constexpr (SEG == 3) static_prio();
  for (;;) {
    if (wr == 1) pp_barrier();         // group 1 runs one barrier behind
    f32x4v acc[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};
    bf16x8v fa[4], fb[4];
    // SEG 3: R segment (DMA of kt+2, B + half-0 A reads, counted wait) | one 32-MFMA M segment
    auto rd1 = [&](const unsigned char* st) {
      return [=](int r) { return ds_read_b128_asm(st + (wr * 16 * RB + 64 + r * 16) * ROWB + fofs); };
    };
    auto ktile3 = [&](int kt, auto steady, auto xstore) {
      constexpr bool STEADY = decltype(steady)::value;
      const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
      if (STEADY || kt + 2 < nk) stage_a(kt + 2), stage_b(kt + 2);
      read_b(fb, st);
      read_a(fa, st, 0);
      if constexpr (STEADY) wait_steady(xstore);
      else pp_wait_vm_dyn(younger_than_b(kt));
      pp_barrier();
      pp_mseg3<RB, 4>(acc, fa, fb, rd1(st));
      pp_barrier();
    };
    auto ktile = [&](int kt, auto steady) {
      constexpr bool STEADY = decltype(steady)::value;
      const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
      if (STEADY || kt + DB < nk) stage_b(kt + DB);
      read_b(fb, st);
      read_a(fa, st, 0);
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
      if (STEADY || kt + DB + 1 < nk) stage_a(kt + DB + 1);
      read_a(fa, st, 1);
      if constexpr (STEADY) wait_steady(IntC<0>{});
      else pp_wait_vm_dyn(younger_than_b(kt));
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < RB - 4; ++r)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
    };
    int kt = 0;
    if constexpr (SEG == 3) {
      if (extra && nk > 2) {           // first K-tile after a tile switch: the previous epilogue's
        ktile3(0, IntC<1>{}, IntC<NSTORE>{});   // stores sit between B(1) and A(2) B(2)
        kt = 1;
      }
      for (; kt < nk - 2; ++kt) ktile3(kt, IntC<1>{}, IntC<0>{});
      for (; kt < nk; ++kt) ktile3(kt, IntC<0>{}, IntC<0>{});
    } else {
    if (extra && nk > DB + 1) {        // first K-tile after a tile switch: the stores of the
      const unsigned char* st = smem;  // previous epilogue sit between A(2) and B(2)
      stage_b(DB);
      read_b(fb, st);
      read_a(fa, st, 0);
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
      stage_a(DB + 1);
      read_a(fa, st, 1);
      wait_steady(IntC<NSTORE>{});
      pp_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int r = 0; r < RB - 4; ++r)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      pp_barrier();
      kt = 1;
    }
    for (; kt < nk - DB - 1; ++kt) ktile(kt, IntC<1>{});
    for (; kt < nk; ++kt) ktile(kt, IntC<0>{});
    }
    if (wr == 0) pp_barrier();         // re-align the groups
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_barrier();                      // every wave is past its last stage read

    // ---- next tile's first K-tiles go out before this tile's epilogue ----
    const int cm0 = m0, cn0 = n0;
    id += gridDim.x;
    const bool more = id < ntiles;
    if (more) {
      setup(id, m0, n0);
      prologue_dma();
    }
    // ---- epilogue: 8 pieces of 16 rows per wave through the wave's 4 KiB region.  Identity
    // loads and output stores are non-temporal: C3 21.6k -> 22.1k img/s median over five
    // interleaved runs (profiles/r03/ppp_nt_epilogue_ab.log) -- fewer caches lines for this
    // stream of read-once / written-once tiles; bits unchanged ----
    float* wt = reinterpret_cast<float*>(smem + ppp::OFF_EPI) + wid * 16 * 64;
    const int c8 = lane & 7;
    const int n = cn0 + wc * 64 + 8 * c8;
    // EPI_DUAL_BIAS_RELU: a whole 256-wide tile lies on one side of nsplit (both % 256 == 0)
    const bool second = EPI == PIPNET_EPI_DUAL_BIAS_RELU && cn0 >= p.nsplit;
    bf16* const cout = second ? p.C2 : p.C;
    const int64_t ldo = second ? p.ldc2 : p.ldc;
    const int no = second ? n - p.nsplit : n;
    f32x4v b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
    if (EPI != PIPNET_EPI_NONE && p.bias) {
      b0 = *reinterpret_cast<const f32x4v*>(p.bias + n);
      b1 = *reinterpret_cast<const f32x4v*>(p.bias + n + 4);
    }
    // Row addresses: lane row (lane >> 3) of 8-row step q is mq = mrow0 + 8 q, clamped to M - 1.
    // One 64-bit row product per tile and a running pointer (+8 rows per step) with a select
    // for the clamped rows -- a per-store (int64) m * ld costs three quarter-rate integer
    // multiplies, which made up a third of this VALU-bound epilogue's cycles.
    const int mrow0 = cm0 + wr * 16 * RB + (lane >> 3);
    bf16x8v rr[16];
    if (HAS_R) {
      const bf16* rp = p.R + (int64_t)mrow0 * p.ldr + n;
      const bf16* const rlast = p.R + (int64_t)(p.M - 1) * p.ldr + n;
#pragma unroll
      for (int q = 0; q < 2 * RB; ++q) {
        const bf16* src = mrow0 + 8 * q < p.M ? rp : rlast;
        rr[q] = __builtin_bit_cast(bf16x8v, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src)));  // read once
        rp += 8 * p.ldr;
      }
    }
    bf16* op = cout + (int64_t)mrow0 * ldo + no;
    bf16* const olast = cout + (int64_t)(p.M - 1) * ldo + no;
    const int fq = lane >> 4;
#pragma unroll
    for (int r = 0; r < RB; ++r) {
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = 4 * fq + i;
          wt[row * 64 + ((nn * 16 + fr) ^ ppp::swz(row))] = acc[r][nn][i];
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int row = it * 8 + (lane >> 3);
        const int sw = ppp::swz(row);
        f32x4v x0 = *reinterpret_cast<const f32x4v*>(wt + row * 64 + ((8 * c8) ^ sw));
        f32x4v x1 = *reinterpret_cast<const f32x4v*>(wt + row * 64 + ((8 * c8 + 4) ^ sw));
        x0 += b0;
        x1 += b1;
        if (HAS_R) add_bf16x8(x0, x1, rr[r * 2 + it]);
        constexpr bool RELU = EPI == PIPNET_EPI_BIAS_RELU || EPI == PIPNET_EPI_BIAS_RESID_RELU;
        const bf16x8v o = (RELU || second) ? to_bf16x8<true>(x0, x1) : to_bf16x8<false>(x0, x1);
        bf16* dst = mrow0 + 16 * r + 8 * it < p.M ? op : olast;     // row = it * 8 + (lane >> 3)
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(dst));
        op += 8 * ldo;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (!more) break;
    // next tile's A(0) / B(0): younger are A1 B1 A2 (6) and this epilogue's stores (and, with a
    // residual, its loads -- already consumed, hence retired with everything older)
    if (nk > (SEG == 3 ? 1 : 2)) wait_steady(IntC<NSTORE>{});
    else pp_wait_vm<NSTORE>();         // fewer pieces follow B(0): wait a little longer
    pp_barrier();
    extra = 1;
  }
}

// ======================================================================================
// 3x3 / stride 1 / pad 1 convolutions on the ping-pong tile with an LDS input halo.
//
// On the pp tile every 32-deep K-tile brings 16 KiB of A (256 pixels x 32 channels of one
// tap) and 16 KiB of B through the LDS-DMA path, and that path -- not the MFMA pipe or the
// LDS port -- is what holds the big layers at 35-40 % of the bf16 peak (profiles/r02/
// bf16_lab.txt: the B-only-DMA ablation recovers most of the no-DMA rate).  For a 3x3
// stride-1 conv the nine taps of a 256-pixel tile read the same input pixels shifted by
// (ky-1)*W + (kx-1) in the linear NHWC pixel index.  This kernel stages, per pair of 32-channel
// chunks, the pixel range [m0 - W - 1, m0 + 256 + W + 1) once (the "halo": 256 + 2W + 2 <= 320
// rows of 64 B per chunk), and the 18 K-tiles of the pair -- taps t = 0..8, each for chunk
// halves h = 0, 1 -- read their A fragments from it at row offset ky*W + kx; only B still
// streams per K-tile.  K order (pair, tap, half): consecutive K-tiles read the two 64-B halves
// of the same 128-B weight line, as the pp kernel's (tap, chunk) order does (a (chunk, tap)
// order that revisits each line 9 K-tiles later measured 15-20 % slower than pp).  A bytes per
// K-tile fall from 16 KiB to 40 KiB / 18.  Taps that fall outside the image (padding, or a row
// / image boundary the linear index would wrap across) read a 256-B zero block at the same
// bank slot.
//
// Halo rows: chunk q of row r at physical chunk q ^ hs(r), hs(r) = ((r >> 2) & 1) << 1 --
// conflict-free for the 16x16x32 operand map at ANY row offset (each ds_read_b128 lane group
// of 16 reads 16 consecutive rows; checked for all offsets: every group hits 16 distinct
// 16-B bank slots), unlike the pp swizzle, which is conflict-free only on 16-row-aligned
// blocks.  A lane's 8 fragment rows differ by multiples of 16, so for a given tap the
// swizzle term is one per lane and the 8 fragment addresses differ by immediates.
// Pipeline, barriers, wave groups and epilogue are those of conv_bf16_pp_kernel: B of K-tile
// kt+2 is fetched in phase 0 of K-tile kt; the halo of pair P+1 (5 x 1 KiB pieces per wave)
// in phase 1 of K-tile 18P + 1 (its two slots were last read two K-tiles earlier, by pair
// P-1), so it is always older than the B pieces the counted waits retire.  The accumulation
// order depends on the layer only, never on M.
// Requirements: KH = KW = 3, stride 1, pad 1, Cin % 64 == 0, W <= 31, no seg.
// ======================================================================================
namespace ph {
constexpr int DB = 2, NS = DB + 2;
PIPNET_DEV int hs(int r) { return ((r >> 2) & 1) << 1; }
// NB = 16-column B fragments per wave: the tile is 256 x 64 NB.  The halo holds 320 rows
// (W <= 31) beside the 256-wide B stages, 384 rows (W <= 63) beside the narrower ones.
template <int NB>
struct Lay {
  static constexpr int BROWS = 64 * NB;                      // B rows of one K-tile
  static constexpr int BSTAGE = BROWS * pp::ROWB;
  static constexpr int HALO_ROWS = NB == 4 ? 320 : 384;
  static constexpr int HPC = HALO_ROWS / 16;                 // DMA pieces per chunk half
  static constexpr int HPW = 2 * HPC / 8;                    // halo pieces per wave per pair (5 / 6)
  static constexpr int BPW = BROWS / 16 >= 8 ? BROWS / 16 / 8 : 1;   // B pieces per wave per K-tile
  static constexpr int HALO_BYTES = HALO_ROWS * pp::ROWB;
  static constexpr int OFF_HALO = NS * BSTAGE;               // 4 halo slots: pair parity x chunk half
  static constexpr int OFF_ZERO = OFF_HALO + 4 * HALO_BYTES;
  static constexpr int SMEM = OFF_ZERO + 256 > pp::EPI_BYTES ? OFF_ZERO + 256 : pp::EPI_BYTES;
  static_assert(2 * HPC % 8 == 0, "halo pieces split evenly over 8 waves");
};
}  // namespace ph

// RB = 16-row blocks per wave group: 8 -> 256-row tiles, 7 -> 224-row tiles (fewer idle CUs in
// the last round of tiles, conv_bf16.hip pick_rb).  Every output element is the same MFMA chain
// over the same K order whatever RB is, so the choice never changes a bit of the result.
// ABL (tuning lab only, tools/bf16_lab.hip lab_halo; 0 in the product): 1 = no B DMA, 2 = no
// epilogue (one store per lane keeps the accumulators live), 4 = no barriers, 8 = no A fragment
// reads after the first, 16 = no halo DMA after pair 0 (stale LDS / registers: timing only).
// (The body is a device function so that the product kernel's name carries no lab parameter.)
// SEG = MFMA segments per 32-deep K-tile: 2 = two 16-MFMA phases (row halves), each between a
// barrier pair (rounds 2-5); 1 = ONE 32-MFMA segment per K-tile (round 6): the R segment issues
// the DMA, reads B and the row-half-0 A fragments and does the counted wait; the M segment runs
// half 0's 16 MFMAs with half 1's four A-fragment reads interleaved (each refills the registers of
// the row whose MFMAs just issued), then half 1's 16 -- half the barriers and priority switches per
// MFMA, the same registers, and the same per-accumulator K order (bitwise equal).
template <int EPI, int NB, int RB, int ABL, int SEG = 2>
__device__ __forceinline__ void conv3x3_bf16_halo_body(const ConvParams& p) {
  using namespace pp;
  using ph::NS;
  using L = ph::Lay<NB>;
  static_assert(RB == 7 || RB == 8, "RB");
  constexpr int BMR = 32 * RB;                                 // tile rows
  // The 64 / 128-wide forms (NB = 1 / 2: 384-row halo, duplicated B pieces) passed the
  // kernel-level tests but measured slower / flat and failed the C3 end-to-end bf16 bound
  // (pooled 0.10 vs 0.05) in their one run -- not dispatched, not validated.
  static_assert(NB == 4, "only the 256-wide halo tile is validated");
  constexpr int WCOLS = 16 * NB;
  __shared__ __attribute__((aligned(256))) unsigned char smem[L::SMEM];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  tile_coords(p, BMR, L::BROWS, m0, n0);
  const int W = p.Wd, HW = p.H * p.Wd;
  const int npair = p.Cin / (2 * BK);
  const int nk = 18 * npair;

  // ---- B DMA sources: BPW pieces of 16 rows x 64 B per wave (pp swizzle); with fewer pieces
  // than waves (NB = 1: 4 pieces) waves 4..7 repeat waves 0..3's pieces -- identical bytes to the
  // same LDS rows, so every wave issues the same count and the vmcnt waits stay uniform ----
  const int drow = lane >> 2;
  const bf16* wsrc[L::BPW];
#pragma unroll
  for (int i = 0; i < L::BPW; ++i) {
    const int pc = L::BROWS / 16 >= 8 ? wid + 8 * i : (wid % (L::BROWS / 16));
    const int row = 16 * pc + drow;
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + 8 * ((lane & 3) ^ g(drow));
  }
  int bdst[L::BPW];
#pragma unroll
  for (int i = 0; i < L::BPW; ++i)    // wave-uniform: SGPRs (as VGPRs they pushed the RB = 8 form into spills)
    bdst[i] = __builtin_amdgcn_readfirstlane((L::BROWS / 16 >= 8 ? wid + 8 * i : (wid % (L::BROWS / 16))) * 1024);
  // ---- halo DMA: 2 HPC pieces per pair, HPW per wave: piece e = wid + 8 i is chunk half
  // e / HPC, halo rows 16 (e % HPC) + ...; halo row i = pixel m0 - W - 1 + i ----
  int hsrc[L::HPW];                                           // element offsets: M * Cin < 2^31 (halo_ok)
  int hdst[L::HPW];
#pragma unroll
  for (int i = 0; i < L::HPW; ++i) {
    const int e = wid + 8 * i, h = e >= L::HPC ? 1 : 0, pc = e - L::HPC * h;
    const int row = 16 * pc + drow;
    const int pix = min(max(m0 - W - 1 + row, 0), p.M - 1);
    hsrc[i] = pix * p.Cin + h * BK + 8 * ((lane & 3) ^ ph::hs(row));
    hdst[i] = __builtin_amdgcn_readfirstlane(h * L::HALO_BYTES + pc * 1024);
  }
  // ---- this lane's 8 fragment rows: tile row wr*128 + j*16 + (lane & 15); 9-bit tap masks ----
  const int fr = lane & 15;
  unsigned vmask[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = m0 + wr * 16 * RB + j * 16 + fr;
    unsigned mk = 0;
    if (m < p.M) {
      const int rr = m % HW;
      const int y = rr / W, x = rr - (rr / W) * W;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
          if ((unsigned)(y + ky - 1) < (unsigned)p.H && (unsigned)(x + kx - 1) < (unsigned)W)
            mk |= 1u << (ky * 3 + kx);
    }
    vmask[j] = mk;
  }
  if (tid < 16) *reinterpret_cast<u32x4*>(smem + L::OFF_ZERO + 16 * tid) = u32x4{0u, 0u, 0u, 0u};

  auto stage_b = [&](int kt) {
    if constexpr ((ABL & 1) != 0) {
      if (kt > 1) return;
    }
    const int P = kt / 18, rem = kt - 18 * P;
    const int k0 = (rem >> 1) * p.Cin + (2 * P + (rem & 1)) * BK;
    unsigned char* base = smem + (kt % NS) * L::BSTAGE;
#pragma unroll
    for (int i = 0; i < L::BPW; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + k0),
                                       (__attribute__((address_space(3))) void*)(base + bdst[i]), 16, 0, 0);
  };
  auto stage_halo = [&](int P) {
    if constexpr ((ABL & 16) != 0) {
      if (P > 0) return;
    }
    unsigned char* base = smem + L::OFF_HALO + (P & 1) * 2 * L::HALO_BYTES;
#pragma unroll
    for (int i = 0; i < L::HPW; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p.A + hsrc[i] + P * 2 * BK),
                                       (__attribute__((address_space(3))) void*)(base + hdst[i]), 16, 0, 0);
  };
  const int fofs_b = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));
  const int q16 = (lane >> 4) << 4;
  auto read_b = [&](bf16x8v (&fb)[NB], const unsigned char* st) {
#pragma unroll
    for (int n = 0; n < NB; ++n)
      fb[n] = *reinterpret_cast<const bf16x8v*>(st + (wc * WCOLS + n * 16) * ROWB + fofs_b);
  };
  const unsigned char* zb = smem + L::OFF_ZERO;
  // lane byte offset inside a halo slot for this tap (fragment rows j add j * 1 KiB)
  bool a_once = false;
  auto read_a = [&](bf16x8v (&fa)[4], const unsigned char* hb, int half, int loff, unsigned tbit) {
    if constexpr ((ABL & 8) != 0) {
      if (a_once) return;
      if (half) a_once = true;
    }
    const unsigned char* zl = zb + (loff & 255);
#pragma unroll
    for (int r = 0; r < (half ? RB - 4 : 4); ++r) {
      const int j = half * 4 + r;
      const unsigned char* ptr = (vmask[j] & tbit) ? hb + loff + j * 1024 : zl;
      fa[r] = *reinterpret_cast<const bf16x8v*>(ptr);
    }
  };

  f32x4v acc[8][NB];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};

  // prologue: halo(0), B(0), B(1); wait for halo(0) and B(0)
  stage_halo(0);
  stage_b(0);
  if (1 < nk) stage_b(1);
  if (nk > 1) pp_wait_vm<L::BPW>();
  else pp_wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // zero block written
  pp_barrier();
  if (wr == 1) pp_barrier();                                   // group 1 runs one barrier behind
  // lab ABL 64: static priority for the younger half (waves 4-7) instead of per-segment flips
  // (cdna_hip_programming.md T5 static form); ABL 128: no s_setprio at all
  if constexpr ((ABL & 64) != 0) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (SEG == 3 && ABL == 0) static_prio();

  // K-tile kt = 18 P + 2 t + h.  B of K-tile kt+2 is fetched in phase 0 of kt; the halo of
  // pair P+1 in phase 1 of (t, h) = (0, 1).  The wait in phase 1 of kt retires B(kt+1): younger
  // are B(kt+2) and the halo pieces issued at (0, 1) or, for (1, 0), one K-tile earlier; none
  // in the last tap of the last pair.  Everything but the MFMA stream is scalar bookkeeping
  // kept branch-light (one compile-time h per unrolled half).
  auto hbar = [&]() {
    if constexpr ((ABL & 4) == 0) pp_barrier();
  };
  bf16x8v fa[4], fb[NB];
  const int lrow = wr * 16 * RB + fr;
  // one A fragment row j (0..RB*2-1 of the wave group's 16-row blocks) for the SEG = 1 interleave
  auto read_a_row = [&](bf16x8v& f, const unsigned char* hb, int j, int loff, unsigned tbit) {
    if constexpr ((ABL & 8) != 0) {
      if (a_once) return;
    }
    const unsigned char* ptr = (vmask[j] & tbit) ? hb + loff + j * 1024 : zb + (loff & 255);
    if constexpr (SEG == 3) f = ds_read_b128_asm(ptr);      // waited for explicitly (below)
    else f = *reinterpret_cast<const bf16x8v*>(ptr);
  };
  int kt = 0;
  for (int P = 0; P < npair; ++P) {
    const bool more = P + 1 < npair;
    const unsigned char* hp = smem + L::OFF_HALO + (P & 1) * 2 * L::HALO_BYTES;
    for (int t = 0; t < 9; ++t) {
      const int ky = t >= 6 ? 2 : (t >= 3 ? 1 : 0), kx = t - 3 * ky;
      const int hr = lrow + ky * W + kx;                       // this lane's halo row of fragment j = 0
      const int loff = hr * ROWB + (q16 ^ ((hr << 3) & 32));   // chunk ^ hs(hr), in bytes
      const unsigned tbit = 1u << t;
      const bool last = !more && t == 8;
#pragma unroll
      for (int h = 0; h < 2; ++h, ++kt) {
        const unsigned char* st = smem + (kt & (NS - 1)) * L::BSTAGE;
        const unsigned char* hb = hp + h * L::HALO_BYTES;
        if constexpr (SEG == 1 || SEG == 3) {
          // ---- R segment: DMA (B of kt+2; the next pair's halo at (t, h) = (0, 1)), B and
          // row-half-0 A fragments, wait for this wave's pieces of K-tile kt+1 ----
          if (!last) stage_b(kt + 2);
          if (h == 1 && t == 0 && more) stage_halo(P + 1);
          read_b(fb, st);
          read_a(fa, hb, 0, loff, tbit);
          if (last) pp_wait_vm<0>();
          else if (more && ((h == 1 && t == 0) || (h == 0 && t == 1))) pp_wait_vm<L::BPW + L::HPW>();
          else pp_wait_vm<L::BPW>();
          hbar();
          // ---- M segment: 16 MFMAs of half 0 with half 1's A reads interleaved, 16 of half 1 ----
          if constexpr ((ABL & (64 | 128)) == 0) seg_prio(1);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int n = 0; n < NB; ++n)
              acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
            if (r < RB - 4) {
              __builtin_amdgcn_sched_barrier(0);
              read_a_row(fa[r], hb, 4 + r, loff, tbit);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          if constexpr ((ABL & 8) != 0) a_once = true;
#pragma unroll
          for (int r = 0; r < RB - 4; ++r) {
            if constexpr (SEG == 3) {
              // the compiler sees the inline-asm reads as ready at issue: wait for row r's own read
              // only (LDS returns in order; the LDS-DMA in the loop makes the compiler's own waits
              // lgkmcnt(0), which would stall on the last of the four reads)
              __builtin_amdgcn_sched_barrier(0);
              lgkm_wait_dyn(RB - 5 - r);
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int n = 0; n < NB; ++n)
              acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
          }
          if constexpr ((ABL & (64 | 128)) == 0) seg_prio(0);
          hbar();
          continue;
        }
        // ---- phase 0: rows 0..63 of the wave's block ----
        if (!last) stage_b(kt + 2);
        read_b(fb, st);
        read_a(fa, hb, 0, loff, tbit);
        hbar();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int n = 0; n < NB; ++n)
            acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        hbar();
        // ---- phase 1: rows 64..127 ----
        if (h == 1 && t == 0 && more) stage_halo(P + 1);
        read_a(fa, hb, 1, loff, tbit);
        if (last) pp_wait_vm<0>();
        else if (more && ((h == 1 && t == 0) || (h == 0 && t == 1))) pp_wait_vm<L::BPW + L::HPW>();
        else pp_wait_vm<L::BPW>();
        hbar();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int r = 0; r < RB - 4; ++r)
#pragma unroll
          for (int n = 0; n < NB; ++n)
            acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        hbar();
      }
    }
  }
  if (wr == 0) hbar();                                   // re-align the groups
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pp_barrier();                                                // stage / halo buffers free for the epilogue
  if constexpr ((ABL & 2) != 0) {
    float tsum = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int e = 0; e < 4; ++e) tsum += acc[r][n][e];
    reinterpret_cast<float*>(p.C)[(int64_t)blockIdx.x * pp::NT + tid] = tsum;
    return;
  }
  pp_epilogue<EPI, NB, RB>(p, acc, smem, m0, n0, wr, wc, lane, wid);
}

template <int EPI, int NB = 4, int RB = 8>
__global__ __launch_bounds__(pp::NT, 1) void conv3x3_bf16_halo_kernel(ConvParams p) {
  conv3x3_bf16_halo_body<EPI, NB, RB, 0, PIPNET_HALO_SEG>(p);
}

template <int EPI, int NB, int RB, int ABL, int SEG = 2>   // tuning lab only (tools/bf16_lab.hip lab_halo)
__global__ __launch_bounds__(pp::NT, 1) void conv3x3_bf16_halo_abl_kernel(ConvParams p) {
  conv3x3_bf16_halo_body<EPI, NB, RB, ABL, SEG>(p);
}

// ======================================================================================
// 3x3 / stride 1 / pad 1 convolutions with Cin = N = 64 (ResNet layer1 conv2, tile M 256) or
// Cin = N = 128 (layer2 conv2, tile M 128) on an LDS input halo -- "tile 11".
//
// The generic tiles for these layers (tile 6, 256 x 64; tile 4, 128 x 128) walk K = 9 Cin as
// 32-deep K-tiles and bring every tap's A block through the LDS-DMA path -- the input 9 times --
// with 4 / 8 MFMAs per wave per K-tile: DMA-path bound at ~300 / ~430 TF/s.  Here a BM-pixel
// tile stages the linear pixel range [m0 - W - 1, m0 + BM + W + 1) once, all Cin channels
// (48 KiB: <= 384 rows of 128 B / <= 192 rows of 256 B), and streams the weights through a
// 3-slot ring of 8 KiB K-tiles (N x KT: one tap at N = 64, one 32-channel chunk of a tap at
// N = 128), K-tile k + 2 in flight while k is multiplied: 72 KiB, two workgroups per CU.
// Arithmetic is the generic tiles', bit for bit: MFMA 32x32x16, each of the 4 waves owning 64
// pixels x 64 columns (2 x 2 blocks), K walked in their order -- tap-major, then 32-channel
// chunk, then the chunk's two k-steps, half-wave h supplying channels 8 (2 h + q) .. +7 of step
// q -- and the same epilogue, so choosing this tile changes no output bit (tests/test_gpu_bf16.py).
// Taps that leave the image read a 256-B zero block at the same bank slot (9-bit mask per
// fragment row), the zeros the generic tiles read there.  Rows of RB bytes (halo pixels, weight
// rows) hold 16-B chunk k at k ^ ((r >> log2(256 / RB)) & (RB / 16 - 1)): every ds_read_b128
// lane group covers 16 consecutive rows mod 16 and so 16 distinct bank slots, at any tap offset.
// Requirements: KH = KW = 3, stride 1, pad 1, Cin = N in {64, 128}, W <= 63 / 31, no seg.
// ======================================================================================
namespace hsm {
constexpr int NT = 256, NSLOT = 3, SLOT_BYTES = 8192, HALO_BYTES = 48 * 1024;
constexpr int OFF_B = HALO_BYTES, OFF_ZERO = OFF_B + NSLOT * SLOT_BYTES;
constexpr int SMEM = OFF_ZERO + 256;
constexpr int EPI_LD = 68;                            // epilogue fp32 rows: 64 + 4 pad
static_assert(4 * 32 * EPI_LD * 4 <= SMEM, "epilogue re-lay fits");
static_assert(2 * SMEM <= 160 * 1024, "two workgroups per CU");
template <int CIN>
struct Shape {
  static constexpr int BN = CIN, BM = CIN == 64 ? 256 : 128;
  static constexpr int WN = BN / 64, WM = 4 / WN;     // waves: WM x WN, 64 x 64 each
  static constexpr int KT = SLOT_BYTES / (2 * BN);    // channels per weight K-tile (64 / 32)
  static constexpr int NKT = 9 * CIN / KT;            // K-tiles per tile (9 / 36)
  static constexpr int RB = 2 * CIN, WB = 2 * KT;     // halo / weight row bytes
  static constexpr int HALO_ROWS = HALO_BYTES / RB;   // 384 / 192
  static constexpr int MAX_W = (HALO_ROWS - BM - 2) / 2;
  static_assert(WM * 64 == BM, "wave grid");
};
// 16-B slot swizzle of a row of RB bytes
template <int RB>
PIPNET_DEV int sw(int r) {
  return RB == 256 ? (r & 15) : RB == 128 ? ((r >> 1) & 7) : ((r >> 2) & 3);
}
}  // namespace hsm

template <int CIN, int EPI>
__global__ __launch_bounds__(hsm::NT, 2) void conv3x3_bf16_hsmall_kernel(ConvParams p) {
  using namespace hsm;
  using S = Shape<CIN>;
  constexpr int BM = S::BM, RB = S::RB, WB = S::WB, KT = S::KT, NKT = S::NKT;
  __shared__ __attribute__((aligned(256))) unsigned char smem[SMEM];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / S::WN, wn = wid % S::WN;
  const int nwg = (p.M + BM - 1) / BM;
  const int m0 = xcd_remap(blockIdx.x, nwg) * BM;
  const int W = p.Wd, HW = p.H * p.Wd;
  constexpr int HROWS_PC = 1024 / RB;                   // halo rows per 1-KiB DMA piece
  const int npiece = ((BM + 2 * W + 2) + HROWS_PC - 1) / HROWS_PC;

  // ---- this lane's 2 fragment pixels (64 wm + 32 i + (lane & 31)): 9-bit tap masks ----
  const int lr = lane & 31, lh = lane >> 5;
  unsigned vmask[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + 64 * wm + 32 * i + lr;
    unsigned mk = 0;
    if (m < p.M) {
      const int rr = m % HW;
      const int y = rr / W, x = rr - (rr / W) * W;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
          if ((unsigned)(y + ky - 1) < (unsigned)p.H && (unsigned)(x + kx - 1) < (unsigned)W) mk |= 1u << (ky * 3 + kx);
    }
    vmask[i] = mk;
  }
  if (tid < 16) *reinterpret_cast<u32x4*>(smem + OFF_ZERO + 16 * tid) = u32x4{0u, 0u, 0u, 0u};

  // ---- LDS-DMA: 1-KiB pieces, lane -> (row, 16-B slot) of a piece of RB- / WB-byte rows ----
  auto dma = [&](const bf16* src, int off) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(smem + off), 16, 0, 0);
  };
  {
    const int drow = lane / (RB / 16), dslot = lane % (RB / 16);
    for (int pc = wid; pc < npiece; pc += 4) {
      const int r = HROWS_PC * pc + drow;
      const int pix = min(max(m0 - W - 1 + r, 0), p.M - 1);
      dma(p.A + (int64_t)pix * p.Cinp + 8 * (dslot ^ sw<RB>(r)), pc * 1024);
    }
  }
  const int wrow = lane / (WB / 16), wslot = lane % (WB / 16);
  auto stage_k = [&](int kt) {                          // 8 pieces: this wave's wid, wid + 4
    const int t = kt / (CIN / KT), c0 = (kt % (CIN / KT)) * KT;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pc = wid + 4 * h, n = (1024 / WB) * pc + wrow;
      dma(p.W + (int64_t)n * p.K + t * CIN + c0 + 8 * (wslot ^ sw<WB>(n)),
          OFF_B + (kt % NSLOT) * SLOT_BYTES + pc * 1024);
    }
  };
  stage_k(0);
  stage_k(1);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;

  const int lrow = 64 * wm + lr;                          // halo row of fragment 0 at tap (0, 0)
  auto ktile = [&](int kt) {
    // K-tile kt landed (only kt + 1's 2 pieces may still fly), every wave done with kt - 1
    if (kt + 1 < NKT) wait_dma_barrier<2>();
    else wait_dma_barrier<0>();
    if (kt + 2 < NKT) stage_k(kt + 2);                    // into the slot K-tile kt - 1 used
    const int t = kt / (CIN / KT), c0 = (kt % (CIN / KT)) * KT;
    const int ky = t / 3, kx = t - 3 * (t / 3);
    const unsigned char* bslot = smem + OFF_B + (kt % NSLOT) * SLOT_BYTES;
#pragma unroll
    for (int kk = 0; kk < KT / 16; ++kk) {                // chunk kk >> 1 of the K-tile, k-step kk & 1
      const int gb = 4 * (kk >> 1) + 2 * lh + (kk & 1);   // 16-B channel group within the K-tile
      const int ga = c0 / 8 + gb;                         // ... within the pixel's row
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int hr = lrow + 32 * i + ky * W + kx;
        const int aoff = hr * RB + 16 * (ga ^ sw<RB>(hr));
        const unsigned char* ptr = (vmask[i] >> t) & 1u ? smem + aoff : smem + OFF_ZERO + (aoff & 255);
        fa[i] = *reinterpret_cast<const bf16x8*>(ptr);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 64 * wn + 32 * j + lr;
        fb[j] = *reinterpret_cast<const bf16x8*>(bslot + n * WB + 16 * (gb ^ sw<WB>(n)));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  };
  if constexpr (NKT <= 9) {
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) ktile(kt);
  } else {
    for (int kt = 0; kt < NKT; ++kt) ktile(kt);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // halo / ring free for the epilogue

  // ---- epilogue (the generic tiles'): per 32-row block, re-lay through the wave's LDS rows, 8 channels
  // per lane, bias, residual, ReLU, bf16, one 16-B store ----
  float* wt = reinterpret_cast<float*>(smem) + wid * 32 * EPI_LD;
  const int c8 = lane & 7;
  f32x4 b0 = {0.f, 0.f, 0.f, 0.f}, b1 = b0;
  if (EPI != PIPNET_EPI_NONE && p.bias) {
    b0 = ld4(p.bias + 64 * wn + 8 * c8);
    b1 = ld4(p.bias + 64 * wn + 8 * c8 + 4);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) wt[((v & 3) + 8 * (v >> 2) + 4 * lh) * EPI_LD + 32 * j + lr] = acc[i][j][v];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (i == 0) vm_drain();                      // bias preloads landed (common.hpp)
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = 8 * it + (lane >> 3);
      const int m = m0 + 64 * wm + 32 * i + row;
      f32x4 x0 = ld4(wt + row * EPI_LD + 8 * c8), x1 = ld4(wt + row * EPI_LD + 8 * c8 + 4);
      x0 += b0;
      x1 += b1;
      if (EPI == PIPNET_EPI_BIAS_RESID_RELU && m < p.M) {
        add_bf16x8(x0, x1, *reinterpret_cast<const bf16x8*>(p.R + (int64_t)m * p.ldr + 64 * wn + 8 * c8));
      }
      const bf16x8 o = to_bf16x8<EPI == PIPNET_EPI_BIAS_RELU || EPI == PIPNET_EPI_BIAS_RESID_RELU>(x0, x1);
      if (m < p.M) *reinterpret_cast<bf16x8*>(p.C + (int64_t)m * p.ldc + 64 * wn + 8 * c8) = o;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next block's writes
  }
}


// ======================================================================================
// ResNet stem fused with its max-pool (bf16 build): the 4x4 stride-1 conv over the 2x2
// space-to-depth image (Cin 16, N 64, K 256; resnet_features.py:161-163 conv1 + bn1 + relu,
// see pipnet_nchw_to_s2d_bf16) + bias + ReLU, then MaxPool2d(3, 2, 1) (resnet_features.py:164).
// Unfused, the stem writes a 112x112x64 bf16 map (103 MB per 64 images) that the pool reads
// back.  Here one workgroup owns PR = 2 pooled rows of one image: it computes the 2 PR + 1 = 5
// stem rows they need (1.25x the stem's MFMAs), keeps them in LDS as bf16 and writes only
// the pooled rows.  The 8 s2d input rows (<= 30 KiB) and all of W (64 x 256, 32 KiB) are
// staged once by LDS-DMA; 6 waves x 3 blocks of 32 stem pixels x 2 blocks of 32 channels.
// Arithmetic is tile 6's, bit for bit (MFMA 32x32x16, 32-deep K-tiles of 2 taps, half-wave
// h = tap 2 kt + h, k-step q = channels 8 q .. +7; bias + ReLU + RNE to bf16), and the pool
// is maxpool_nhwc_bf16_kernel's (fmaxf from -inf over (ky, kx) in order), so the pooled map
// is bitwise the unfused one's (tests/test_gpu_bf16.py::test_stem_pool_bf16_matches_unfused).
// LDS rows: input pixel q's two 16-B chunks at c ^ ((q >> 3) & 1); weight row n's 32 chunks
// at c ^ (n & 15).  The stem rows re-use the staging area once every wave has finished.
// Requirements: OW = SW - 3 <= 112, 16-B aligned tensors.
// ======================================================================================
namespace spool {
constexpr int NT = 384, PR = 2, SR = 2 * PR + 1, IR = SR + 3, N = 64, K = 256;
constexpr int MAX_OW = 112, BLOCKS = 18;              // 18 x 32 >= SR x MAX_OW = 560 stem pixels
constexpr int IN_BYTES = 30 * 1024, OFF_WT = IN_BYTES, WT_BYTES = N * K * 2;
constexpr int OUT_BYTES = BLOCKS * 32 * N * 2;        // 72 KiB of bf16 stem rows (576 >= SR x MAX_OW: padding rows too)
constexpr int SMEM = OUT_BYTES > OFF_WT + WT_BYTES ? OUT_BYTES : OFF_WT + WT_BYTES;
static_assert(2 * SMEM <= 160 * 1024, "two workgroups per CU");
static_assert(BLOCKS * 32 >= SR * MAX_OW && BLOCKS == 3 * (NT / 64), "3 blocks per wave");
}  // namespace spool

__global__ __launch_bounds__(spool::NT, 2) void stem_pool_bf16_kernel(const bf16* __restrict__ S, int SH, int SW,
                                                                      const bf16* __restrict__ Wp,
                                                                      const float* __restrict__ bias,
                                                                      bf16* __restrict__ Y, int PH, int PW) {
  using namespace spool;
  __shared__ __attribute__((aligned(256))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int npr = (PH + PR - 1) / PR;
  const int b = blockIdx.x / npr, pr = blockIdx.x - b * npr;
  const int OH = SH - 3, OW = SW - 3;
  const int oy0 = 2 * PR * pr - 1;                     // stem row of local row 0

  // ---- LDS-DMA: input rows oy0 .. oy0 + 7 (clamped; rows outside feed only discarded stem rows)
  auto dma = [&](const bf16* src, int off) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)(smem + off), 16, 0, 0);
  };
  const int npix = IR * SW, npin = (npix + 31) / 32;
  for (int pc = wid; pc < npin; pc += NT / 64) {
    const int q = min(32 * pc + (lane >> 1), npix - 1);
    const int rr = q / SW, x = q - rr * SW;
    const int iy = min(max(oy0 + rr, 0), SH - 1);
    dma(S + (((int64_t)b * SH + iy) * SW + x) * 16 + 8 * ((lane & 1) ^ ((q >> 3) & 1)), pc * 1024);
  }
  for (int pc = wid; pc < WT_BYTES / 1024; pc += NT / 64) {
    const int n = 2 * pc + (lane >> 5), sl = lane & 31;
    dma(Wp + n * K + 8 * (sl ^ (n & 15)), OFF_WT + pc * 1024);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- MFMAs: this wave's blocks 3 wid + i, lane row = stem pixel m = 32 blk + (lane & 31)
  const int lr = lane & 31, lh = lane >> 5;
  int q0[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int m = 32 * (3 * wid + i) + lr;
    const int r = m / OW, ox = m - r * OW;
    q0[i] = m < SR * OW ? r * SW + ox : 0;             // padding rows read row 0, then are dropped
  }
  f32x16 acc[3][2];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][j][v] = 0.f;
#pragma unroll 2
  for (int kt = 0; kt < K / 32; ++kt) {
    const int tap = 2 * kt + lh, a = tap >> 2, a2 = tap & 3;
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      bf16x8 fa[3], fb[2];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int qp = q0[i] + a * SW + a2;
        fa[i] = *reinterpret_cast<const bf16x8*>(smem + qp * 32 + 16 * (qq ^ ((qp >> 3) & 1)));
      }
      const int c = 4 * kt + 2 * lh + qq;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 32 * j + lr;
        fb[j] = *reinterpret_cast<const bf16x8*>(smem + OFF_WT + n * 512 + 16 * (c ^ (n & 15)));
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // staging area free

  // ---- stem rows to LDS as bf16: relu(acc + b), rounded as tile 6's epilogue rounds.  Every
  // block's 32 rows are written, padding rows past SR x OW included (the buffer holds all 576):
  // no per-element guard (a guarded store per element made hipcc branch and wait around each) ----
  bf16* out = reinterpret_cast<bf16*>(smem);
  const float bj[2] = {bias[lr], bias[32 + lr]};
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = 32 * (3 * wid + i) + (v & 3) + 8 * (v >> 2) + 4 * lh;
        out[m * N + 32 * j + lr] = (bf16)fmaxf(acc[i][j][v] + bj[j], 0.f);
      }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- MaxPool2d(3, 2, 1) over the stem rows, 8 channels per item: lane group (tid >> 3) walks
  // the pooled columns, no division.  Window taps outside the stem map are clamped onto an edge
  // tap of the same window (max is idempotent, so the duplicate changes nothing) instead of being
  // skipped: the nine reads carry no branch.  Same fmaxf chain from -inf in (ky, kx) order over
  // the in-range taps, with duplicates inserted -- bitwise the unfused pool's result ----
  const int c8 = tid & 7;
#pragma unroll
  for (int r = 0; r < PR; ++r) {
    const int py = PR * pr + r;
    if (py >= PH) break;
    int lrow[3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) lrow[ky] = min(max(2 * py - 1 + ky, 0), OH - 1) - oy0;
    for (int px = tid >> 3; px < PW; px += NT / 8) {
      int col[3];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) col[kx] = min(max(2 * px - 1 + kx, 0), OW - 1);
      float mx[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) mx[e] = -INFINITY;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const bf16x8 v = *reinterpret_cast<const bf16x8*>(out + (lrow[ky] * OW + col[kx]) * N + 8 * c8);
#pragma unroll
          for (int e = 0; e < 8; ++e) mx[e] = fmaxf(mx[e], (float)v[e]);
        }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (bf16)mx[e];
      *reinterpret_cast<bf16x8*>(Y + (((int64_t)b * PH + py) * PW + px) * N + 8 * c8) = o;
    }
  }
}

}  // namespace pipnet_bf16
