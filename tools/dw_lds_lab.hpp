// Lab-only (not in the product library): LDS-staged depthwise 7x7 + LayerNorm, measured
// against the product's register-tile kernel (convnext_dw.hpp) in round 3 and not adopted --
// profiles/r03/dw_lds_lab.txt.  Included by tools/dw_lab.hip after convnext_dw.hpp.
#pragma once
#include "../count_pipnet_amd/csrc/convnext_dw.hpp"

namespace pipnet_dw {

// ======================================================================================
// LDS-staged depthwise 7x7 + bias + LayerNorm(C) (C <= 384).
//
// Why: the register-tile kernel above re-reads every input row from L2 / L1 for each output
// row it touches (7 rows x (TX+6)/TX columns per output pixel) and fetches the weights per
// lane from the vector cache: ~150 vector-memory instructions per 98 packed FMAs, so it runs
// on the texture path (64 B/clk/CU) at 2.3-2.6 TB/s.  Here the 7x7 re-reads come from LDS
// (256 B/clk/CU) and the weights from SGPRs:
//
//   * a 512-thread workgroup owns a TH x TWC pixel tile of one image and ALL C channels
//     (LayerNorm needs them); the C channels go through LDS in 32-channel chunks: the
//     (TH+6) x (TWC+6) input patch of a chunk (128 B per pixel, one cache line) is fetched
//     by LDS-DMA into one of two buffers while the previous chunk is being computed;
//   * wave w computes channel quad w of every chunk (so its 49 weight quads are
//     wave-uniform: scalar loads, SGPR operands of v_pk_fma_f32); lane = (row pair, column):
//     two vertically adjacent output pixels, so the 7 kx reads of an input row feed both
//     (8 rows x 7 reads per 98 packed FMAs, a two-row register ring walking ky);
//   * LDS pixel stride 144 B (128 B of channels + 16 B pad): the 16 lanes of a ds_read_b128
//     lane group read 16 pixels that are distinct mod 16 (the tile pitch PP makes sure), and
//     9p mod 16 is then distinct -- conflict-free, with every tap's offset a compile-time
//     immediate (an XOR swizzle would cost address VALU per read);
//   * the raw conv outputs stay in registers (C/32 quads x 2 pixels per lane); LayerNorm is
//     two-pass (mean, then the centred sum of squares) with the 8 waves' partial sums of a
//     pixel combined through LDS in wave order, then the normalised tile leaves through LDS
//     in 128-B pixel rows (full-line, coalesced stores).
// Tap order per output is (ky, kx) row-major after the bias, as in the register-tile kernel,
// so the conv sums are bitwise identical to it; only the LayerNorm reduction order differs.
// Per pixel the arithmetic does not depend on the tile or the batch (batch-invariant).
// ======================================================================================
static __device__ __attribute__((aligned(16))) float g_dw_zero[4] = {0.f, 0.f, 0.f, 0.f};

template <int C, int TWC>
struct DwLdsGeo {
  static constexpr int NT = 512;
  static constexpr int NCH = C / 32;                     // 32-channel chunks
  static constexpr int RG = 64 / TWC;                    // lane row groups (2 output rows each)
  static constexpr int TH = 2 * RG;                      // tile rows
  static constexpr int PW = TWC + 6, PH = TH + 6;        // patch columns / rows
  // patch pitch: the lanes of a ds_read_b128 group span two row groups when TWC = 16, whose
  // pixels differ by 2 PP -- it must be a multiple of 16 to keep them distinct mod 16
  static constexpr int PP = TWC == 16 ? 24 : PW;
  static constexpr int PXB = 144;                        // LDS bytes per patch pixel
  static constexpr int NSLOT = PH * PP * 9;              // 16-B slots per chunk (pad slot included)
  static constexpr int NI = (NSLOT + 63) / 64;           // LDS-DMA wave instructions per chunk
  static constexpr int NPI = (NI + 7) / 8;               // per wave (at most)
  static constexpr int BUFB = NI * 1024;                 // bytes per patch buffer
  static constexpr int TPX = TH * TWC;                   // tile pixels (128)
  static constexpr int STGC = TPX * 128;                 // staging bytes per chunk (tile x 32 ch)
  static constexpr int NST = (2 * BUFB / STGC) < NCH ? (2 * BUFB / STGC) : NCH;   // chunks per store round
  static_assert(C % 32 == 0 && NCH <= 12, "C");
  static_assert(TWC == 16 || TWC == 32, "TWC");
  static_assert(TPX == 128 && NST >= 1, "tile");
};

// ABL (tuning lab only, tools/dw_lab.hip; 0 in the product): 1 = no LDS-DMA after chunk 0,
// 2 = no weight loads (the bias quad stands in), 4 = no row reads / FMAs
template <int C, int TWC, bool S3, int ABL = 0>
__global__ __launch_bounds__(512, 1) void dwconv7_ln_lds_kernel(const float* __restrict__ x, int H, int W,
                                                                 const float* __restrict__ wp,
                                                                 const float* __restrict__ bias,
                                                                 const float* __restrict__ lnw,
                                                                 const float* __restrict__ lnb,
                                                                 void* __restrict__ yv, int tiles_x, int tiles_y) {
  using G = DwLdsGeo<C, TWC>;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * G::BUFB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int txi = tile % tiles_x;
  const int tyi = (tile / tiles_x) % tiles_y;
  const int b = tile / (tiles_x * tiles_y);
  const int ty0 = tyi * G::TH, tx0 = txi * TWC;
  const float* ximg = x + (int64_t)b * H * W * C;

  // ---- LDS-DMA sources of this wave's instructions: slot e -> pixel e / 9, quad e % 9 (8 =
  // pad), element offset inside the image (-1: outside the image / pad -> zero source) ----
  int doff[G::NPI];
#pragma unroll
  for (int k = 0; k < G::NPI; ++k) {
    const int i = wid + 8 * k;
    const int e = i * 64 + lane;
    const int px = e / 9, s = e - 9 * px;
    const int pr = px / G::PP, pc = px - pr * G::PP;
    const int iy = ty0 + pr - 3, ix = tx0 + pc - 3;
    const bool ok = i < G::NI && e < G::NSLOT && s < 8 && pc < G::PW && (unsigned)iy < (unsigned)H &&
                    (unsigned)ix < (unsigned)W;
    doff[k] = ok ? (iy * W + ix) * C + 4 * s : -1;
  }
  auto dma = [&](int j, int buf) {
#pragma unroll
    for (int k = 0; k < G::NPI; ++k) {
      const int i = wid + 8 * k;
      if (i < G::NI) {
        const float* src = doff[k] >= 0 ? ximg + doff[k] + 32 * j : g_dw_zero;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(smem + buf * G::BUFB + i * 1024), 16,
                                         0, 0);
      }
    }
  };
  auto sync = [&]() { asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); };

  const int rg = lane / TWC, col = lane % TWC;
  const int lbase = ((2 * rg) * G::PP + col) * G::PXB + 16 * wid;   // pixel (2 rg, col) of the patch, quad wid
  f32x4 acc[G::NCH][2];

  dma(0, 0);
  sync();
#pragma unroll
  for (int j = 0; j < G::NCH; ++j) {
    if (j + 1 < G::NCH && (ABL & 1) == 0) dma(j + 1, (j + 1) & 1);   // into the buffer every wave finished with
    const unsigned char* bp = smem + (j & 1) * G::BUFB + lbase;
    const int c = 32 * j + 4 * wid;
    const f32x4 bq = ld4(bias + c);
    acc[j][0] = bq;
    acc[j][1] = bq;
    // Software pipeline over ky: one lgkmcnt(0) per step retires patch row ky+1 and the ky
    // weights (both issued a step earlier); then the ky+1 weights (SGPR) and row ky+2 are
    // issued and the step's FMAs run on registers that already arrived.  (Scalar and LDS
    // loads share the lgkm counter and scalar ones return out of order, so a compiler wait
    // placed at the FMAs would drain the prefetch too; the sched_barriers keep hipcc from
    // hoisting every read of the chunk, which spilled.)
    f32x4 rw[3][7];                                     // ring: patch rows 2 rg + r, r = 0 .. 7
    f32x4 wc[7], wn[7];
    auto ldrow = [&](f32x4(&dst)[7], int r) {
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) dst[kx] = *reinterpret_cast<const f32x4*>(bp + (r * G::PP + kx) * G::PXB);
    };
    // the weight offset is laundered through an empty asm at each issue point: the loads are
    // loop-invariant, and hipcc otherwise hoists all 12 x 49 scalar loads to the kernel entry
    // and spills them through v_writelane (laundering the pointer itself loses its address
    // space: flat loads)
    auto ldw = [&](f32x4(&dst)[7], int ky) {
      if constexpr ((ABL & 2) != 0) {
#pragma unroll
        for (int kx = 0; kx < 7; ++kx) dst[kx] = bq * (float)(kx + ky);
        return;
      }
      int wo = ky * 7 * C + c;
      asm volatile("" : "+s"(wo));
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) dst[kx] = ld4(wp + wo + kx * C);
    };
    ldw(wc, 0);
    ldrow(rw[0], 0);
    ldrow(rw[1], 1);
#pragma unroll
    for (int ky = 0; ky < ((ABL & 4) ? 0 : 7); ++ky) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if (ky + 1 < 7) ldw(wn, ky + 1);
      if (ky + 2 <= 7) ldrow(rw[(ky + 2) % 3], ky + 2);
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) {
        acc[j][0] += rw[ky % 3][kx] * wc[kx];
        acc[j][1] += rw[(ky + 1) % 3][kx] * wc[kx];
      }
      // pin the step's FMAs here (IR passes otherwise sink them past every later load)
      asm volatile("" : "+v"(acc[j][0]), "+v"(acc[j][1]));
#pragma unroll
      for (int kx = 0; kx < 7; ++kx) wc[kx] = wn[kx];
      __builtin_amdgcn_sched_barrier(0);
    }
    sync();                                             // chunk j+1 landed, buffer j & 1 free
  }

  // ---- LayerNorm: per-pixel partial sums of the wave's channels, combined in wave order ----
  float* red = reinterpret_cast<float*>(smem);
  float mean[2], rstd[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < G::NCH; ++j) sm += (acc[j][t][0] + acc[j][t][1]) + (acc[j][t][2] + acc[j][t][3]);
    red[(wid * 64 + lane) * 2 + t] = sm;
  }
  sync();
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float sm = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) sm += red[(w * 64 + lane) * 2 + t];
    mean[t] = sm * (1.0f / C);
  }
  float* red2 = red + 8 * 64 * 2;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float qq = 0.f;
#pragma unroll
    for (int j = 0; j < G::NCH; ++j) {
      acc[j][t] -= mean[t];
#pragma unroll
      for (int e = 0; e < 4; ++e) qq = fmaf(acc[j][t][e], acc[j][t][e], qq);
    }
    red2[(wid * 64 + lane) * 2 + t] = qq;
  }
  sync();
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float qq = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) qq += red2[(w * 64 + lane) * 2 + t];
    rstd[t] = 1.0f / sqrtf(qq * (1.0f / C) + LN_EPS);
  }
#pragma unroll
  for (int j = 0; j < G::NCH; ++j) {
    const int c = 32 * j + 4 * wid;
    const f32x4 g = ld4(lnw + c), be = ld4(lnb + c);
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[j][t] = acc[j][t] * rstd[t] * g + be;
  }

  // ---- store through LDS: NST chunks per round, [chunk][tile pixel][32 ch], 16-B slot of
  // quad q at q ^ (px & 7) (conflict-free for the 8-lane groups of ds_write_b128) ----
  const int64_t img_px0 = (int64_t)b * H * W;
#pragma unroll
  for (int r0 = 0; r0 < G::NCH; r0 += G::NST) {
    sync();                                             // previous reads of smem done
#pragma unroll
    for (int jj = 0; jj < G::NST; ++jj) {
      if (r0 + jj < G::NCH) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int px = (2 * rg + t) * TWC + col;
          *reinterpret_cast<f32x4*>(smem + (jj * G::TPX + px) * 128 + 16 * (wid ^ (px & 7))) = acc[r0 + jj][t];
        }
      }
    }
    sync();
#pragma unroll
    for (int it = 0; it < 2 * G::NST; ++it) {
      const int e = it * G::NT + tid;                   // 16-B piece: chunk jj, pixel px, slot s
      const int jj = e >> 10, px = (e >> 3) & (G::TPX - 1), s = e & 7;
      if (r0 + jj >= G::NCH) continue;
      const int r = px / TWC, cl = px % TWC;
      const int oy = ty0 + r, ox = tx0 + cl;
      if (oy >= H || ox >= W) continue;
      const f32x4 v = *reinterpret_cast<const f32x4*>(smem + (jj * G::TPX + px) * 128 + 16 * s);
      const int c = 32 * (r0 + jj) + 4 * (s ^ (px & 7));
      const int64_t opix = img_px0 + (int64_t)oy * W + ox;
      if constexpr (S3) {
        __bf16* dst = reinterpret_cast<__bf16*>(yv) + opix * 2 * C + c;
        __bf16 hi[4], lo[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) split_bf16(v[q], hi[q], lo[q]);
        *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(hi);
        *reinterpret_cast<uint2*>(dst + C) = *reinterpret_cast<const uint2*>(lo);
      } else {
        st4(reinterpret_cast<float*>(yv) + opix * C + c, v);
      }
    }
  }
}

template <int C, int TWC, bool S3 = false, int ABL = 0>
inline int launch_dw_lds(const float* x, int B, int H, int W, const float* wp, const float* bias, const float* lnw,
                         const float* lnb, void* y, hipStream_t s) {
  using G = DwLdsGeo<C, TWC>;
  const int tx = (W + TWC - 1) / TWC, ty = (H + G::TH - 1) / G::TH;
  const int64_t n = (int64_t)tx * ty * B;
  if (n <= 0 || n >= (1LL << 31) || (int64_t)H * W * C >= (1LL << 31)) return PIPNET_ERR_ARG;
  hipLaunchKernelGGL((dwconv7_ln_lds_kernel<C, TWC, S3, ABL>), dim3((unsigned)n), dim3(G::NT), 0, s, x, H, W, wp, bias, lnw,
                     lnb, y, tx, ty);
  return hipGetLastError() == hipSuccess ? PIPNET_OK : PIPNET_ERR_LAUNCH;
}

}  // namespace pipnet_dw
