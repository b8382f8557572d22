// depthwise 7x7 + LayerNorm(C), row-ring formulation -- LAB ONLY (tools/dw_lab.hip); the product
// uses the register-tile kernel in count_pipnet_amd/csrc/convnext_dw.hpp.
//
// Each thread owns one channel pair (f32x2 -> v_pk_fma_f32) of a strip of TX adjacent output
// columns and walks DOWN a chunk of output rows.  Its 49 weight pairs live in registers for
// the whole walk; every input row of the chunk (plus its 6 halo rows) is read exactly once
// (TX + 6 loads) and scattered into the 7 output rows it touches, which are kept as a ring
// of 7 accumulator rows (slot = output row mod 7; the step loop is unrolled by 7 so every
// ring index is a compile-time register).  Per output channel this issues (TX+6)/TX *
// (RH+6)/RH loads instead of the 7 (TX+6)/TX input + 7 weight loads of the tile kernel in
// convnext_dw.hpp -- the tile kernel was bound by the L1 / TA request rate, not by HBM.
//
// A completed output row goes to an LDS ring buffer; every 7 steps the workgroup
// LayerNorms the buffered rows (LPP lanes per pixel, two-pass mean / variance as torch) and
// stores them coalesced.  A workgroup holds NS strips that need not be neighbours: strips
// are numbered over (image, strip column) so no workgroup is partly empty when W is not a
// multiple of NS*TX; row chunks are the fastest grid index, so the chunks that share halo
// rows run on one XCD (xcd_remap).  S3: the output is written as split-bf16 planes [hi|lo].
#pragma once
#include <algorithm>

#include "../count_pipnet_amd/csrc/common.hpp"

namespace pipnet_dw {

constexpr float RING_LN_EPS = 1e-6f;

// ABL (tools/dw_lab only): bit 1 skips the LayerNorm (raw conv rows stored), bit 2 skips the
// FMAs, bit 4 skips the input loads.
template <int C, int TX, int NS, int MINB, bool S3, int LPP, int ABL = 0>
__global__ __launch_bounds__(NS * C / 2, MINB) void dwconv7_ln_ring_kernel(
    const float* __restrict__ x, int B, int H, int W, int RH, int nchunk, const float* __restrict__ wp,
    const float* __restrict__ bias, const float* __restrict__ lnw, const float* __restrict__ lnb,
    void* __restrict__ yv) {
  constexpr int CP = C / 2;           // channel pairs = threads per strip
  constexpr int NT = NS * CP;
  constexpr int NP = NS * TX;         // pixels of one buffered output row
  constexpr int CS = C + 4;           // LDS pixel stride (floats): staggers strips over banks
  constexpr int NR = TX + 6;          // input columns per strip row
  __shared__ __attribute__((aligned(16))) float buf[7 * NP * CS];

  const int tid = threadIdx.x;
  const int cp = tid % CP, s = tid / CP;
  const int nsx = (W + TX - 1) / TX;
  const int nstrip = B * nsx;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int rc = lin % nchunk;
  const int sg = lin / nchunk;
  const int r0 = rc * RH;
  const int nrows = min(RH, H - r0);

  const int gs = sg * NS + s;
  const bool sval = gs < nstrip;
  const int b = sval ? gs / nsx : 0;
  const int x0 = (sval ? gs - b * nsx : 0) * TX;

  f32x2 w[49];
#pragma unroll
  for (int k = 0; k < 49; ++k) w[k] = *reinterpret_cast<const f32x2*>(wp + k * C + 2 * cp);
  const f32x2 bq = *reinterpret_cast<const f32x2*>(bias + 2 * cp);

  // 32-bit element offsets from the uniform base x (the launcher splits the batch so that
  // one launch spans < 2^31 elements): global_load ... v_off, s[x] -- no 64-bit VGPR addresses
  const uint32_t pix0 = (uint32_t)b * H * W;
  const int xs = x0 - 3;

  // raw loads (clamped column); the zeroing of out-of-image columns is applied when the row
  // is consumed, so that a prefetch does not wait on its own loads
  bool cok[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) cok[r] = (unsigned)(xs + r) < (unsigned)W;
  // unconditional (row clamped): a load under a branch makes the compiler wait for it at
  // the join; rows outside the image are loaded but never accumulated
  auto load_row = [&](int iy, f32x2 (&v)[NR]) {
    if constexpr ((ABL & 4) != 0) {
#pragma unroll
      for (int r = 0; r < NR; ++r) v[r] = f32x2{(float)iy, 1.f};
      return;
    }
    const uint32_t rowoff = (pix0 + (uint32_t)min(max(iy, 0), H - 1) * W) * C + 2 * cp;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const uint32_t off = rowoff + (uint32_t)min(max(xs + r, 0), W - 1) * C;
      v[r] = *reinterpret_cast<const f32x2*>(x + off);
    }
  };

  f32x2 acc[7][TX];
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int i = 0; i < TX; ++i) acc[k][i] = bq;

  const int nsteps = nrows + 6;                     // input rows r0-3 .. r0+nrows+2
  f32x2 vc[NR], vn[NR];
  load_row(r0 - 3, vn);
#pragma unroll
  for (int r = 0; r < NR; ++r) vc[r] = cok[r] ? vn[r] : f32x2{0.f, 0.f};

  constexpr int PPW = 64 / LPP;
  constexpr int CJ = (C + LPP - 1) / LPP;
  const int lane = tid & 63, wv = tid >> 6;
  const int sub = lane / LPP, sl = lane % LPP;

  for (int j0 = 0; j0 < nsteps; j0 += 7) {
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int j = j0 + u;
      const int iy = r0 - 3 + j;
      load_row(iy + 1, vn);                         // prefetch the next input row
      if ((ABL & 2) == 0 && j < nsteps && iy >= 0 && iy < H) {
#pragma unroll
        for (int ky = 0; ky < 7; ++ky) {
          const int o = j - ky;                     // output row fed by kernel row ky
          if (o < 0 || o >= nrows) continue;
          const int slot = (u - ky + 7) % 7;        // compile-time after unrolling
#pragma unroll
          for (int kx = 0; kx < 7; ++kx) {
#pragma unroll
            for (int px = 0; px < TX; ++px)
              acc[slot][px] = __builtin_elementwise_fma(vc[px + kx], w[ky * 7 + kx], acc[slot][px]);
          }
        }
      }
      {                                              // output row j - 6 is complete
        const int o = j - 6;
        const int slot = (u + 1) % 7;
        if (o >= 0 && o < nrows) {
#pragma unroll
          for (int px = 0; px < TX; ++px)
            *reinterpret_cast<f32x2*>(buf + (slot * NP + s * TX + px) * CS + 2 * cp) = acc[slot][px];
        }
#pragma unroll
        for (int px = 0; px < TX; ++px) acc[slot][px] = bq;
      }
#pragma unroll
      for (int r = 0; r < NR; ++r) vc[r] = cok[r] ? vn[r] : f32x2{0.f, 0.f};
    }
    __syncthreads();
    // LayerNorm + store of the rows completed in this group: o in [j0-6, j0] ∩ [0, nrows)
    const int oa = max(j0 - 6, 0), ob = min(j0 + 1, nrows);
    const int npx = (ob - oa) * NP;
    if constexpr ((ABL & 1) != 0) {
      for (int ro = oa; ro < ob; ++ro)
#pragma unroll
        for (int px = 0; px < TX; ++px)
          if (sval && x0 + px < W)
            *reinterpret_cast<f32x2*>(reinterpret_cast<float*>(yv) + ((int64_t)(pix0 + (r0 + ro) * W + x0 + px)) * C +
                                      2 * cp) = *reinterpret_cast<const f32x2*>(buf + ((ro % 7) * NP + s * TX + px) * CS + 2 * cp);
      __syncthreads();
      continue;
    }
    for (int base = wv * PPW; base < npx; base += (NT / 64) * PPW) {
      const int pp = base + sub;
      const int ro = oa + pp / NP, p = pp % NP;
      const int slot = ro % 7;
      const int gs2 = sg * NS + p / TX;
      const int b2 = gs2 / nsx;
      const int ox = (gs2 - b2 * nsx) * TX + p % TX;
      const bool ok = pp < npx && gs2 < nstrip && ox < W;   // lane-group uniform; all lanes shuffle
      const float* src = buf + (slot * NP + p) * CS;
      float vv[CJ];
      float sm = 0.f;
#pragma unroll
      for (int jj = 0; jj < CJ; ++jj) {
        const int c = sl + LPP * jj;
        vv[jj] = (ok && c < C) ? src[c] : 0.f;
        sm += vv[jj];
      }
#pragma unroll
      for (int o = LPP / 2; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
      const float mean = sm * (1.0f / C);
      float qq = 0.f;
#pragma unroll
      for (int jj = 0; jj < CJ; ++jj) {
        const int c = sl + LPP * jj;
        const float d = (c < C) ? vv[jj] - mean : 0.f;
        qq = fmaf(d, d, qq);
      }
#pragma unroll
      for (int o = LPP / 2; o > 0; o >>= 1) qq += __shfl_xor(qq, o, 64);
      const float rstd = 1.0f / sqrtf(qq * (1.0f / C) + RING_LN_EPS);
      if (!ok) continue;
      const int64_t opix = ((int64_t)b2 * H + r0 + ro) * W + ox;
      if constexpr (S3) {
        __bf16* dst = reinterpret_cast<__bf16*>(yv) + opix * 2 * C;
#pragma unroll
        for (int jj = 0; jj < CJ; ++jj) {
          const int c = sl + LPP * jj;
          if (c < C) {
            __bf16 hi, lo;
            split_bf16((vv[jj] - mean) * rstd * lnw[c] + lnb[c], hi, lo);
            dst[c] = hi;
            dst[C + c] = lo;
          }
        }
      } else {
        float* dst = reinterpret_cast<float*>(yv) + opix * C;
#pragma unroll
        for (int jj = 0; jj < CJ; ++jj) {
          const int c = sl + LPP * jj;
          if (c < C) dst[c] = (vv[jj] - mean) * rstd * lnw[c] + lnb[c];
        }
      }
    }
    __syncthreads();
  }
}

// Row chunking: rows per chunk RH so that the grid has at least ~min_wg workgroups, but no
// chunk shorter than min_rh rows (each chunk re-reads 6 halo rows).  Batches spanning 2^31
// elements or more go out in slices (the kernel's 32-bit offsets).
template <int C, int TX, int NS, int MINB, bool S3, int LPP, int ABL = 0>
inline int launch_dw_ring(const float* x, int B, int H, int W, const float* wp, const float* bias, const float* lnw,
                          const float* lnb, void* y, hipStream_t s, int min_wg = 2048, int min_rh = 7) {
  const int64_t img = (int64_t)H * W * C;
  if (img >= 0x7fffffff) return PIPNET_ERR_ARG;
  const int bmax = (int)std::min<int64_t>(B, 0x7fffffff / img);
  for (int b0 = 0; b0 < B; b0 += bmax) {
    const int nb = std::min(bmax, B - b0);
    const int nsx = (W + TX - 1) / TX;
    const int64_t ngroups = ((int64_t)nb * nsx + NS - 1) / NS;
    int nchunk = (int)std::min<int64_t>((min_wg + ngroups - 1) / ngroups, (H + min_rh - 1) / min_rh);
    nchunk = std::max(nchunk, 1);
    const int rh = (H + nchunk - 1) / nchunk;
    nchunk = (H + rh - 1) / rh;
    const int64_t grid = ngroups * nchunk;
    if (grid <= 0 || grid > 0x7fffffff) return PIPNET_ERR_ARG;
    void* yb = S3 ? (void*)(reinterpret_cast<__bf16*>(y) + b0 * img * 2) : (void*)(reinterpret_cast<float*>(y) + b0 * img);
    hipLaunchKernelGGL((dwconv7_ln_ring_kernel<C, TX, NS, MINB, S3, LPP, ABL>), dim3((unsigned)grid), dim3(NS * C / 2), 0,
                       s, x + b0 * img, nb, H, W, rh, nchunk, wp, bias, lnw, lnb, yb);
    if (hipGetLastError() != hipSuccess) return PIPNET_ERR_LAUNCH;
  }
  return PIPNET_OK;
}

}  // namespace pipnet_dw
