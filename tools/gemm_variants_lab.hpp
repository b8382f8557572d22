// Lab-only fp32 GEMM variants (tools/gemm_lab.hip; never part of the product library): the
// persistent 128x128 tile and the streaming persistent tile with deferred epilogues.  Both are
// bitwise the product tile and measured 3-7 % slower on the C2 shapes (profiles/r01/
// gemm_lab_persistent.txt, profiles/r03/gemm_stream_ab.txt); kept here as the record of those
// A/B runs and as a starting point for the next persistent design.
#pragma once
#include "../count_pipnet_amd/csrc/gemm_f32_impl.hpp"

namespace pipnet_gemm {

// ======================================================================================
// Persistent form of the 128x128 / BK 32 / 2-stage tile (dense A, N % 128 == 0, float4
// epilogue).  Two workgroups per CU walk tiles blockIdx.x, +gridDim.x, ... of the same
// XCD-grouped raster.  After a tile's last K-tile every wave has passed the loop's final
// barrier, so both stages are free: the next tile's K-tile 0 is issued into stage 0 BEFORE
// this tile's epilogue, which re-lays the accumulators through stage 1 with wave-local
// ordering only (each wave owns 8 KiB of it; no workgroup barrier inside the epilogue).  The
// epilogue's LDS accesses are inline asm: hipcc cannot tell that they miss the LDS-DMA's
// stage and would otherwise drain that DMA (vmcnt(0)) before the first of them.  The bias /
// scale / residual loads are issued before that DMA, and every lane stores exactly TM * 8
// float4s (rows past M are clamped to row M-1, whose values they recompute from the clamped
// A row -- identical bits), so one vmcnt(TM * 8) retires the next tile's K-tile 0 without
// waiting for the stores.  What this removes per tile: the workgroup launch, the first
// K-tile's load latency and the store drain of a retiring workgroup -- the per-tile gaps the
// stamps saw as 1.76-1.88 resident workgroups per CU (of 2) on the stage-3/4 fc1 shapes.
// ======================================================================================
PIPNET_DEV void tile_coords_id(const GemmParams& p, int id, int bm, int& m0, int& n0) {
  const int nwg = p.mt * p.nt;
  const int tile = xcd_remap(id, nwg);
  const int gm = p.group_m;
  const int group = tile / (gm * p.nt);
  const int first_m = group * gm;
  const int gsz = min(p.mt - first_m, gm);
  const int in_group = tile - group * gm * p.nt;
  m0 = (first_m + in_group % gsz) * bm;
  n0 = (in_group / gsz) * BN;
}

PIPNET_DEV unsigned lds_u32(const float* ptr) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) float*)ptr;
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_f32_tn_persist_kernel(GemmParams p) {
  constexpr int BK = 32, TM = 2;
  using G = Geo<BK, TM>;
  constexpr bool HAS_R = EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_MUL || EPI == PIPNET_EPI_BIAS_RESID_RELU ||
                         EPI == PIPNET_EPI_RESID_ROWSCALE || EPI == PIPNET_EPI_GELU_BWD;
  __shared__ __attribute__((aligned(16))) float smem[2 * G::TILE_FLOATS];
  static_assert(G::TILE_FLOATS >= 4 * 32 * 64, "epilogue region = one stage");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int nk = p.K / BK;
  const int ntiles = p.mt * p.nt;
  const int drow = lane / G::CHUNKS;
  const float* asrc[G::A_DMA];
  const float* wsrc[G::B_DMA];
  auto setup = [&](int id, int& m0, int& n0) {
    tile_coords_id(p, id, G::BMT, m0, n0);
#pragma unroll
    for (int i = 0; i < G::A_DMA; ++i) {
      const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + drow;
      asrc[i] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + 4 * G::swz(row, lane % G::CHUNKS);
    }
#pragma unroll
    for (int i = 0; i < G::B_DMA; ++i) {
      const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + drow;
      wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + 4 * G::swz(row, lane % G::CHUNKS);
    }
  };
  auto stage = [&](int kt, int buf) {
    float* base = smem + buf * G::TILE_FLOATS;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < G::A_DMA; ++i) dma16(asrc[i] + k0, base + (i * NWAVES + wid) * G::ROWS_PER_DMA * BK);
#pragma unroll
    for (int i = 0; i < G::B_DMA; ++i)
      dma16(wsrc[i] + k0, base + G::BMT * BK + (i * NWAVES + wid) * G::ROWS_PER_DMA * BK);
  };

  int id = blockIdx.x, m0, n0;
  setup(id, m0, n0);
  stage(0, 0);
  __syncthreads();
  const int c4 = lane & 15;
  // this wave's 8 KiB of stage 1: MFMA-layout writes at (row (v&3) + 8 (v>>2) + 4 lh, column
  // j*32 + lr), float4 reads of row it*4 + (lane>>4), columns 4 c4 .. +3
  const unsigned wt = lds_u32(smem + G::TILE_FLOATS + wid * 32 * 64);
  const unsigned wa = wt + (unsigned)((4 * lh * 64 + lr) * 4);
  const unsigned ra = wt + (unsigned)(((lane >> 4) * 64 + 4 * c4) * 4);
  for (;;) {
    Acc acc;
    zero_acc(acc);
    {
      Frag fa, fb;
      read_frag<BK, TM>(fa, smem, wm, wn, lr, lh, 0);
      int cur = 0;
      for (int kt = 0; kt < nk; ++kt) {
        const float* buf = smem + cur * G::TILE_FLOATS;
        if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
        read_frag<BK, TM>(fb, buf, wm, wn, lr, lh, 1);
        mfma_frag<TM>(acc, fa);
        read_frag<BK, TM>(fa, buf, wm, wn, lr, lh, 2);
        mfma_frag<TM>(acc, fb);
        read_frag<BK, TM>(fb, buf, wm, wn, lr, lh, 3);
        mfma_frag<TM>(acc, fa);
        __syncthreads();                                 // tile kt+1 landed, tile kt read
        if (kt + 1 < nk) read_frag<BK, TM>(fa, smem + (cur ^ 1) * G::TILE_FLOATS, wm, wn, lr, lh, 0);
        mfma_frag<TM>(acc, fb);
        cur ^= 1;
      }
    }
    // ---- this tile's epilogue operands, then the next tile's K-tile 0, then the epilogue ----
    const int cm0 = m0;
    const int n = n0 + wn * 64 + 4 * c4;
    f32x4 bn = {0.f, 0.f, 0.f, 0.f}, sn = {1.f, 1.f, 1.f, 1.f};
    if (EPI != PIPNET_EPI_NONE && EPI != PIPNET_EPI_MUL && EPI != PIPNET_EPI_GELU_BWD && p.bias) bn = ld4(p.bias + n);
    if ((EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_RESID_ROWSCALE) && p.scale) sn = ld4(p.scale + n);
    // bias / scale in registers before the DMA below: hipcc waits vmcnt(0) for any load still
    // pending behind an LDS-DMA, which would drain the next tile's K-tile 0 here
    asm volatile("" : "+v"(bn), "+v"(sn));
    f32x4 r[TM][8];
    if (HAS_R) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int m = min(cm0 + wm * 32 * TM + i * 32 + it * 4 + (lane >> 4), p.M - 1);
          r[i][it] = ld4(p.R + (int64_t)m * p.ldr + n);
        }
    }
    id += gridDim.x;
    const bool more = id < ntiles;
    // issued unconditionally (the last tile re-fetches its own K-tile 0, unused) so the number
    // of VMEM ops in flight is the same on every path and hipcc's own waits for the epilogue
    // operands above stay counted instead of falling back to vmcnt(0)
    setup(more ? id : id - gridDim.x, m0, n0);
    stage(0, 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          asm volatile("ds_write_b32 %0, %1 offset:%2" ::"v"(wa), "v"(acc[i][j][v]),
                       "i"((((v & 3) + 8 * (v >> 2)) * 64 + j * 32) * 4)
                       : "memory");
      f32x4 x[8];
#pragma unroll
      for (int it = 0; it < 8; ++it)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(x[it]) : "v"(ra), "i"(it * 4 * 64 * 4) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int m = min(cm0 + wm * 32 * TM + i * 32 + it * 4 + (lane >> 4), p.M - 1);
        float rs = 1.f;
        if constexpr (EPI == PIPNET_EPI_RESID_ROWSCALE) rs = p.row_scale[m / p.rows_per_scale];
        st4_c(p.C + (int64_t)m * p.ldc + n, epi_math<EPI>(x[it], bn, sn, HAS_R ? r[i][it] : bn, rs));
      }
    }
    if (!more) break;
    // K-tile 0 of the next tile is older than exactly TM * 8 stores; every wave is done with
    // its epilogue reads of stage 1 (lgkmcnt(0) above) before the barrier
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(TM * 8) : "memory");
  }
}

// ======================================================================================
// Streaming persistent form of the 128x128 / BK 32 / 2-stage tile, with the epilogue of
// each tile deferred into the main loop of the next (dense A, N % 128 == 0, K >= 256).
//
// The stamps of the product tile (profiles/r01/gemm_stamps.txt) put 15-27 % of a workgroup's
// time on the fc1 shapes in its epilogue (GELU + 64 KiB of stores), during which the CU's
// other workgroup runs alone -- one wave per SIMD, which paces the MFMA pipe at ~2/3
// (6,079 instead of 4,096 cycles per K-tile).  Here two workgroups per CU walk tiles
// blockIdx.x, +gridDim.x, ... as ONE stream of K-tiles: the LDS-DMA of the next K-tile is
// issued one iteration ahead whether or not it belongs to the next tile, so there is no
// prologue per tile; when a tile's last K-tile is multiplied its accumulators move to a
// second register set and the next tile starts at once.  The finished tile leaves in 8
// slices of 8 values per lane, one slice per K-tile of the next tile, written straight from
// the MFMA layout (lane = column, 2 rows x 128 B per store instruction: whole cache lines)
// right after the K-tile's barrier, so the epilogue math runs under the last MFMA group and
// the stores drain under the following K-tile.  The residual operand of a slice is loaded
// at the start of its K-tile (the barrier's vmcnt(0) has retired it by the time it is used).
// Results are bitwise those of gemm_f32_tn_kernel<32, 2, ...>: same K order, same MFMA
// sequence per tile, same epilogue arithmetic (gelu_pk16 on the same pairs of values).
// ======================================================================================
template <int EPI>
PIPNET_DEV float epi_scalar(float x, float bn, float sn, float r) {
  if (EPI == PIPNET_EPI_BIAS) x = x + bn;
  if (EPI == PIPNET_EPI_RESID) x = fmaf(sn, x + bn, r);          // = epi_math's vector fma
  if (EPI == PIPNET_EPI_MUL) x = x * r;
  if (EPI == PIPNET_EPI_BIAS_RELU) x = fmaxf(x + bn, 0.f);
  if (EPI == PIPNET_EPI_BIAS_RESID_RELU) x = fmaxf(x + bn + r, 0.f);
  if (EPI == PIPNET_EPI_GELU_BWD) x = x * gelu_grad(r);
  return x;
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_f32_tn_stream_kernel(GemmParams p) {
  constexpr int BK = 32, TM = 2, NSLICE = 8, SV = 8;      // 8 slices of 8 values per lane
  using G = Geo<BK, TM>;
  constexpr bool HAS_R = EPI == PIPNET_EPI_RESID || EPI == PIPNET_EPI_MUL || EPI == PIPNET_EPI_BIAS_RESID_RELU ||
                         EPI == PIPNET_EPI_GELU_BWD;
  constexpr bool HAS_B = EPI != PIPNET_EPI_NONE && EPI != PIPNET_EPI_MUL && EPI != PIPNET_EPI_GELU_BWD;
  __shared__ __attribute__((aligned(16))) float smem[2 * G::TILE_FLOATS];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int nk = p.K / BK;                        // >= NSLICE (host guarantees)
  const int ntiles = p.mt * p.nt;
  const int mytiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int drow = lane / G::CHUNKS;
  // DMA sources as 32-bit element offsets from the (uniform) A / W bases: half the VGPRs of
  // 64-bit pointers, which the second accumulator set needs (host: M*lda, N*K < 2^31)
  uint32_t aoff[G::A_DMA], woff[G::B_DMA];
  auto setup = [&](int t, int& m0, int& n0) __attribute__((always_inline)) {
    tile_coords_id(p, (int)blockIdx.x + t * (int)gridDim.x, G::BMT, m0, n0);
#pragma unroll
    for (int i = 0; i < G::A_DMA; ++i) {
      const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + drow;
      aoff[i] = (uint32_t)(min(m0 + row, p.M - 1) * (int)p.lda + 4 * G::swz(row, lane % G::CHUNKS));
    }
#pragma unroll
    for (int i = 0; i < G::B_DMA; ++i) {
      const int row = (i * NWAVES + wid) * G::ROWS_PER_DMA + drow;
      woff[i] = (uint32_t)((n0 + row) * p.K + 4 * G::swz(row, lane % G::CHUNKS));
    }
  };
  auto stage = [&](int kt, int buf) __attribute__((always_inline)) {
    float* base = smem + buf * G::TILE_FLOATS;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < G::A_DMA; ++i) dma16(p.A + (aoff[i] + k0), base + (i * NWAVES + wid) * G::ROWS_PER_DMA * BK);
#pragma unroll
    for (int i = 0; i < G::B_DMA; ++i)
      dma16(p.W + (woff[i] + k0), base + G::BMT * BK + (i * NWAVES + wid) * G::ROWS_PER_DMA * BK);
  };

  // The finished tile waiting for its epilogue.  A lane's values of slice q = (i, j, half h of
  // v) sit in rows prow + i*32 + (v&3) + 8(v>>2) (prow = tile row + wm*64 + 4 lh) of column
  // pcol + j*32.  Addresses are 32-bit element offsets (coff / roff, one VGPR each) plus
  // wave-uniform row offsets; both are laundered through an empty asm at each use so the
  // compiler cannot hoist the 64 per-store addresses out of the loop (it did, and spilled them).
  uint32_t coff = 0, roff = 0;
  int prow = 0;
  float pb[2] = {0.f, 0.f}, ps[2] = {1.f, 1.f};
  float rv[SV];
  auto park = [&](int pm0, int pn0) __attribute__((always_inline)) {
    prow = pm0 + wm * 64 + 4 * lh;
    const int pcol = pn0 + wn * 64 + lr;
    coff = (uint32_t)(prow * (int)p.ldc + pcol);
    if (HAS_R) roff = (uint32_t)(prow * (int)p.ldr + pcol);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (HAS_B && p.bias) pb[j] = p.bias[pcol + j * 32];
      if ((EPI == PIPNET_EPI_RESID) && p.scale) ps[j] = p.scale[pcol + j * 32];
    }
  };
  auto vrow = [](int q, int e) __attribute__((always_inline)) {
    return (q >> 2) * 32 + (((q & 1) * SV + e) & 3) + 8 * (((q & 1) * SV + e) >> 2);
  };
  auto load_r = [&](auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    uint32_t ro = roff;
    int pr = prow;
    asm volatile("" : "+v"(ro), "+v"(pr));
#pragma unroll
    for (int e = 0; e < SV; ++e) {
      const int rr = vrow(q, e);
      // rows past M read row M-1 (never stored)
      const int rcl = pr + rr < p.M ? rr : p.M - 1 - pr;
      rv[e] = p.R[ro + (uint32_t)(rcl * (int)p.ldr + ((q >> 1) & 1) * 32)];
    }
  };
  auto store_slice = [&](const Acc& pend, auto qc) __attribute__((always_inline)) {
    constexpr int q = decltype(qc)::value;
    constexpr int i = q >> 2, j = (q >> 1) & 1, v0 = (q & 1) * SV;
    float x[SV];
    if constexpr (EPI == PIPNET_EPI_BIAS_GELU) {
#pragma unroll
      for (int e = 0; e < SV; e += 2) {
        const f32x2 g = gelu_pk16(f32x2{pend[i][j][v0 + e] + pb[j], pend[i][j][v0 + e + 1] + pb[j]});
        x[e] = g[0];
        x[e + 1] = g[1];
      }
    } else {
#pragma unroll
      for (int e = 0; e < SV; ++e) x[e] = epi_scalar<EPI>(pend[i][j][v0 + e], pb[j], ps[j], HAS_R ? rv[e] : 0.f);
    }
    uint32_t co = coff;
    int pr = prow;
    asm volatile("" : "+v"(co), "+v"(pr));
#pragma unroll
    for (int e = 0; e < SV; ++e) {
      const int rr = vrow(q, e);
      if (pr + rr < p.M) __builtin_nontemporal_store(x[e], p.C + (co + (uint32_t)(rr * (int)p.ldc + j * 32)));
    }
  };
  // wave-uniform dispatch to a compile-time slice index
  auto for_slice = [&](int q, auto fn) __attribute__((always_inline)) {
    if (q == 0) fn(IntC<0>{});
    else if (q == 1) fn(IntC<1>{});
    else if (q == 2) fn(IntC<2>{});
    else if (q == 3) fn(IntC<3>{});
    else if (q == 4) fn(IntC<4>{});
    else if (q == 5) fn(IntC<5>{});
    else if (q == 6) fn(IntC<6>{});
    else if (q == 7) fn(IntC<7>{});
  };

  int m0, n0;
  setup(0, m0, n0);
  stage(0, 0);
  __syncthreads();
  Frag fa, fb;
  read_frag<BK, TM>(fa, smem, wm, wn, lr, lh, 0);
  int cur = 0;
  // One tile: multiply into acc (K-tiles 0..nk-1, the DMA stream running one K-tile ahead,
  // into the next tile at the end) while pend's slices leave in K-tiles 0..7.  Called with
  // the two register sets alternating, so neither is ever copied.
  auto tile = [&](Acc& acc, const Acc& pend, bool have_pend, int t) __attribute__((always_inline)) {
    zero_acc(acc);
    const bool last = t + 1 == mytiles;
    int nm0 = m0, nn0 = n0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk || !last;
      if (kt + 1 < nk) {
        stage(kt + 1, cur ^ 1);
      } else if (!last) {
        setup(t + 1, nm0, nn0);
        stage(0, cur ^ 1);
      }
      const bool do_slice = have_pend && kt < NSLICE;
      if (HAS_R && do_slice) for_slice(kt, load_r);
      const float* buf = smem + cur * G::TILE_FLOATS;
      read_frag<BK, TM>(fb, buf, wm, wn, lr, lh, 1);
      mfma_frag<TM>(acc, fa);
      read_frag<BK, TM>(fa, buf, wm, wn, lr, lh, 2);
      mfma_frag<TM>(acc, fb);
      read_frag<BK, TM>(fb, buf, wm, wn, lr, lh, 3);
      mfma_frag<TM>(acc, fa);
      __syncthreads();                            // next K-tile landed, this one read, slice operands retired
      if (more) read_frag<BK, TM>(fa, smem + (cur ^ 1) * G::TILE_FLOATS, wm, wn, lr, lh, 0);
      mfma_frag<TM>(acc, fb);
      if (do_slice) {
        __builtin_amdgcn_sched_barrier(0);
        for_slice(kt, [&](auto qc) __attribute__((always_inline)) { store_slice(pend, qc); });
        __builtin_amdgcn_sched_barrier(0);
      }
      cur ^= 1;
    }
    park(m0, n0);
    m0 = nm0;
    n0 = nn0;
  };
  auto drain = [&](const Acc& pend) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NSLICE; ++q)
      for_slice(q, [&](auto qc) __attribute__((always_inline)) {
        if (HAS_R) load_r(qc);
        store_slice(pend, qc);
      });
  };
  Acc acc, pend;
  for (int t = 0; t < mytiles; ++t) {
    tile(acc, pend, t > 0, t);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) pend[i][j] = acc[i][j];
  }
  drain(pend);
}

}  // namespace pipnet_gemm
