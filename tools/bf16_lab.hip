// Tuning lab for the bf16 GEMM tiles (not part of the product library): the product's
// ping-pong kernel (gemm_bf16_impl.hpp) instantiated with its ABL ablation switches on a
// dense GEMM C[M][N] = A[M][K] W[N][K]^T (bf16 in / out, fp32 accumulation).
// Built by tools/bf16_lab.py into tools/libbf16_lab.so.
#include "../count_pipnet_amd/csrc/gemm_bf16_impl.hpp"

using namespace pipnet_bf16;

namespace pipnet_bf16 {
// Lab-only kernel (measured, not adopted: profiles/r02/bf16_lab.txt): ABL bits as the product
// kernel's, plus 16 = every DMA re-reads K-tile 0 (cache-hot sources), 32 = no A DMA (B only).
// ======================================================================================
// 256x256 ping-pong tile with 64-deep K-tiles in full 128-B LDS rows (tile 8).
//
// Same wave roles as conv_bf16_pp_kernel (8 waves = 2 row groups x 4 column blocks, wave
// (wr, wc) owns rows wr*128.., cols wc*64.. as 8 x 4 MFMA 16x16 tiles, group 1 one barrier
// behind group 0) but every LDS-DMA piece moves 8 whole 128-B lines (8 rows x 64 k) instead
// of 16 half lines: half the TA / L2 requests per byte (cdna_hip_programming.md 5, x through
// LDS in full lines).  A K-tile is four PHASES of 16 MFMAs, ordered so that the operands
// free up early:
//     q0 = (rows r0, k 0..31)   reads B[k0] (4) + A[r0,k0] (4)
//     q1 = (rows r0, k 32..63)  reads B[k1] (4) + A[r0,k1] (4)
//     q2 = (rows r1, k 0..31)   reads A[r1,k0] (4), B[k0] kept in registers
//     q3 = (rows r1, k 32..63)  reads A[r1,k1] (4), B[k1] kept in registers
// (r0 / r1 = the first / last 64 rows of a wave's 128).  So B and the r0 A rows of K-tile t
// are dead after phase q1 of t, the r1 A rows after q3.  Two LDS stages of 64 KiB (tile t in
// stage t & 1) then give each piece a long flight: per wave and phase one 2-piece item,
//     (t,0): A_r0(t+1)   (t,1): A_r1(t+1)   (t,2): B(t+2) first half   (t,3): B(t+2) second half
// -- B(t+2) lands in stage t & 1 once B(t) is dead, A(t+1) in the other stage once K-tile t-1
// is dead.  Waits (counted vmcnt, in the load segment, after that phase's DMA issue):
//     (t-1,3): B(t), A_r0(t)    younger: A_r1(t), B(t+1) x2          -> 6 (2 if t+1 = nk)
//     (t,1)  : A_r1(t)          younger: B(t+1) x2, A_r0/A_r1(t+1)   -> 8 (0 if t+1 = nk)
// Every load segment ends with lgkmcnt(0) before its barrier, so a region's last reads have
// completed at the barrier after which the next DMA into it is issued (WAR), and every
// wave's wait precedes a barrier that the readers pass (RAW; group 1 one barrier later).
// Swizzle: logical 16-B chunk c of row r at physical chunk c ^ (r & 7): conflict-free for
// the 16x16x32 fragment reads (lane l: row l & 15, chunk 4 s + (l >> 4)); the DMA writes
// lane-linear, so the inverse is applied to its source address.
// Requirements: K % 64 == 0 (packed weights), Cin % 64 == 0 for the implicit conv (a K-tile
// never straddles two taps), N % 8 == 0.
// ======================================================================================
namespace p64 {
constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int ROWB = 128;                                     // one LDS row = 64 bf16
constexpr int A_BYTES = BM * ROWB, STAGE_BYTES = (BM + BN) * ROWB;   // 32 + 32 KiB
constexpr int SMEM_BYTES = 2 * STAGE_BYTES > pp::EPI_BYTES ? 2 * STAGE_BYTES : pp::EPI_BYTES;
}  // namespace p64

template <int EPI, int ALOAD, int ABL = 0, int CPA = 0, int CPB = 0>   // CPA / CPB: cache-policy bits of the A / B LDS-DMA
__global__ __launch_bounds__(p64::NT, 1) void conv_bf16_p64_kernel(ConvParams p) {
  using namespace p64;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  tile_coords(p, BM, BN, m0, n0);
  const int nk = p.K / BK;

  // ---- DMA: lane L of a piece writes row (L >> 3) of its 8, physical chunk L & 7 ----
  const int drow = lane >> 3;
  const int dchunk = 8 * ((lane & 7) ^ drow);                  // logical chunk (elements); row & 7 = drow
  // A pieces of this wave: r0 rows = pieces wid, 16 + wid; r1 rows = pieces 8 + wid, 24 + wid
  ARow ar[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int piece = (i & 1) * 8 + (i >> 1) * 16 + wid;     // i: 0 = r0a, 1 = r1a, 2 = r0b, 3 = r1b
    ar[i] = a_row<ALOAD>(p, min(m0 + 8 * piece + drow, p.M - 1));
  }
  // B pieces of this wave: wid, 8 + wid (first half), 16 + wid, 24 + wid (second half)
  const bf16* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wsrc[i] = p.W + (int64_t)min(n0 + 8 * (8 * i + wid) + drow, p.N - 1) * p.K + dchunk;
  // (tap, channel) of the A K-tile being staged (both of its items), advanced after its r1 item
  int d_c = 0, d_kx = 0, d_ky = 0;
  auto a_src = [&](const ARow& r, int k0) -> const void* {
    if (k0 >= p.Kv) return g_zero_bf;
    if (ALOAD == ALOAD_DENSE) return p.A + r.base + seg_remap(p, k0) + dchunk;
    const int iy = r.iy0 + d_ky, ix = r.ix0 + d_kx;
    if ((unsigned)iy >= (unsigned)p.H || (unsigned)ix >= (unsigned)p.Wd) return g_zero_bf;
    return p.A + r.base + ((int64_t)iy * p.Wd + ix) * p.Cinp + seg_remap(p, d_c) + dchunk;
  };
  auto dma = [&](const void* src, unsigned char* dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, CPA);
  };
  auto dmab = [&](const void* src, unsigned char* dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, CPB);
  };
  auto stage_a = [&](int kt, int half) {                      // half 0 = r0 rows, 1 = r1 rows
    if constexpr ((ABL & 1) != 0) return;
    unsigned char* base = smem + (kt & 1) * STAGE_BYTES;
    if constexpr ((ABL & 16) != 0) kt = 0;                    // lab: always the first K-tile (cache-hot)
    if constexpr ((ABL & 32) != 0) return;                    // lab: B operand only
    dma(a_src(ar[half], kt * BK), base + (half * 8 + wid) * 1024);
    dma(a_src(ar[2 + half], kt * BK), base + (half * 8 + 16 + wid) * 1024);
    if (half == 1 && ALOAD != ALOAD_DENSE) {
      d_c += BK;
      if (d_c == p.Cin) {
        d_c = 0;
        if (++d_kx == p.KW) d_kx = 0, ++d_ky;
      }
    }
  };
  auto stage_b = [&](int kt, int half) {                      // half 0 = pieces wid, 8 + wid
    if constexpr ((ABL & 1) != 0) return;
    unsigned char* base = smem + (kt & 1) * STAGE_BYTES + A_BYTES;
    if constexpr ((ABL & 16) != 0) kt = 0;
    dmab(wsrc[2 * half] + kt * BK, base + (16 * half + wid) * 1024);
    dmab(wsrc[2 * half + 1] + kt * BK, base + (16 * half + 8 + wid) * 1024);
  };
  // ---- fragments: lane reads row (l & 15) of a 16-row block, logical chunk 4 s + (l >> 4) ----
  const int fr = lane & 15;
  const int fofs0 = fr * ROWB + 16 * ((lane >> 4) ^ (fr & 7));          // k-step s = 0
  const int fofs1 = fr * ROWB + 16 * ((4 + (lane >> 4)) ^ (fr & 7));    // k-step s = 1
  auto read_a = [&](bf16x8v (&fa)[4], const unsigned char* st, int rh, int s) {
    if constexpr ((ABL & 8) != 0) {
      if (st != smem || rh != 0) return;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
      fa[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 128 + rh * 64 + r * 16) * ROWB + (s ? fofs1 : fofs0));
  };
  auto read_b = [&](bf16x8v (&fb)[4], const unsigned char* st, int s) {
    if constexpr ((ABL & 8) != 0) {
      if (st != smem) return;
    }
#pragma unroll
    for (int n = 0; n < 4; ++n)
      fb[n] = *reinterpret_cast<const bf16x8v*>(st + A_BYTES + (wc * 64 + n * 16) * ROWB + (s ? fofs1 : fofs0));
  };
  auto bar = [&]() {
    if constexpr ((ABL & 4) == 0) pp_barrier();
  };
  auto wait_vm = [&](int n) {
    if constexpr ((ABL & 32) != 0) {
      pp_wait_vm_dyn(n >= 8 ? 4 : (n >= 6 ? 4 : 0));          // lab: B-only counts (conservative)
    } else if constexpr ((ABL & 1) == 0) {
      pp_wait_vm_dyn(n);
    }
  };
  auto reads_done = [&]() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };

  f32x4v acc[8][4];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  auto mfma16 = [&](const bf16x8v (&fa)[4], const bf16x8v (&fb)[4], int rh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[rh * 4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[rh * 4 + r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: B(0), A_r0(0), A_r1(0), B(1) in flight; wait for B(0), A_r0(0)
  stage_b(0, 0), stage_b(0, 1), stage_a(0, 0), stage_a(0, 1);
  if (nk > 1) stage_b(1, 0), stage_b(1, 1);
  wait_vm(nk > 1 ? 6 : 2);
  reads_done();
  pp_barrier();
  if (wr == 1) pp_barrier();                                   // group 1 runs one barrier behind

  bf16x8v fa[4], fb0[4], fb1[4];
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* st = smem + (kt & 1) * STAGE_BYTES;
    const bool more = kt + 1 < nk;
    // ---- q0: rows r0, k 0..31; stage A_r0(kt+1) ----
    if (more) stage_a(kt + 1, 0);
    read_b(fb0, st, 0);
    read_a(fa, st, 0, 0);
    reads_done();
    bar();
    mfma16(fa, fb0, 0);
    bar();
    // ---- q1: rows r0, k 32..63; stage A_r1(kt+1); wait for A_r1(kt) ----
    if (more) stage_a(kt + 1, 1);
    read_b(fb1, st, 1);
    read_a(fa, st, 0, 1);
    wait_vm(more ? 8 : 0);
    reads_done();
    bar();
    mfma16(fa, fb1, 0);
    bar();
    // ---- q2: rows r1, k 0..31; stage B(kt+2) first half (B(kt) is dead) ----
    if (kt + 2 < nk) stage_b(kt + 2, 0);
    read_a(fa, st, 1, 0);
    reads_done();
    bar();
    mfma16(fa, fb0, 1);
    bar();
    // ---- q3: rows r1, k 32..63; stage B(kt+2) second half; wait for B(kt+1), A_r0(kt+1) ----
    if (kt + 2 < nk) stage_b(kt + 2, 1);
    read_a(fa, st, 1, 1);
    if (more) wait_vm(kt + 2 < nk ? 6 : 2);
    reads_done();
    bar();
    mfma16(fa, fb1, 1);
    bar();
  }
  if (wr == 0) pp_barrier();                                   // re-align the groups
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  pp_barrier();                                                // stage buffers free for the epilogue
  if constexpr ((ABL & 2) != 0) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) t += acc[r][n][i];
    reinterpret_cast<float*>(p.C)[(int64_t)blockIdx.x * p64::NT + tid] = t;
    return;
  }
  pp_epilogue<EPI, 4>(p, acc, smem, m0, n0, wr, wc, lane, wid);
}

}  // namespace pipnet_bf16


namespace pipnet_bf16 {
// Lab-only: the product ping-pong tile (conv_bf16_pp_kernel, DB = 2) with REGISTER staging
// instead of LDS-DMA: each phase ds_writes the 2 pieces it loaded (global_load_dwordx4) one
// K-tile earlier, then loads the next 2 -- B(t+2) written / B(t+3) loaded in phase 0 of K-tile
// t, A(t+3) / A(t+4) in phase 1.  Same LDS image (lane-linear pieces, swizzled source).
// Dense A only.  ABL: 2 = no epilogue.
template <int ABL>
__global__ __launch_bounds__(pp::NT, 1) void lab_prs_kernel(ConvParams p) {
  using namespace pp;
  constexpr int NS = 4, NB = 4, WCOLS = 64;
  __shared__ __attribute__((aligned(16))) unsigned char smem[smem_bytes<2>()];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  tile_coords(p, BM, 4 * WCOLS, m0, n0);
  const int nk = p.K / BK;
  const int drow = lane >> 2;
  const int dchunk = 8 * ((lane & 3) ^ g(drow));
  const bf16* asrc[2];
  const bf16* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (wid + 8 * i) + drow;
    asrc[i] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + dchunk;
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + dchunk;
  }
  bf16x8v ra[2], rb[2];
  auto load_a = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) ra[i] = *reinterpret_cast<const bf16x8v*>(asrc[i] + kt * BK);
  };
  auto load_b = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) rb[i] = *reinterpret_cast<const bf16x8v*>(wsrc[i] + kt * BK);
  };
  auto write_a = [&](int kt) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<bf16x8v*>(base + (wid + 8 * i) * 1024 + lane * 16) = ra[i];
  };
  auto write_b = [&](int kt) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES + BM * ROWB;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<bf16x8v*>(base + (wid + 8 * i) * 1024 + lane * 16) = rb[i];
  };
  const int fr = lane & 15;
  const int fofs = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));
  auto read_a = [&](bf16x8v (&fa)[4], const unsigned char* st, int half) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      fa[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 128 + half * 64 + r * 16) * ROWB + fofs);
  };
  auto read_b = [&](bf16x8v (&fb)[4], const unsigned char* st) {
#pragma unroll
    for (int n = 0; n < NB; ++n)
      fb[n] = *reinterpret_cast<const bf16x8v*>(st + BM * ROWB + (wc * WCOLS + n * 16) * ROWB + fofs);
  };
  f32x4v acc[8][NB];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  // prologue: tiles 0, 1 and A(2) written; B(2), A(3) in registers
  for (int t = 0; t < 2 && t < nk; ++t) load_a(t), load_b(t), write_a(t), write_b(t);
  if (2 < nk) load_a(2), write_a(2);
  if (2 < nk) load_b(2);
  if (3 < nk) load_a(3);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pp_barrier();
  if (wr == 1) pp_barrier();
  bf16x8v fa[4], fb[4];
  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
    if (kt + 2 < nk) write_b(kt + 2);
    if (kt + 3 < nk) load_b(kt + 3);
    read_b(fb, st);
    read_a(fa, st, 0);
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
    if (kt + 3 < nk) write_a(kt + 3);
    if (kt + 4 < nk) load_a(kt + 4);
    read_a(fa, st, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
  }
  if (wr == 0) pp_barrier();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  pp_barrier();
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
  pp_epilogue<PIPNET_EPI_NONE, 4>(p, acc, smem, m0, n0, wr, wc, lane, wid);
}
}  // namespace pipnet_bf16

namespace pipnet_bf16 {
// Lab-only: register staging two K-tiles deep.  Same LDS schedule as lab_prs_kernel (B(t+2)
// written in phase 0 of K-tile t, A(t+3) in phase 1), but each piece is LOADED two K-tiles
// before its write (B(t+4) / A(t+5) issued in K-tile t) into a register ring of two slots,
// so a global load has two K-tiles (~4 MFMA phases of both groups) to land.  The K loop is
// unrolled by two so the ring slot is a compile-time register.  Dense A only.
template <int ABL>
__global__ __launch_bounds__(pp::NT, 1) void lab_prs2_kernel(ConvParams p) {
  using namespace pp;
  constexpr int NS = 4, NB = 4, WCOLS = 64;
  __shared__ __attribute__((aligned(16))) unsigned char smem[smem_bytes<2>()];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  tile_coords(p, BM, 4 * WCOLS, m0, n0);
  const int nk = p.K / BK;
  const int drow = lane >> 2;
  const int dchunk = 8 * ((lane & 3) ^ g(drow));
  const bf16* asrc[2];
  const bf16* wsrc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 16 * (wid + 8 * i) + drow;
    asrc[i] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + dchunk;
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + dchunk;
  }
  bf16x8v ra[2][2], rb[2][2];                 // [ring slot][piece]
  auto load_a = [&](int kt, bf16x8v (&r)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = *reinterpret_cast<const bf16x8v*>(asrc[i] + (kt < nk ? kt : 0) * BK);
  };
  auto load_b = [&](int kt, bf16x8v (&r)[2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i) r[i] = *reinterpret_cast<const bf16x8v*>(wsrc[i] + (kt < nk ? kt : 0) * BK);
  };
  auto write_a = [&](int kt, const bf16x8v (&r)[2]) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<bf16x8v*>(base + (wid + 8 * i) * 1024 + lane * 16) = r[i];
  };
  auto write_b = [&](int kt, const bf16x8v (&r)[2]) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES + BM * ROWB;
#pragma unroll
    for (int i = 0; i < 2; ++i) *reinterpret_cast<bf16x8v*>(base + (wid + 8 * i) * 1024 + lane * 16) = r[i];
  };
  const int fr = lane & 15;
  const int fofs = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));
  auto read_a = [&](bf16x8v (&fa)[4], const unsigned char* st, int half) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      fa[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 128 + half * 64 + r * 16) * ROWB + fofs);
  };
  auto read_b = [&](bf16x8v (&fb)[4], const unsigned char* st) {
#pragma unroll
    for (int n = 0; n < NB; ++n)
      fb[n] = *reinterpret_cast<const bf16x8v*>(st + BM * ROWB + (wc * WCOLS + n * 16) * ROWB + fofs);
  };
  f32x4v acc[8][NB];
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  // prologue: tiles 0, 1 (A and B) and A(2) in LDS; ring: B(2) B(3) and A(3) A(4) in flight
  {
    bf16x8v t[2];
    for (int k = 0; k < 2 && k < nk; ++k) {
      load_a(k, t); write_a(k, t);
      load_b(k, t); write_b(k, t);
    }
    if (2 < nk) { load_a(2, t); write_a(2, t); }
  }
  load_b(2, rb[0]);
  load_b(3, rb[1]);
  load_a(3, ra[0]);
  load_a(4, ra[1]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  pp_barrier();
  if (wr == 1) pp_barrier();
  bf16x8v fa[4], fb[4];
  auto ktile = [&](int kt, auto slotc) {
    constexpr int S = decltype(slotc)::value;
    const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
    if (kt + 2 < nk) write_b(kt + 2, rb[S]);             // loaded two K-tiles ago
    load_b(kt + 4, rb[S]);                               // (clamped past nk: harmless reload)
    read_b(fb, st);
    read_a(fa, st, 0);
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
    if (kt + 3 < nk) write_a(kt + 3, ra[S]);
    load_a(kt + 5, ra[S]);
    read_a(fa, st, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pp_barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int n = 0; n < NB; ++n)
        acc[4 + r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[r], fb[n], acc[4 + r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    pp_barrier();
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    ktile(kt, IntC<0>{});
    ktile(kt + 1, IntC<1>{});
  }
  if (kt < nk) ktile(kt, IntC<0>{});
  if (wr == 0) pp_barrier();
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  pp_barrier();
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
  pp_epilogue<PIPNET_EPI_NONE, 4>(p, acc, smem, m0, n0, wr, wc, lane, wid);
}
}  // namespace pipnet_bf16

namespace pipnet_bf16 {
// Lab-only: 256x256 tile on FOUR waves (one per SIMD), each wave 128x128 = 8 x 8 MFMA 16x16
// tiles (256 accumulator registers), so an A fragment feeds 8 MFMAs and a B fragment 8: a
// third fewer LDS fragment bytes per MFMA than the 8-wave ping-pong tile (128x64 per wave).
// 32-deep K-tiles in 4 LDS stages (the pp image and swizzle), LDS-DMA 3 tiles ahead, fragments
// of K-tile t+1 read (double-buffered registers) during the second half of K-tile t's MFMAs;
// one barrier per K-tile.  Dense A only.  ABL: 2 = no epilogue.
template <int ABL>
__global__ __launch_bounds__(256, 1) void lab_q4_kernel(ConvParams p) {
  using namespace pp;
  constexpr int NS = 4, NW = 4, TMF = 8, TNF = 8;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  tile_coords(p, BM, BN, m0, n0);
  const int nk = p.K / BK;
  const int drow = lane >> 2;
  const int dchunk = 8 * ((lane & 3) ^ g(drow));
  const bf16* asrc[4];
  const bf16* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 16 * (wid + NW * i) + drow;
    asrc[i] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + dchunk;
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + dchunk;
  }
  auto stage = [&](int kt) {                      // 4 A + 4 B pieces of 1 KiB per wave
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(asrc[i] + kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + (wid + NW * i) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + BM * ROWB + (wid + NW * i) * 1024),
                                       16, 0, 0);
  };
  const int fr = lane & 15;
  const int fofs = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));
  bf16x8v fa[2][TMF], fb[2][TNF];
  auto read = [&](int kt, bf16x8v (&a)[TMF], bf16x8v (&b)[TNF]) {
    const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int n = 0; n < TNF; ++n)
      b[n] = *reinterpret_cast<const bf16x8v*>(st + BM * ROWB + (wc * 128 + n * 16) * ROWB + fofs);
#pragma unroll
    for (int r = 0; r < TMF; ++r) a[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 128 + r * 16) * ROWB + fofs);
  };
  f32x4v acc[TMF][TNF];
#pragma unroll
  for (int r = 0; r < TMF; ++r)
#pragma unroll
    for (int n = 0; n < TNF; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < 3 && t < nk; ++t) stage(t);
  // own pieces of tile 0 landed: younger tiles 1, 2 (8 pieces each)
  pp_wait_vm_dyn(8 * ((nk > 1) + (nk > 2)) > 10 ? 10 : 8 * ((nk > 1) + (nk > 2)));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // (simple prologue: drain)
  pp_barrier();
  read(0, fa[0], fb[0]);
  auto step = [&](int kt, auto sc) {
    constexpr int S = decltype(sc)::value;
    if (kt + 3 < nk) stage(kt + 3);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < TMF / 2; ++r)
#pragma unroll
      for (int n = 0; n < TNF; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[S][r], fb[S][n], acc[r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // own pieces of tile kt+1 landed: younger in flight = tiles kt+2, kt+3 that were issued
    const int younger = (kt + 2 < nk) + (kt + 3 < nk);
    if (younger == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    if (kt + 1 < nk) read(kt + 1, fa[S ^ 1], fb[S ^ 1]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = TMF / 2; r < TMF; ++r)
#pragma unroll
      for (int n = 0; n < TNF; ++n) acc[r][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[S][r], fb[S][n], acc[r][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, IntC<0>{});
    step(kt + 1, IntC<1>{});
  }
  if (kt < nk) step(kt, IntC<0>{});
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr ((ABL & 2) != 0) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < TMF; ++r)
#pragma unroll
      for (int n = 0; n < TNF; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) t += acc[r][n][i];
    reinterpret_cast<float*>(p.C)[(int64_t)blockIdx.x * 256 + tid] = t;
    return;
  }
  // plain epilogue (lab): D[row = 4 (lane >> 4) + i][col = lane & 15] of each 16x16 tile
#pragma unroll
  for (int r = 0; r < TMF; ++r)
#pragma unroll
    for (int n = 0; n < TNF; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wr * 128 + r * 16 + 4 * (lane >> 4) + i;
        const int nn = n0 + wc * 128 + n * 16 + (lane & 15);
        if (m < p.M && nn < p.N) p.C[(int64_t)m * p.ldc + nn] = (bf16)acc[r][n][i];
      }
}
}  // namespace pipnet_bf16

namespace pipnet_bf16 {
// Lab-only: lab_q4_kernel with the accumulators pinned to AGPRs by inline-asm MFMAs ("+a"
// operands): hipcc's own allocation of the 256 accumulators split them over VGPRs and AGPRs
// (361 v_accvgpr moves + scratch in the loop, profiles/r02/bf16_lab.txt).  Same k order and
// MFMA as pp: bitwise equal outputs.  ABL: 2 = no epilogue.
PIPNET_DEV void mfma_acc(f32x4v& c, const bf16x8v& a, const bf16x8v& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
template <int ABL>
__global__ __launch_bounds__(256, 1) void lab_q4a_kernel(ConvParams p) {
  using namespace pp;
  constexpr int NS = 4, NW = 4, TMF = 8, TNF = 8;
  __shared__ __attribute__((aligned(16))) unsigned char smem[NS * STAGE_BYTES];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  int m0, n0;
  tile_coords(p, BM, BN, m0, n0);
  const int nk = p.K / BK;
  const int drow = lane >> 2;
  const int dchunk = 8 * ((lane & 3) ^ g(drow));
  const bf16* asrc[4];
  const bf16* wsrc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 16 * (wid + NW * i) + drow;
    asrc[i] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + dchunk;
    wsrc[i] = p.W + (int64_t)min(n0 + row, p.N - 1) * p.K + dchunk;
  }
  auto stage = [&](int kt) {
    unsigned char* base = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(asrc[i] + kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + (wid + NW * i) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(wsrc[i] + kt * BK),
                                       (__attribute__((address_space(3))) void*)(base + BM * ROWB + (wid + NW * i) * 1024),
                                       16, 0, 0);
  };
  const int fr = lane & 15;
  const int fofs = fr * ROWB + 16 * ((lane >> 4) ^ g(fr));
  bf16x8v fa[2][TMF], fb[2][TNF];
  auto read = [&](int kt, bf16x8v (&a)[TMF], bf16x8v (&b)[TNF]) {
    const unsigned char* st = smem + (kt % NS) * STAGE_BYTES;
#pragma unroll
    for (int n = 0; n < TNF; ++n)
      b[n] = *reinterpret_cast<const bf16x8v*>(st + BM * ROWB + (wc * 128 + n * 16) * ROWB + fofs);
#pragma unroll
    for (int r = 0; r < TMF; ++r) a[r] = *reinterpret_cast<const bf16x8v*>(st + (wr * 128 + r * 16) * ROWB + fofs);
  };
  f32x4v acc[TMF][TNF];
#pragma unroll
  for (int r = 0; r < TMF; ++r)
#pragma unroll
    for (int n = 0; n < TNF; ++n) acc[r][n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  for (int t = 0; t < 3 && t < nk; ++t) stage(t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  pp_barrier();
  read(0, fa[0], fb[0]);
  auto step = [&](int kt, auto sc) {
    constexpr int S = decltype(sc)::value;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 3 < nk) stage(kt + 3);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = 0; r < TMF / 2; ++r)
#pragma unroll
      for (int n = 0; n < TNF; ++n) mfma_acc(acc[r][n], fa[S][r], fb[S][n]);
    __builtin_amdgcn_s_setprio(0);
    const int younger = (kt + 2 < nk) + (kt + 3 < nk);
    if (younger == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pp_barrier();
    if (kt + 1 < nk) read(kt + 1, fa[S ^ 1], fb[S ^ 1]);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int r = TMF / 2; r < TMF; ++r)
#pragma unroll
      for (int n = 0; n < TNF; ++n) mfma_acc(acc[r][n], fa[S][r], fb[S][n]);
    __builtin_amdgcn_s_setprio(0);
  };
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    step(kt, IntC<0>{});
    step(kt + 1, IntC<1>{});
  }
  if (kt < nk) step(kt, IntC<0>{});
  // the MFMAs are opaque to the hazard recognizer: pad before the accumulators are read
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  if constexpr ((ABL & 2) != 0) {
    float t = 0.f;
#pragma unroll
    for (int r = 0; r < TMF; ++r)
#pragma unroll
      for (int n = 0; n < TNF; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) t += acc[r][n][i];
    reinterpret_cast<float*>(p.C)[(int64_t)blockIdx.x * 256 + tid] = t;
    return;
  }
#pragma unroll
  for (int r = 0; r < TMF; ++r)
#pragma unroll
    for (int n = 0; n < TNF; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wr * 128 + r * 16 + 4 * (lane >> 4) + i;
        const int nn = n0 + wc * 128 + n * 16 + (lane & 15);
        if (m < p.M && nn < p.N) p.C[(int64_t)m * p.ldc + nn] = (bf16)acc[r][n][i];
      }
}
}  // namespace pipnet_bf16

namespace {
int group_for(int K, double budget) {
  const double panel = 128.0 * K * 2.0;
  int g = (int)(budget / panel);
  return g < 1 ? 1 : (g > 16 ? 16 : g);
}
}  // namespace

// 3x3 / stride 1 / pad 1 conv on the LDS-halo ping-pong tile (conv3x3_bf16_halo_kernel, product tile 8)
// with its ABL ablation bits (0 = the product kernel, EPI_NONE): x NHWC [B][H][W][Cin] bf16, w packed
// [N][9 Cin] bf16, y NHWC [B][H][W][N] bf16.  Same ConvParams as pipnet_conv2d_nhwc_bf16_tile.
extern "C" int lab_halo(int abl, const void* x, int B, int H, int W, int Cin, const void* w, int N, void* y,
                        void* stream) {
  ConvParams p{};
  p.A = reinterpret_cast<const bf16*>(x);
  p.W = reinterpret_cast<const bf16*>(w);
  p.C = reinterpret_cast<bf16*>(y);
  p.ldc = N;
  p.M = B * H * W; p.N = N;
  p.Kv = 9 * Cin;
  p.K = (p.Kv + KPAD - 1) / KPAD * KPAD;
  p.H = H; p.Wd = W; p.Cin = Cin; p.OH = H; p.OW = W; p.stride = 1; p.KW = 3; p.pad = 1; p.Cinp = Cin;
  if (Cin % 64 || W > 31 || N % 256 || (int64_t)p.M * Cin >= ((int64_t)1 << 31)) return 1;
  p.nt = N / 256;
  p.mt = (p.M + 255) / 256;
  p.group_m = group_for(p.K, 2.0 * 1024 * 1024);
  const dim3 grid(p.mt * p.nt);
  hipStream_t s = (hipStream_t)stream;
#define HALO_CASE(X) \
  case X: hipLaunchKernelGGL((conv3x3_bf16_halo_abl_kernel<PIPNET_EPI_NONE, 4, 8, X>), grid, dim3(512), 0, s, p); break;
  // 1000 + bits: the one-segment-per-K-tile schedule (SEG = 1, round 6)
#define HALO1_CASE(X) \
  case 1000 + X: hipLaunchKernelGGL((conv3x3_bf16_halo_abl_kernel<PIPNET_EPI_NONE, 4, 8, X, 1>), grid, dim3(512), 0, s, p); break;
  // 3000 + bits: SEG = 1 with the half-1 A reads as inline asm and explicit per-row lgkmcnt waits
#define HALO3_CASE(X) \
  case 3000 + X: hipLaunchKernelGGL((conv3x3_bf16_halo_abl_kernel<PIPNET_EPI_NONE, 4, 8, X, 3>), grid, dim3(512), 0, s, p); break;
  switch (abl) {
    case 0: hipLaunchKernelGGL((conv3x3_bf16_halo_kernel<PIPNET_EPI_NONE, 4, 8>), grid, dim3(512), 0, s, p); break;
    HALO_CASE(1) HALO_CASE(2) HALO_CASE(4) HALO_CASE(8) HALO_CASE(16) HALO_CASE(3) HALO_CASE(17)
    HALO_CASE(19) HALO_CASE(10) HALO_CASE(12) HALO_CASE(27)
    HALO1_CASE(0) HALO1_CASE(1) HALO1_CASE(2) HALO1_CASE(4) HALO1_CASE(8) HALO1_CASE(16) HALO1_CASE(3)
    HALO1_CASE(17) HALO1_CASE(19) HALO1_CASE(27)
    HALO3_CASE(0) HALO3_CASE(2) HALO3_CASE(19) HALO3_CASE(3) HALO3_CASE(64) HALO3_CASE(128) HALO3_CASE(83)
    default: return 1;
  }
#undef HALO_CASE
#undef HALO1_CASE
#undef HALO3_CASE
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int lab_pp(int abl, const void* A, const void* W, void* C, int M, int N, int K, double group_budget,
                      void* stream) {
  ConvParams p{};
  p.A = reinterpret_cast<const bf16*>(A);
  p.lda = K;
  p.W = reinterpret_cast<const bf16*>(W);
  p.C = reinterpret_cast<bf16*>(C);
  p.ldc = N;
  p.M = M; p.N = N; p.K = K; p.Kv = K;
  p.Cin = K; p.Cinp = K; p.H = 1; p.Wd = 1; p.OH = 1; p.OW = 1; p.stride = 1; p.KW = 1;
  p.nt = (N + 255) / 256;
  p.mt = (M + 255) / 256;
  p.group_m = group_for(K, group_budget);
  const dim3 grid(p.mt * p.nt);
  hipStream_t s = (hipStream_t)stream;
  // abl = ablation bits (0..15) + 16 * (DB - 2) for the 32-deep ping-pong kernel; 32 + bits
  // for the 64-deep full-line kernel (conv_bf16_p64_kernel)
#define LAB_CASE(X, D) \
  case X + 16 * (D - 2): hipLaunchKernelGGL((conv_bf16_pp_kernel<PIPNET_EPI_NONE, ALOAD_DENSE, 4, X, D>), grid, dim3(512), 0, s, p); break;
#define LAB_P64(X) \
  case 32 + X: hipLaunchKernelGGL((conv_bf16_p64_kernel<PIPNET_EPI_NONE, ALOAD_DENSE, X>), grid, dim3(512), 0, s, p); break;
  // 128 + cpolicy index: p64 with LDS-DMA cache-policy bits (A, B)
#define LAB_CP(I, A_, B_) \
  case 128 + I: hipLaunchKernelGGL((conv_bf16_p64_kernel<PIPNET_EPI_NONE, ALOAD_DENSE, 0, A_, B_>), grid, dim3(512), 0, s, p); break;
  switch (abl) {
    case 256: hipLaunchKernelGGL((lab_prs_kernel<0>), grid, dim3(512), 0, s, p); break;
    case 258: hipLaunchKernelGGL((lab_prs_kernel<2>), grid, dim3(512), 0, s, p); break;
    case 512: hipLaunchKernelGGL((lab_prs2_kernel<0>), grid, dim3(512), 0, s, p); break;
    case 1024: hipLaunchKernelGGL((lab_q4_kernel<0>), grid, dim3(256), 0, s, p); break;
    case 1026: hipLaunchKernelGGL((lab_q4_kernel<2>), grid, dim3(256), 0, s, p); break;
    case 1040: hipLaunchKernelGGL((lab_q4a_kernel<0>), grid, dim3(256), 0, s, p); break;
    case 1042: hipLaunchKernelGGL((lab_q4a_kernel<2>), grid, dim3(256), 0, s, p); break;
    case 514: hipLaunchKernelGGL((lab_prs2_kernel<2>), grid, dim3(512), 0, s, p); break;
    LAB_CP(0, 0, 0) LAB_CP(1, 1, 1) LAB_CP(2, 2, 2) LAB_CP(3, 16, 16) LAB_CP(4, 17, 17) LAB_CP(5, 2, 0)
    LAB_CP(6, 0, 2) LAB_CP(7, 3, 3) LAB_CP(8, 16, 0) LAB_CP(9, 0, 16)
    LAB_P64(0) LAB_P64(1) LAB_P64(2) LAB_P64(4) LAB_P64(8) LAB_P64(16) LAB_P64(18) LAB_P64(32) LAB_P64(34)
    LAB_CASE(0, 2) LAB_CASE(1, 2) LAB_CASE(2, 2) LAB_CASE(4, 2) LAB_CASE(8, 2)
    LAB_CASE(0, 3) LAB_CASE(1, 3) LAB_CASE(2, 3) LAB_CASE(4, 3) LAB_CASE(8, 3)
    default: return 1;
  }
#undef LAB_CASE
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
