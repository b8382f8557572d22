// Fused CNBlock MLP of the narrow ConvNeXt stages (C = 96 / 192), exact fp32 on
// v_mfma_f32_16x16x4_f32:
//     x <- x + gamma * (W2 gelu(W1 t + b1) + b2)              (torchvision CNBlock, SURVEY.md 2.3:
//                                                             block.3 Linear, block.4 GELU, block.5
//                                                             Linear, layer_scale, + residual)
// for NHWC rows t = dwconv+LN output [M, C], x = the residual stream [M, C] (updated in place).
//
// Why: at C = 96 / 192 the two Linears are K = 96 / N = 96-shaped GEMMs (49-57 % MFMA busy in
// the unfused kernels) and the 4C-wide hidden activation makes an HBM round trip (308 MB per
// stage-1 block at C2).  Here the hidden activation never leaves the registers:
//
//   * both products are computed TRANSPOSED, one wave per 16 pixels: GEMM1 h^T[hid][pix] =
//     W1[hid][:] . t[pix][:] (A = W1 from LDS, B = t from registers), so the 16x16 result of
//     one hidden block has the pixel on the lane and 4 hidden indices in the registers --
//     exactly the B operand layout of GEMM2 out^T[c][pix] = W2[c][hid] . h^T[hid][pix] for 4
//     k-steps (lane l supplies hidden 4(l>>4) + s at step s; the A operand W2[c][.] is read
//     with the same index map: one float4 per lane per 4 MFMAs);
//   * t stays in registers for the whole block (C/4 floats per lane), the accumulator of
//     out^T (C/16 tiles x 4 floats) too; GELU (+ b1) is applied in registers;
//   * the weights stream through LDS in hidden chunks of HC (W1 rows / W2 columns), double
//     buffered by LDS-DMA (global_load_lds_dwordx4), XOR-swizzled 16-B chunks so that every
//     ds_read_b128 lane group of the fragment reads hits 16 distinct bank slots;
//   * epilogue: lane l owns pixel l & 15 and 4 consecutive channels per tile -> one float4
//     read-modify-write of x per tile, with gamma and b2.
// k order of both contractions: t / hidden index 16 g + 4 q + s (q = lane >> 4, MFMA step s), GEMM1
// as two chains over even / odd g summed at the end -- a different (equally exact) fp32 summation
// order than the unfused GEMMs.
#include "common.hpp"

namespace {

template <int C, int HC, int NW, int PX = 1, int HS = 1>
struct MlpGeo {
  static constexpr int NT = 64 * NW;
  static constexpr int PXW = 16 * PX;                                      // pixels per wave
  static constexpr int W1F = HC * C, W2F = C * HC, CHUNK_F = W1F + W2F;   // floats per chunk
  static constexpr int NCH = 4 * C / HC;                                   // hidden chunks
  static constexpr int NCHH = NCH / HS;                                    // chunks per hidden part
  static constexpr int STAGE_F = HS * CHUNK_F;                             // one chunk per part
  static constexpr int W1_PIECES = W1F / 256, PIECES = CHUNK_F / 256;      // 1-KiB LDS-DMA pieces
  static constexpr int PPW = HS * PIECES / NW;                             // pieces per wave
  static_assert(NCH % HS == 0 && NW % HS == 0 && (HS * PIECES) % NW == 0, "HS");
  static constexpr int RC1 = C / 4, RC2 = HC / 4;                          // 16-B chunks per row
  static_assert(C % 32 == 0 && RC1 % 8 == 0, "C");
  static_assert(HC == 16 || HC == 32, "HC");
  static_assert(W1F % 256 == 0 && W2F % 256 == 0, "pieces");
  // chunk swizzles (XOR inside aligned groups of 16 / 8 / 4 chunks): conflict-free for the
  // fragment reads (row = 16 blk + (l & 15), chunk = 4 g + (l >> 4)), checked exhaustively
  static PIPNET_DEV int f1(int r) { return RC1 % 16 == 0 ? (r & 15) : (r & 7); }
  static PIPNET_DEV int f2(int r) { return HC == 32 ? (r & 7) : ((r >> 1) & 3); }
};

// PX = 16-pixel groups per wave: each W fragment read from LDS feeds PX MFMAs.  HS = hidden
// parts: HS waves share a pixel group, wave part j contracting hidden chunks [j NCH/HS, (j+1)
// NCH/HS) (both parts' chunks staged side by side), the partial out^T summed part 0 + part 1
// through LDS before the epilogue -- HS x the waves per pixel (C5's stage 2 has 1024 pixel
// groups: one wave per SIMD at HS = 1).  The hidden order, and so the rounding, depends on HS
// only (never on M), so choosing HS from the layer alone keeps the results batch-invariant.
// The product (pipnet_cnblock_mlp_hw_f32) takes HS = 2 for C = 192 on maps of at most
// MLP_HS2_MAX_HW pixels per image (C5's stage 2 and C1: 16x16 / 8x8 maps) and HS = 1 otherwise
// (C2's 28x28 stage 2, every C = 96 stage; profiles/r02/mlp_lab.txt, profiles/r03/bench_mlp_hs2.log).
// (A staggered-halves form -- the second wave of each SIMD pair one chunk period late, so the two
// waves' GELUs do not coincide -- was bitwise equal and no faster on any C2 / C5 shape in round 4;
// profiles/r04/mlp_stagger_lab.txt.)
// Launch bounds: at least 2 waves per SIMD for every workgroup size (MINB = 8 / NW workgroups per
// CU), so the register allocation stays within 256 -- with the plain 256-thread bound hipcc spread
// the C = 192 kernels over 198 VGPRs + 70 AGPRs, one wave per SIMD.
// ABL (tuning lab only, tools/mlp_lab.hip; 0 in the product): 1 = no GELU, 2 = no per-chunk
// barrier / DMA wait, 4 = no GEMM2 (h added into acc), 8 = no GEMM1, 16 = no weight DMA
// (profiles/r05/mlp_ablation.txt), 32 = GEMM1 on one accumulator chain (the round-2..4 form).
// (The body is a device function so that the product kernel's name -- what rocprof reports and
// bench.py / profiles/ key on -- carries no lab parameter; the lab launches cnblock_mlp_abl_kernel.)
template <int C, int HC, int NW, int PX, int HS, int ABL>
__device__ __forceinline__ void cnblock_mlp_body(const float* __restrict__ t, const float* __restrict__ W1,
                                                 const float* __restrict__ b1, const float* __restrict__ W2,
                                                 const float* __restrict__ b2, const float* __restrict__ gamma,
                                                 float* x, int M) {
  using G = MlpGeo<C, HC, NW, PX, HS>;
  constexpr int NSTG = 2;
  // one LDS array (a second __shared__ object can make hipcc drain the DMA early): NSTG stage
  // buffers (HS chunks each), then b1 (staged once: a per-chunk global load of it would wait
  // for the DMA)
  __shared__ __attribute__((aligned(16))) float smem[NSTG * G::STAGE_F + 4 * C];
  float* sb1 = smem + NSTG * G::STAGE_F;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int part = wid % HS, grp = wid / HS;
  const int q = lane >> 4, pl = lane & 15;
  const int pix0 = blockIdx.x * (G::PXW * NW / HS) + G::PXW * grp + pl;   // pixel of group 0; group u: + 16 u

  // ---- LDS-DMA sources of this wave's pieces (stage 0); piece P of a stage belongs to part
  // P / PIECES, whose chunk i is chunk part*NCHH + i: it adds that chunk's c*HC*C (W1) / c*HC (W2) ----
  const float* src[G::PPW];
  int dst[G::PPW];
  bool is_w1[G::PPW];
#pragma unroll
  for (int j = 0; j < G::PPW; ++j) {
    const int pp = wid + NW * j;
    const int pt = pp / G::PIECES, p = pp - pt * G::PIECES;
    dst[j] = pt * G::CHUNK_F + p * 256;
    if (p < G::W1_PIECES) {
      const int e = p * 64 + lane;                        // 16-B chunk index inside the W1 image
      const int r = e / G::RC1, pc = e - r * G::RC1;
      src[j] = W1 + (int64_t)r * C + 4 * (pc ^ G::f1(r)) + (int64_t)pt * G::NCHH * HC * C;
      is_w1[j] = true;
    } else {
      const int e = (p - G::W1_PIECES) * 64 + lane;
      const int r = e / G::RC2, pc = e - r * G::RC2;
      src[j] = W2 + (int64_t)r * (4 * C) + 4 * (pc ^ G::f2(r)) + (int64_t)pt * G::NCHH * HC;
      is_w1[j] = false;
    }
  }
  auto stage = [&](int ch) {                           // ch = chunk index within a part
    if constexpr ((ABL & 16) != 0) return;
    float* base = smem + (ch % NSTG) * G::STAGE_F;
#pragma unroll
    for (int j = 0; j < G::PPW; ++j) {
      const float* s = src[j] + (is_w1[j] ? (int64_t)ch * HC * C : (int64_t)ch * HC);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)s,
                                       (__attribute__((address_space(3))) void*)(base + dst[j]), 16, 0, 0);
    }
  };
  for (int i = tid; i < C; i += G::NT) st4(sb1 + 4 * i, ld4(b1 + 4 * i));
  stage(0);

  // ---- t of this lane's pixels in registers: tb[u][g] = t[pixel u][16 g + 4 q .. + 3] ----
  f32x4 tb[PX][C / 16];
#pragma unroll
  for (int u = 0; u < PX; ++u) {
    const int pix = pix0 + 16 * u;
    const int prow = pix < M ? pix : M - 1;             // rows past M compute garbage, never stored
#pragma unroll
    for (int g = 0; g < C / 16; ++g) tb[u][g] = ld4(t + (int64_t)prow * C + 16 * g + 4 * q);
  }
  f32x4 acc[PX][C / 16];
#pragma unroll
  for (int u = 0; u < PX; ++u)
#pragma unroll
    for (int cb = 0; cb < C / 16; ++cb) acc[u][cb] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment offsets (floats) inside a chunk image
  auto w1_off = [&](int hb, int g) {
    const int r = 16 * hb + pl;
    return r * C + 4 * ((4 * g + q) ^ G::f1(r));
  };
  auto w2_off = [&](int cb, int hb) {
    const int r = 16 * cb + pl;
    return G::W1F + r * HC + 4 * ((4 * hb + q) ^ G::f2(r));
  };
  constexpr int NHB = HC / 16;
  // GEMM1 accumulator chains: 2 (even / odd t groups, summed after the chunk; lab bit 32 = the
  // single chain of rounds 2-4): -0.6 / -1.8 / -2.3 / -0.2 % on C5 stage 1 / 2 and C2's stage 1 / 2
  // half batches (profiles/r05/mlp_g1c.txt); a different -- equally exact -- fp32 association
  constexpr int G1C = (ABL & 32) ? 1 : 2;

  for (int ci = 0; ci < G::NCHH; ++ci) {
    // this wave's pieces of stage ci landed, every wave's reads of stage ci-1 retired
    if constexpr ((ABL & 2) == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ci + 1 < G::NCHH) stage(ci + 1);                // into the buffer of stage ci-1
    const float* buf = smem + (ci & 1) * G::STAGE_F + part * G::CHUNK_F;
    const int ch = part * G::NCHH + ci;                 // global hidden chunk
    // GEMM1: h^T[16 hb + 4q + i][pixel] for the NHB hidden blocks of the chunk; consecutive
    // MFMAs go to different accumulators (16x16x4: 40-cycle dependent latency, 32-cycle issue)
    f32x4 h[PX][NHB];
#pragma unroll
    for (int u = 0; u < PX; ++u)
#pragma unroll
      for (int hb = 0; hb < NHB; ++hb) h[u][hb] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr ((ABL & 8) != 0) {
#pragma unroll
      for (int u = 0; u < PX; ++u)
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb) h[u][hb] = tb[u][hb % (C / 16)] + ld4(buf + w1_off(hb, 0));
    } else if constexpr (G1C == 2) {
      // two accumulator chains (even / odd t groups), added at the end: with one hidden block per
      // chunk (HC = 16) a single chain issues each MFMA on the previous one's result
      f32x4 h2[PX][NHB];
#pragma unroll
      for (int u = 0; u < PX; ++u)
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb) h2[u][hb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < C / 16; g += 2) {
        f32x4 w[NHB], w2[NHB];
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb) {
          w[hb] = ld4(buf + w1_off(hb, g));
          w2[hb] = ld4(buf + w1_off(hb, g + 1));
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int hb = 0; hb < NHB; ++hb)
#pragma unroll
            for (int u = 0; u < PX; ++u) {
              h[u][hb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[hb][s], tb[u][g][s], h[u][hb], 0, 0, 0);
              h2[u][hb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w2[hb][s], tb[u][g + 1][s], h2[u][hb], 0, 0, 0);
            }
      }
#pragma unroll
      for (int u = 0; u < PX; ++u)
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb) h[u][hb] = h[u][hb] + h2[u][hb];
    } else {
#pragma unroll
      for (int g = 0; g < C / 16; ++g) {
        f32x4 w[NHB];
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb) w[hb] = ld4(buf + w1_off(hb, g));
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int hb = 0; hb < NHB; ++hb)
#pragma unroll
            for (int u = 0; u < PX; ++u)
              h[u][hb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[hb][s], tb[u][g][s], h[u][hb], 0, 0, 0);
      }
    }
    // + b1, GELU (the unfused Linear1 epilogue's packed form)
#pragma unroll
    for (int hb = 0; hb < NHB; ++hb) {
      const f32x4 bb = ld4(sb1 + ch * HC + 16 * hb + 4 * q);
#pragma unroll
      for (int u = 0; u < PX; ++u) {
        const f32x4 v = h[u][hb] + bb;
        if constexpr ((ABL & 1) != 0) {
          h[u][hb] = v;
          continue;
        }
        const f32x2 lo = gelu_pk16(f32x2{v[0], v[1]}), hi = gelu_pk16(f32x2{v[2], v[3]});
        h[u][hb] = f32x4{lo[0], lo[1], hi[0], hi[1]};
      }
    }
    // GEMM2: out^T[c][pixel] += W2[c][hidden] h^T[hidden][pixel]; the cb loop innermost, so
    // consecutive MFMAs go to different accumulators
    if constexpr ((ABL & 4) != 0) {
#pragma unroll
      for (int u = 0; u < PX; ++u)
#pragma unroll
        for (int hb = 0; hb < NHB; ++hb) acc[u][hb % (C / 16)] += h[u][hb] * ld4(buf + w2_off(hb % (C / 16), hb));
    } else
#pragma unroll
    for (int hb = 0; hb < NHB; ++hb) {
      f32x4 w[C / 16];
#pragma unroll
      for (int cb = 0; cb < C / 16; ++cb) w[cb] = ld4(buf + w2_off(cb, hb));
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int cb = 0; cb < C / 16; ++cb)
#pragma unroll
          for (int u = 0; u < PX; ++u)
            acc[u][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[cb][s], h[u][hb][s], acc[u][cb], 0, 0, 0);
    }
  }
  if constexpr (HS > 1) {
    // part sums through LDS (the stage buffers are free once every wave passed this barrier):
    // parts 1.. store, part 0 adds them in part order
    static_assert(HS == 2, "HS");
    static_assert((NW / HS) * 64 * PX * C / 4 <= NSTG * G::STAGE_F, "part-sum LDS");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* ex = smem + (grp * 64 + lane) * (PX * C / 4);
    if (part == 1) {
#pragma unroll
      for (int u = 0; u < PX; ++u)
#pragma unroll
        for (int cb = 0; cb < C / 16; ++cb) st4(ex + (u * (C / 16) + cb) * 4, acc[u][cb]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (part != 0) return;
#pragma unroll
    for (int u = 0; u < PX; ++u)
#pragma unroll
      for (int cb = 0; cb < C / 16; ++cb) acc[u][cb] = acc[u][cb] + ld4(ex + (u * (C / 16) + cb) * 4);
  }
  // ---- epilogue: x[pixel][c .. c+3] += gamma * (acc + b2), c = 16 cb + 4 q.  Every load (x rows
  // clamped to M - 1) is issued, and retired by one vm_drain, before the first store: loads
  // issued between row-guarded stores made hipcc wait vmcnt(0) -- for the stores too -- per chunk ----
#pragma unroll
  for (int u = 0; u < PX; ++u) {
    const int pix = pix0 + 16 * u;
    const float* xs = x + (int64_t)(pix < M ? pix : M - 1) * C;
    f32x4 r[C / 16], bb[C / 16], gm[C / 16];
#pragma unroll
    for (int cb = 0; cb < C / 16; ++cb) {
      const int c = 16 * cb + 4 * q;
      r[cb] = ld4(xs + c);
      bb[cb] = ld4(b2 + c);
      gm[cb] = ld4(gamma + c);
    }
    vm_drain();
    if (pix < M) {
      float* xr = x + (int64_t)pix * C;
#pragma unroll
      for (int cb = 0; cb < C / 16; ++cb) {
        const int c = 16 * cb + 4 * q;
        st4(xr + c, r[cb] + gm[cb] * (acc[u][cb] + bb[cb]));
      }
    }
  }
}

// Occupancy: HIP's second __launch_bounds__ argument is min WAVES PER EU (amdgpu_waves_per_eu), not
// workgroups per CU, so the target is stated directly: two waves per SIMD (a 256-register budget)
// for the 2- and 4-wave workgroups, one for the 8-wave forms, the 1-wave forms and C = 192 / HC = 32
// (their LDS allows fewer than 8 waves per CU anyway).  (The former `8 / NW` asked NW = 1 / 2 for 8 / 4 waves
// per EU; LLVM clipped that to the LDS-bound occupancy, so no kernel spilled -- tools/isa_dump.sh
// mlp_f32 shows scratch 0 for every instantiation either way.)
constexpr int mlp_waves_per_eu(int C, int HC, int NW) { return (NW >= 8 || NW == 1 || (C == 192 && HC == 32)) ? 1 : 2; }
#define PIPNET_MLP_BOUNDS(NW) __launch_bounds__(64 * (NW)) __attribute__((amdgpu_waves_per_eu(mlp_waves_per_eu(C, HC, NW))))
template <int C, int HC, int NW, int PX, int HS = 1>
__global__ PIPNET_MLP_BOUNDS(NW) void cnblock_mlp_kernel(
    const float* __restrict__ t, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ gamma, float* x, int M) {
  cnblock_mlp_body<C, HC, NW, PX, HS, 0>(t, W1, b1, W2, b2, gamma, x, M);
}

template <int C, int HC, int NW, int PX, int HS, int ABL>   // tuning lab only (tools/mlp_lab.hip)
__global__ PIPNET_MLP_BOUNDS(NW) void cnblock_mlp_abl_kernel(
    const float* __restrict__ t, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ gamma, float* x, int M) {
  cnblock_mlp_body<C, HC, NW, PX, HS, ABL>(t, W1, b1, W2, b2, gamma, x, M);
}

template <int C, int HC, int NW, int PX, int HS = 1, int ABL = 0>
int launch_mlp(const float* t, const float* W1, const float* b1, const float* W2, const float* b2, const float* gamma,
               float* x, int M, hipStream_t s) {
  const int px = 16 * PX * NW / HS;
  if constexpr (ABL == 0)
    hipLaunchKernelGGL((cnblock_mlp_kernel<C, HC, NW, PX, HS>), dim3((M + px - 1) / px), dim3(64 * NW), 0, s, t, W1,
                       b1, W2, b2, gamma, x, M);
  else
    hipLaunchKernelGGL((cnblock_mlp_abl_kernel<C, HC, NW, PX, HS, ABL>), dim3((M + px - 1) / px), dim3(64 * NW), 0, s,
                       t, W1, b1, W2, b2, gamma, x, M);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// Instantiations chosen with tools/mlp_lab.py (profiles/r02/mlp_lab.txt).  The per-pixel
// arithmetic does not depend on them (the hidden index is summed in 16-blocks in order for
// any HC), so the M-dependent choice keeps results batch-invariant.

}  // namespace

#ifdef PIPNET_MLP_LAB
bool pipnet_mlp_lab_variant(int C, const float* t, const float* W1, const float* b1, const float* W2, const float* b2,
                            const float* gamma, float* x, int M, hipStream_t s);
#endif

// Small maps (C = 192, <= 16 x 16 pixels per image: C5's stage 2) split the hidden dimension
// over two waves per 16-pixel group (HS = 2): 16384 pixels give 1024 pixel groups, one wave per
// SIMD at HS = 1 (tools/mlp_lab.py, profiles/r02/mlp_lab.txt: 103 -> 93 us).  HS changes the
// hidden summation order, so it is chosen from the layer's map size only -- never from M -- and
// a pixel's result stays independent of the batch it runs in.
constexpr int MLP_HS2_MAX_HW = 256;

// Workgroup shapes per M (tools/mlp_lab.py, profiles/r05/mlp_lab.txt; round 5 retuned the
// two-stream half batches of C2): C = 96 takes 4-wave workgroups from 98,304 pixels (C2 stage 1:
// 100,352 px 165.9 -> 150.7 us, 200,704 px 285.9 -> 273.8) and 8-wave ones at C5's 65,536
// (89.3 vs 93.3); C = 192 takes HC = 16 chunks at every M >= 8192 -- the HC = 32 chunks need
// 101 KiB of LDS, one 4-wave workgroup (one wave per SIMD) per CU: C2's 25,088-pixel stage-2
// half batch 198.6 -> 162.2 us on (16, 8), C5-sized 16,384 px 101.6 -> 99.4 on (16, 4).  Small M
// (C1: 16 images of 64^2) gets smaller workgroups so that the grid still covers the CUs.
// Plan code = HC * 100 + NW * 10 + HS (the instantiation cnblock_mlp_kernel<C, HC, NW, 1, HS>).
int mlp_plan(int m, int C, int hw) {
  if (C == 96) {
    if (m >= 98304) return 3241;       // C2 stage 1
    if (m >= 65536) return 3281;       // C5 stage 1
    if (m >= 16384) return 3241;
    if (m >= 8192) return 3221;
    return 3211;
  }
  if (hw > 0 && hw <= MLP_HS2_MAX_HW) return 1682;   // C5 stage 2
  if (m >= 24576) return 1681;         // C2 stage 2
  if (m >= 8192) return 1641;
  if (m >= 4096) return 3221;
  return 3211;
}

extern "C" int pipnet_cnblock_mlp_plan(int64_t M, int C, int hw) {
  if (M < 0 || M >= ((int64_t)1 << 31) || (C != 96 && C != 192) || hw < 0) return -PIPNET_ERR_ARG;
  return mlp_plan((int)M, C, hw);
}

extern "C" int pipnet_cnblock_mlp_hw_f32(const float* t, const float* W1, const float* b1, const float* W2,
                                         const float* b2, const float* gamma, float* x, int64_t M, int C, int hw,
                                         void* stream) {
  if (M < 0 || M >= ((int64_t)1 << 31) || (C != 96 && C != 192) || hw < 0) return PIPNET_ERR_ARG;
  if (!t || !W1 || !b1 || !W2 || !b2 || !gamma || !x) return PIPNET_ERR_ARG;
  if (!aligned16(t) || !aligned16(W1) || !aligned16(b1) || !aligned16(W2) || !aligned16(b2) || !aligned16(gamma) ||
      !aligned16(x))
    return PIPNET_ERR_ALIGN;
  if (M == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
#ifdef PIPNET_MLP_LAB
  if (pipnet_mlp_lab_variant(C, t, W1, b1, W2, b2, gamma, x, (int)M, s)) return PIPNET_OK;
#endif
  const int m = (int)M;
  switch (C * 10000 + mlp_plan(m, C, hw)) {
    case 963241: return launch_mlp<96, 32, 4, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 963281: return launch_mlp<96, 32, 8, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 963221: return launch_mlp<96, 32, 2, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 963211: return launch_mlp<96, 32, 1, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 1921682: return launch_mlp<192, 16, 8, 1, 2>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 1921681: return launch_mlp<192, 16, 8, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 1921641: return launch_mlp<192, 16, 4, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 1923221: return launch_mlp<192, 32, 2, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    case 1923211: return launch_mlp<192, 32, 1, 1>(t, W1, b1, W2, b2, gamma, x, m, s);
    default: return PIPNET_ERR_ARG;
  }
}

// map size unknown: the HS = 1 instantiations only
extern "C" int pipnet_cnblock_mlp_f32(const float* t, const float* W1, const float* b1, const float* W2,
                                      const float* b2, const float* gamma, float* x, int64_t M, int C,
                                      void* stream) {
  return pipnet_cnblock_mlp_hw_f32(t, W1, b1, W2, b2, gamma, x, M, C, 0, stream);
}
