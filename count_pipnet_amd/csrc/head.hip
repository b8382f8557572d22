// Prototype heads on gfx950 (HBM-bound wavefront-reduction kernels):
//   * softmax_pool   nn.Softmax(dim=1) over P channels per patch + AdaptiveMaxPool2d(1)
//                    (or spatial sum), proto map written exactly once      -- pipnet.py:33-34
//   * nonneg_linear  where(x<0.1,0,x) then F.linear(x, relu(W), b)         -- pipnet.py:36-37,70-71
//   * count_gumbel   F.gumbel_softmax(hard=True) + per-prototype count      -- count_pipnet.py:83-88
//   * count_finish   STE_Round / ClampSTE forwards                          -- count_pipnet.py:90-97
//   * count_encode   OneHotEncoder / LinearIntermediate forwards            -- count_pipnet_utils.py
// One wave owns one patch: lane l holds channels l, l+64, ... so every HBM access is a
// coalesced 256-B row segment, and the per-patch reductions are 64-lane butterflies.
#include <type_traits>

#include "common.hpp"
#include "philox.hpp"

namespace {
// Zero-fill by a kernel rather than a memset call: the launch is captured as an ordinary
// kernel node when the stream is being recorded into a HIP graph (count_pipnet_amd.graph); a
// memset issued during capture was observed NOT to take effect on replay.
// Two ranges per launch (the fused head zeroes pooled and its arrival tickets together).
__global__ __launch_bounds__(256) void zero_u32_kernel(uint32_t* __restrict__ p, int64_t n, uint32_t* __restrict__ p2,
                                                       int64_t n2) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n + n2; i += (int64_t)gridDim.x * 256) {
    if (i < n) p[i] = 0u;
    else p2[i - n] = 0u;
  }
}
inline bool zero_fill(void* p, int64_t n_u32, hipStream_t s, void* p2 = nullptr, int64_t n2_u32 = 0) {
  const int64_t n = n_u32 + (p2 ? n2_u32 : 0);
  const int64_t blocks = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(zero_u32_kernel, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(256), 0, s,
                     reinterpret_cast<uint32_t*>(p), n_u32, reinterpret_cast<uint32_t*>(p2), p2 ? n2_u32 : 0);
  return hipGetLastError() == hipSuccess;
}
}  // namespace

namespace {

constexpr int HEAD_THREADS = 256;
constexpr int PIX_PER_BLOCK = 32;

// ---------------------------------------------------------------------------------------
// NonNegLinear (pipnet.py:36-37, 54-71) fused into the softmax-pool head -- the whole head is ONE
// launch (no zero-fill ahead of it):
//   * every workgroup atomicMax-es its pixel block's per-channel maxima into a scratch row pmax[b]
//     (memory-side atomics: non-negative floats order like their bit patterns) and, once they are
//     acknowledged (vmcnt(0): a no-return atomic stays counted until performed at the memory side),
//     takes an arrival ticket for its image (atomicAdd, also performed there);
//   * the workgroup that draws gridDim.x - 1 takes the row back with atomicExch(.., 0) -- read at
//     the memory side (no XCD's stale L2 copy) and reset in the same operation -- writes pooled[b],
//     applies the 0.1 presence threshold in inference mode, writes the clamped row (x_out), runs the
//     GEMV x' relu(W)^T + bias against W as it is at call time, and resets its ticket: scratch and
//     tickets are zero again after every completed call (the caller zeroes them once);
//   * no fences: a release fence per workgroup (partial-slab stores + agent-scope release /
//     acquire, tried first in round 5) wrote back the L2 behind the streaming proto stores 3,200
//     times per C3 call and tripled the head's time;
//   * the GEMV runs nonneg_linear_kernel's per-class arithmetic exactly (nonneg_linear_wave: per-lane
//     float4 slices, fmaf order, one wave_sum), spread over the workgroup's 4 waves without a
//     barrier, so the fused head is bitwise the two-kernel path.
constexpr int NN_CLS_PER_BLOCK = 16;

struct HeadLinear {
  const float* W;        // [K, P] classifier weight (relu applied here, not stored)
  const float* bias;     // [K] or null
  int K;
  int apply_thresh;
  float thresh;
  float* x_out;          // [B, P] clamped (or copied) pooled row, or null
  float* out;            // [B, K] logits
  int32_t* tickets;      // [B] arrival tickets: zero on entry, zero again on exit
  float* part;           // [B, P] running maxima (pmax): zero on entry, zero again on exit
};

inline int64_t head_part_floats(int B, int HW, int P) { return HW > 0 ? (int64_t)B * P : 0; }

// NonNegLinear classes [k0, k0 + nk) (nk <= NC) of one row, by ONE wave: lane l owns the float4
// slices c = 4 l + 256 i of the feature dimension (scalars c = l + 64 i when D % 4 != 0), i
// ascending, and keeps NC class partials (4 fmaf per slice, .x .. .w); one wave_sum per class; lane
// 0 writes out[k] = sum + bias[k].  A class's arithmetic depends on (D, class) only -- not on NC,
// on which wave or workgroup runs it, or on the batch -- so the class-block kernel and the fused
// head's tail give the same bits.  apply_thresh / x_out: the 0.1 presence threshold applied on
// load and the clamped row stored (x_out != null only for one wave per row).  x: global or LDS.
// UNR = slices per unrolled step (registers / loads in flight; not the arithmetic).
template <int NC, int UNR>
PIPNET_DEV void nonneg_linear_wave(const float* x, int D, const float* __restrict__ W, const float* __restrict__ bias,
                                   int k0, int nk, float* __restrict__ outr, int apply_thresh, float thresh,
                                   float* __restrict__ x_out) {
  const int lane = threadIdx.x & 63;
  const float* w0 = W + (int64_t)k0 * D;
  float s[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) s[j] = 0.f;
  if ((D & 3) == 0) {
#pragma unroll UNR
    for (int c = 4 * lane; c < D; c += 256) {
      f32x4 xv = ld4(x + c);
      if (apply_thresh) {
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[e] = xv[e] < thresh ? 0.f : xv[e];
      }
      if (x_out) st4(x_out + c, xv);
      // rows past nk load row nk-1 and are discarded: a load under a per-class branch
      // made the compiler wait for each one (serialised round trips per slice)
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const f32x4 w = ld4(w0 + (int64_t)(j < nk ? j : nk - 1) * D + c);
        s[j] = fmaf(xv[0], fmaxf(w[0], 0.f), s[j]);
        s[j] = fmaf(xv[1], fmaxf(w[1], 0.f), s[j]);
        s[j] = fmaf(xv[2], fmaxf(w[2], 0.f), s[j]);
        s[j] = fmaf(xv[3], fmaxf(w[3], 0.f), s[j]);
      }
    }
  } else {
    for (int c = lane; c < D; c += 64) {
      float xv = x[c];
      if (apply_thresh && xv < thresh) xv = 0.f;
      if (x_out) x_out[c] = xv;
#pragma unroll
      for (int j = 0; j < NC; ++j) s[j] = fmaf(xv, fmaxf(w0[(int64_t)(j < nk ? j : nk - 1) * D + c], 0.f), s[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const float t = wave_sum(s[j]);
    if (lane == 0 && j < nk) outr[k0 + j] = t + (bias ? bias[k0 + j] : 0.f);
  }
}

// The fused head's tail, called after the workgroup's atomicMax loop into hl.part.  xs = >= P
// floats of LDS the workgroup no longer needs.
template <int TAIL_NC>
PIPNET_DEV void head_linear_tail(const HeadLinear& hl, int b, int P, float* pooled, float* xs) {
  __shared__ int is_last;
  vm_drain();                                  // this thread's atomicMax ops performed
  __syncthreads();
  if (threadIdx.x == 0) is_last = atomicAdd(hl.tickets + b, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!is_last) return;
  unsigned* prow = reinterpret_cast<unsigned*>(hl.part + (int64_t)b * P);
  for (int c = threadIdx.x; c < P; c += HEAD_THREADS) {
    float v = __uint_as_float(atomicExch(prow + c, 0u));   // read at the memory side, scratch reset
    pooled[(int64_t)b * P + c] = v;
    if (hl.apply_thresh && v < hl.thresh) v = 0.f;
    xs[c] = v;
    if (hl.x_out) hl.x_out[(int64_t)b * P + c] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) atomicExch(hl.tickets + b, 0);   // every workgroup of b has drawn
  // the GEMV spread over the 4 waves: wave w takes class groups w, w + 4, ... of TAIL_NC classes,
  // each wave on its own (no barrier) -- K = 200: 13 / 7 groups (TAIL_NC 4 / 8) on the longest wave
  // instead of 13 workgroup-wide passes with two barriers each.  One slice per step, TAIL_NC per
  // kernel so that the tail's registers stay under the streaming loop's (a kernel is allocated for
  // its maximum): fp32 logits 4 (59 VGPRs, the two-kernel head's 55), bf16 quads 8 (118, unchanged).
  const int wv = threadIdx.x >> 6;
  for (int k0 = wv * TAIL_NC; k0 < hl.K; k0 += (HEAD_THREADS / 64) * TAIL_NC)
    nonneg_linear_wave<TAIL_NC, 1>(xs, P, hl.W, hl.bias, k0, min(TAIL_NC, hl.K - k0), hl.out + (int64_t)b * hl.K, 0,
                                   0.f, nullptr);
}

// ---------------------------------------------------------------------------------------
// MODE 0 = max pool, 1 = sum pool; T = float / __bf16 logits; LIN: + the fused NonNegLinear tail
template <int NJ, int MODE, typename T = float, bool LIN = false>
__global__ __launch_bounds__(HEAD_THREADS) void softmax_pool_kernel(const T* __restrict__ feat, int HW, int P,
                                                                    float* __restrict__ proto,
                                                                    float* __restrict__ pooled, HeadLinear hl) {
  __shared__ float red[HEAD_THREADS / 64][NJ * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int pix0 = blockIdx.x * PIX_PER_BLOCK;
  float racc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) racc[j] = 0.f;   // softmax outputs are >= 0
  for (int pi = wv; pi < PIX_PER_BLOCK; pi += HEAD_THREADS / 64) {
    const int pix = pix0 + pi;
    if (pix >= HW) break;
    const int64_t base = ((int64_t)b * HW + pix) * P;
    float v[NJ];
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      v[j] = c < P ? (float)feat[base + c] : -INFINITY;
      m = fmaxf(m, v[j]);
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      v[j] = c < P ? expf(v[j] - m) : 0.f;
      s += v[j];
    }
    const float inv = 1.0f / wave_sum(s);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = lane + 64 * j;
      if (c < P) {
        const float yv = v[j] * inv;
        __builtin_nontemporal_store(yv, proto + base + c);   // written once, never re-read here
        racc[j] = MODE == 0 ? fmaxf(racc[j], yv) : racc[j] + yv;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) red[wv][lane + 64 * j] = racc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < P; c += HEAD_THREADS) {
    float r = red[0][c];
#pragma unroll
    for (int w = 1; w < HEAD_THREADS / 64; ++w) r = MODE == 0 ? fmaxf(r, red[w][c]) : r + red[w][c];
    float* dst = (LIN ? hl.part : pooled) + (int64_t)b * P + c;   // LIN: the scratch row, read back by the last workgroup
    if (MODE == 0)   // non-negative floats order like their bit patterns
      atomicMax(reinterpret_cast<unsigned int*>(dst), __float_as_uint(r));
    else
      atomicAdd(dst, r);
  }
  if constexpr (LIN) head_linear_tail<4>(hl, b, P, pooled, &red[0][0]);   // (its barriers guard red's reuse)
}

// bf16 logits (the C3 ResNet build, P = 2048), quad layout (round 4): lane l holds channels
// 4l + 256q .. +3 (8-B bf16 loads, 512 B contiguous per wave instruction), so each 16-B fp32
// proto store instruction writes 1 KiB contiguous -- 8 whole 128-B lines (an 8-channels-per-lane
// layout wrote every line in two halves from two instructions: 322 vs 250 us per 128 images,
// profiles/r04/pmc_summary_c3.txt; proto is 2/3 of this kernel's bytes).  The next pixel's
// logits are requested under the current one's math (one HBM latency per wave per pixel
// otherwise).  P % 8 == 0, P <= 512 NV.
template <int NV, int MODE, bool LIN = false>
__global__ __launch_bounds__(HEAD_THREADS) void softmax_pool_bf16q_kernel(const __bf16* __restrict__ feat, int HW,
                                                                          int P, float* __restrict__ proto,
                                                                          float* __restrict__ pooled, HeadLinear hl) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  constexpr int NQ = 2 * NV;
  __shared__ float red[HEAD_THREADS / 64][NV * 512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int pix0 = blockIdx.x * PIX_PER_BLOCK;
  float racc[NQ][4];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) racc[q][e] = 0.f;
  constexpr int STEP = HEAD_THREADS / 64;
  bf16x4_t xc[NQ], xn[NQ];
  auto load_pix = [&](int pix, bf16x4_t (&x)[NQ]) {
    const int64_t base = ((int64_t)b * HW + pix) * P;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = 4 * lane + 256 * q;
      if (c < P) x[q] = *reinterpret_cast<const bf16x4_t*>(feat + base + c);
    }
  };
  if (wv < PIX_PER_BLOCK && pix0 + wv < HW) load_pix(pix0 + wv, xc);
  for (int pi = wv; pi < PIX_PER_BLOCK; pi += STEP) {
    const int pix = pix0 + pi;
    if (pix >= HW) break;
    if (pi + STEP < PIX_PER_BLOCK && pix + STEP < HW) load_pix(pix + STEP, xn);
    const int64_t base = ((int64_t)b * HW + pix) * P;
    float v[NQ][4];
    float m = -INFINITY;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool ok = 4 * lane + 256 * q < P;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[q][e] = ok ? (float)xc[q][e] : -INFINITY;
        m = fmaxf(m, v[q][e]);
      }
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[q][e] = 4 * lane + 256 * q < P ? expf(v[q][e] - m) : 0.f;
        s += v[q][e];
      }
    const float inv = 1.0f / wave_sum(s);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int c = 4 * lane + 256 * q;
      if (c < P) {
        f32x4 y;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = v[q][e] * inv;
        __builtin_nontemporal_store(y, reinterpret_cast<f32x4*>(proto + base + c));   // write-once map
#pragma unroll
        for (int e = 0; e < 4; ++e) racc[q][e] = MODE == 0 ? fmaxf(racc[q][e], y[e]) : racc[q][e] + y[e];
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) xc[q] = xn[q];
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) red[wv][4 * lane + 256 * q + e] = racc[q][e];
  __syncthreads();
  for (int c = threadIdx.x; c < P; c += HEAD_THREADS) {
    float r = red[0][c];
#pragma unroll
    for (int w = 1; w < HEAD_THREADS / 64; ++w) r = MODE == 0 ? fmaxf(r, red[w][c]) : r + red[w][c];
    float* dst = (LIN ? hl.part : pooled) + (int64_t)b * P + c;   // LIN: the scratch row, read back by the last workgroup
    if (MODE == 0)   // non-negative floats order like their bit patterns
      atomicMax(reinterpret_cast<unsigned int*>(dst), __float_as_uint(r));
    else
      atomicAdd(dst, r);
  }
  if constexpr (LIN) head_linear_tail<8>(hl, b, P, pooled, &red[0][0]);   // (its barriers guard red's reuse)
}

// ---------------------------------------------------------------------------------------
// NonNegLinear: grid (image, class block of 16), one wave per 4 classes (nonneg_linear_wave): a
// lane owns the float4 slices 4 l + 256 i and keeps 4 class partials, four slices per unrolled step
// (C5: D = 6144, K = 9 -> 24 slices; C2: D = 768, K = 200 -> 13 blocks of 4 waves per image).  No
// cross-wave reduction: a class's sum is one wave's (batch-invariant, and the fused head's bits).
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(HEAD_THREADS) void nonneg_linear_kernel(const float* __restrict__ x, int D,
                                                                     const float* __restrict__ W,
                                                                     const float* __restrict__ bias, int K,
                                                                     int apply_thresh, float thresh,
                                                                     float* __restrict__ x_out,
                                                                     float* __restrict__ out) {
  constexpr int NCW = NN_CLS_PER_BLOCK / (HEAD_THREADS / 64);     // 4 classes per wave
  const int b = blockIdx.x, wv = threadIdx.x >> 6;
  const int k0 = blockIdx.y * NN_CLS_PER_BLOCK + wv * NCW;
  if (k0 >= K) return;                                             // wave-uniform, no barrier below
  nonneg_linear_wave<NCW, 4>(x + (int64_t)b * D, D, W, bias, k0, min(NCW, K - k0), out + (int64_t)b * K, apply_thresh,
                          thresh, (x_out && blockIdx.y == 0 && wv == 0) ? x_out + (int64_t)b * D : nullptr);
}

// Philox4x32-10 and the Exp(1) / log Exp(1) draws: philox.hpp (shared with the fused add-on
// GEMM's Gumbel epilogue, csrc/gemm_f32_impl.hpp).

// One wave per pixel, four consecutive channels per lane (float4 logits / proto): the noise
// of channels 4k..4k+3 of pixel (b, pix) is the Philox block (offset + (b*HW + pix)*P/4 + k)
// -- one block per four elements, no word wasted.  Per pixel: z = (x - log E) / tau, argmax
// (first index on ties), y_soft at the argmax = 1 / sum exp(z - max), one-hot written as
// (1 - y_soft) + y_soft (F.gumbel_softmax(hard=True)'s straight-through value).
// P % 4 == 0.
//
// SOFT (train mode, F.gumbel_softmax(hard=False), count_pipnet_utils.py:34-35): proto =
// softmax((x - log E) / tau) written for every channel, and the per-prototype spatial sums
// (the raw counts, count_pipnet.py:88) reduced per workgroup in LDS, one float atomic per
// (workgroup, channel) into `sums`.
constexpr int CG_PIX_PER_BLOCK = 16;        // 4 pixels per wave: C5 (64 x 256 px) -> 1024 workgroups

template <int NJ, bool SOFT = false, bool NOISE = false>   // NOISE: injected Exp(1) draw, else Philox
__global__ __launch_bounds__(HEAD_THREADS) void count_gumbel_kernel(const float* __restrict__ logits, int HW, int P,
                                                                    float inv_tau,
                                                                    const float* __restrict__ exp_noise,
                                                                    uint64_t seed, uint64_t offset,
                                                                    const uint64_t* __restrict__ seed_dev,
                                                                    float* __restrict__ proto,
                                                                    int32_t* __restrict__ hist,
                                                                    float* __restrict__ sums = nullptr) {
  constexpr int NJ4 = (NJ + 3) / 4;         // float4 channel chunks per lane (256 channels each)
  // hard head on Philox noise: hardware log2 / exp2 (~1 ulp) for the noise and the running
  // sum -- 3 transcendentals per element dominated its VALU time at C5
  constexpr bool FAST = !SOFT && !NOISE;
  if (seed_dev) seed = *seed_dev;            // graph-replay form: the seed lives in device memory
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.y;
  const int pix0 = blockIdx.x * CG_PIX_PER_BLOCK;
  float racc[SOFT ? NJ4 : 1][4];
  if constexpr (SOFT) {
#pragma unroll
    for (int j = 0; j < NJ4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) racc[j][e] = 0.f;
  }
  // the wave's pixels pix0 + wv, + 4, ...: the next pixel's logits are loaded before the
  // current pixel's noise / argmax / exp work, so HBM reads overlap the VALU part
  f32x4 xn[NJ4];
  auto load_px = [&](int pix) {
    const int64_t base = ((int64_t)b * HW + pix) * P;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      if (c < P) xn[j] = ld4(logits + base + c);
    }
  };
  if (pix0 + wv < HW) load_px(pix0 + wv);
  for (int pi = wv; pi < CG_PIX_PER_BLOCK; pi += HEAD_THREADS / 64) {
    const int pix = pix0 + pi;
    if (pix >= HW) break;
    const int64_t base = ((int64_t)b * HW + pix) * P;
    f32x4 xc[NJ4];
#pragma unroll
    for (int j = 0; j < NJ4; ++j) xc[j] = xn[j];
    if (pi + HEAD_THREADS / 64 < CG_PIX_PER_BLOCK && pix + HEAD_THREADS / 64 < HW) load_px(pix + HEAD_THREADS / 64);
    // hard (eval) head: one pass per lane with a running (max, first argmax, sum of exp(z - max))
    // -- no per-element z kept, so the kernel stays at 4 waves per SIMD; the lanes' sums are
    // rescaled to the wave max before the wave sum.  SOFT keeps z for the normalised write.
    float z[SOFT ? NJ4 : 1][4];
    float m = -INFINITY, ls = 0.f;
    int mi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      if (c < P) {
        float lE[4];                                       // log of the Exp(1) draw
        if constexpr (NOISE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) lE[e] = logf(exp_noise[((int64_t)b * P + c + e) * HW + pix]);   // NCHW draw
        } else {
          uint32_t w[4];
          philox4(seed, offset + (uint64_t)((base + c) >> 2), w);
#pragma unroll
          for (int e = 0; e < 4; ++e) lE[e] = FAST ? log_exp1_from_bits_fast(w[e]) : logf(exp1_from_bits(w[e]));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float zv = (xc[j][e] - lE[e]) * inv_tau;
          if constexpr (SOFT) {
            z[j][e] = zv;
            if (zv > m) { m = zv; mi = c + e; }
          } else {
            const bool up = zv > m;
            const float nd = up ? m - zv : zv - m;             // -|zv - m|; -inf first
            const float d = FAST ? __builtin_amdgcn_exp2f(nd * 1.44269504f) : expf(nd);
            ls = up ? fmaf(ls, d, 1.0f) : ls + d;
            if (up) { m = zv; mi = c + e; }
          }
        }
      } else if constexpr (SOFT) {
#pragma unroll
        for (int e = 0; e < 4; ++e) z[j][e] = -INFINITY;
      }
    }
    const float lm = m;
    // wave argmax, first index on ties
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(m, o, 64);
      const int oi = __shfl_xor(mi, o, 64);
      if (om > m || (om == m && oi < mi)) { m = om; mi = oi; }
    }
    float sum = 0.f;
    if constexpr (SOFT) {
#pragma unroll
      for (int j = 0; j < NJ4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float ez = (4 * lane + 256 * j < P) ? expf(z[j][e] - m) : 0.f;
          z[j][e] = ez;
          sum += ez;
        }
    } else {
      sum = lm == -INFINITY ? 0.f : ls * expf(lm - m);
    }
    if constexpr (SOFT) {
      const float inv = 1.0f / wave_sum(sum);
#pragma unroll
      for (int j = 0; j < NJ4; ++j) {
        const int c = 4 * lane + 256 * j;
        if (c < P) {
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            o[e] = z[j][e] * inv;
            racc[j][e] += o[e];
          }
          __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(proto + base + c));
        }
      }
      continue;
    }
    const float ysoft = 1.0f / wave_sum(sum);              // softmax value at the argmax
    const float hard = (1.0f - ysoft) + ysoft;             // y_hard - y_soft + y_soft
#pragma unroll
    for (int j = 0; j < NJ4; ++j) {
      const int c = 4 * lane + 256 * j;
      if (c < P) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (c + e == mi) ? hard : 0.f;
        __builtin_nontemporal_store(o, reinterpret_cast<f32x4*>(proto + base + c));
      }
    }
    if (lane == 0 && (unsigned)mi < (unsigned)P) atomicAdd(hist + (int64_t)b * P + mi, 1);   // NaN rows: no argmax
  }
  if constexpr (SOFT) {
    __shared__ float red[HEAD_THREADS / 64][NJ4 * 256];
#pragma unroll
    for (int j = 0; j < NJ4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[wv][4 * lane + 256 * j + e] = racc[j][e];
    __syncthreads();
    for (int c = threadIdx.x; c < P; c += HEAD_THREADS) {
      float r = red[0][c];
#pragma unroll
      for (int w = 1; w < HEAD_THREADS / 64; ++w) r += red[w][c];
      atomicAdd(sums + (int64_t)b * P + c, r);
    }
  }
}

__global__ void count_finish_kernel(const int32_t* __restrict__ hist, const float* __restrict__ sums, int64_t n,
                                    float max_count, int do_round, float* __restrict__ raw,
                                    float* __restrict__ clamped) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float c = hist ? (float)hist[i] : sums[i];
    if (raw) raw[i] = c;
    const float r = do_round ? rintf(c) : c;   // torch.round: half to even
    clamped[i] = fminf(fmaxf(r, 0.f), max_count);
  }
}

__global__ void count_encode_kernel(const float* __restrict__ x, int64_t BP, int C, int kind, int do_round,
                                    const float* __restrict__ w, float* __restrict__ out) {
  const int64_t n = BP * C;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bp = i / C;
    const int c = (int)(i - bp * C);
    float v = x[bp];
    if (kind == 0) {
      if (do_round) v = rintf(v);
      int idx = (int)v - 1;                    // .long() truncates toward zero
      idx = idx < 0 ? 0 : (idx > C - 1 ? C - 1 : idx);
      out[i] = (v > 0.1f && c == idx) ? 1.0f : 0.0f;
    } else {
      out[i] = v * w[c];
    }
  }
}

int nj_bucket(int P) {
  const int nj = (P + 63) / 64;
  if (nj <= 1) return 1;
  if (nj <= 2) return 2;
  if (nj <= 4) return 4;
  if (nj <= 8) return 8;
  if (nj <= 12) return 12;
  if (nj <= 16) return 16;
  if (nj <= 32) return 32;
  return -1;
}

}  // namespace

#define PIPNET_NJ_SWITCH(NJV, CALL) \
  switch (NJV) {                    \
    case 1: CALL(1); break;         \
    case 2: CALL(2); break;         \
    case 4: CALL(4); break;         \
    case 8: CALL(8); break;         \
    case 12: CALL(12); break;       \
    case 16: CALL(16); break;       \
    case 32: CALL(32); break;       \
    default: return PIPNET_ERR_ARG; \
  }

// softmax + pool (+ the fused NonNegLinear when hl.W is set: max pool only).  bf16 logits with
// P % 8 == 0, P <= 2048 and 16-B aligned operands take the quad-layout kernel.
template <typename T>
int head_launch(const T* feat, int B, int HW, int P, int pool_mode, float* proto, float* pooled, const HeadLinear& hl,
                void* stream) {
  const bool lin = hl.W != nullptr;
  if (B < 0 || HW <= 0 || P <= 0 || (pool_mode != 0 && pool_mode != 1) || (lin && pool_mode != 0)) return PIPNET_ERR_ARG;
  if (!feat || !proto || !pooled) return PIPNET_ERR_ARG;
  if (lin && (hl.K <= 0 || !hl.out || !hl.tickets || !hl.part)) return PIPNET_ERR_ARG;
  if (lin && (P & 3) == 0 && !aligned16(hl.W)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int nj = nj_bucket(P);
  if (nj < 0) return PIPNET_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (!lin && !zero_fill(pooled, (int64_t)B * P, s)) return PIPNET_ERR_LAUNCH;   // the fused head needs none
  const dim3 grid((HW + PIX_PER_BLOCK - 1) / PIX_PER_BLOCK, B);
  const dim3 block(HEAD_THREADS);
  constexpr bool BF = std::is_same<T, __bf16>::value;
  if (BF && P % 8 == 0 && P <= 2048 && aligned16(feat) && aligned16(proto)) {
    const __bf16* f = reinterpret_cast<const __bf16*>(feat);
#define SPQ_CALL(N)                                                                                      \
    if (lin) hipLaunchKernelGGL((softmax_pool_bf16q_kernel<N, 0, true>), grid, block, 0, s, f, HW, P, proto, pooled, hl); \
    else if (pool_mode == 0) hipLaunchKernelGGL((softmax_pool_bf16q_kernel<N, 0>), grid, block, 0, s, f, HW, P, proto, pooled, hl); \
    else hipLaunchKernelGGL((softmax_pool_bf16q_kernel<N, 1>), grid, block, 0, s, f, HW, P, proto, pooled, hl);
    if (P <= 512) {
      SPQ_CALL(1)
    } else if (P <= 1024) {
      SPQ_CALL(2)
    } else {
      SPQ_CALL(4)
    }
#undef SPQ_CALL
  } else {
#define SP_CALL(N)                                                                                          \
    if (lin) hipLaunchKernelGGL((softmax_pool_kernel<N, 0, T, true>), grid, block, 0, s, feat, HW, P, proto, pooled, hl); \
    else if (pool_mode == 0) hipLaunchKernelGGL((softmax_pool_kernel<N, 0, T>), grid, block, 0, s, feat, HW, P, proto, pooled, hl); \
    else hipLaunchKernelGGL((softmax_pool_kernel<N, 1, T>), grid, block, 0, s, feat, HW, P, proto, pooled, hl);
    PIPNET_NJ_SWITCH(nj, SP_CALL)
#undef SP_CALL
  }
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_softmax_pool_f32(const float* feat, int B, int HW, int P, int pool_mode, float* proto,
                                       float* pooled, void* stream) {
  return head_launch(feat, B, HW, P, pool_mode, proto, pooled, HeadLinear{}, stream);
}

extern "C" int pipnet_softmax_pool_bf16(const void* feat, int B, int HW, int P, int pool_mode, float* proto,
                                        float* pooled, void* stream) {
  return head_launch(reinterpret_cast<const __bf16*>(feat), B, HW, P, pool_mode, proto, pooled, HeadLinear{}, stream);
}

extern "C" int pipnet_softmax_pool_linear_f32(const float* feat, int B, int HW, int P, float* proto, float* pooled,
                                              const float* W, const float* bias, int K, int apply_thresh,
                                              float thresh, float* x_out, float* out, float* part,
                                              int32_t* tickets, void* stream) {
  if (!W) return PIPNET_ERR_ARG;
  return head_launch(feat, B, HW, P, 0, proto, pooled,
                     HeadLinear{W, bias, K, apply_thresh, thresh, x_out, out, tickets, part}, stream);
}

extern "C" int pipnet_softmax_pool_linear_bf16(const void* feat, int B, int HW, int P, float* proto, float* pooled,
                                               const float* W, const float* bias, int K, int apply_thresh,
                                               float thresh, float* x_out, float* out, float* part,
                                               int32_t* tickets, void* stream) {
  if (!W) return PIPNET_ERR_ARG;
  return head_launch(reinterpret_cast<const __bf16*>(feat), B, HW, P, 0, proto, pooled,
                     HeadLinear{W, bias, K, apply_thresh, thresh, x_out, out, tickets, part}, stream);
}

extern "C" int64_t pipnet_softmax_pool_linear_part_floats(int B, int HW, int P) {
  return (B < 0 || HW <= 0 || P <= 0) ? 0 : head_part_floats(B, HW, P);
}

extern "C" int pipnet_nonneg_linear_f32(const float* x, int B, int D, const float* W, const float* bias, int K,
                                        int apply_thresh, float thresh, float* x_out, float* out, void* stream) {
  if (B < 0 || D <= 0 || K <= 0 || !x || !W || !out) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  if ((D & 3) == 0 && (!aligned16(W) || !aligned16(x))) return PIPNET_ERR_ALIGN;
  const dim3 grid(B, (K + NN_CLS_PER_BLOCK - 1) / NN_CLS_PER_BLOCK);
  hipLaunchKernelGGL(nonneg_linear_kernel, grid, dim3(HEAD_THREADS), 0, (hipStream_t)stream, x,
                     D, W, bias, K, apply_thresh, thresh, x_out, out);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

namespace {
int count_gumbel_launch(const float* logits, int B, int HW, int P, float tau, const float* exp_noise, uint64_t seed,
                        uint64_t offset, const uint64_t* seed_dev, float* proto, int32_t* hist, void* stream) {
  if (B < 0 || HW <= 0 || P <= 0 || (P & 3) || !(tau > 0.f) || !logits || !proto || !hist) return PIPNET_ERR_ARG;
  if (!aligned16(logits) || !aligned16(proto)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int nj = nj_bucket(P);
  if (nj < 0) return PIPNET_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (!zero_fill(hist, (int64_t)B * P, s)) return PIPNET_ERR_LAUNCH;
  const dim3 grid((HW + CG_PIX_PER_BLOCK - 1) / CG_PIX_PER_BLOCK, B);
  const float inv_tau = 1.0f / tau;
#define CG_CALL(N)                                                                                              \
  if (exp_noise)                                                                                                \
    hipLaunchKernelGGL((count_gumbel_kernel<N, false, true>), grid, dim3(HEAD_THREADS), 0, s, logits, HW, P, inv_tau, \
                       exp_noise, seed, offset, seed_dev, proto, hist);                                          \
  else                                                                                                          \
    hipLaunchKernelGGL((count_gumbel_kernel<N, false, false>), grid, dim3(HEAD_THREADS), 0, s, logits, HW, P, inv_tau, \
                       exp_noise, seed, offset, seed_dev, proto, hist);
  PIPNET_NJ_SWITCH(nj, CG_CALL)
#undef CG_CALL
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

// splitmix64 step of the device-resident Philox key (one thread).
__global__ void seed_advance_kernel(uint64_t* seed) {
  uint64_t z = (*seed += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  seed[1] = z ^ (z >> 31);
}
// The head's noise draw on its own: element i of a [n] stream (n % 4 == 0) = the Exp(1) value
// (log_e = 0: exp1_from_bits, the soft / injected-form libm draw) or its log on the hard head's
// hardware-log form (log_e = 1: log_exp1_from_bits_fast) of word i % 4 of Philox block offset + i / 4
// -- exactly what count_gumbel_kernel consumes for element i of its NHWC [B, HW, P] map.
__global__ __launch_bounds__(256) void philox_exp1_kernel(uint64_t seed, uint64_t offset, int64_t nblk, int log_e,
                                                          float* __restrict__ out) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nblk; q += (int64_t)gridDim.x * blockDim.x) {
    uint32_t w[4];
    philox4(seed, offset + (uint64_t)q, w);
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = log_e ? log_exp1_from_bits_fast(w[e]) : exp1_from_bits(w[e]);
    st4(out + 4 * q, o);
  }
}
}  // namespace

extern "C" int pipnet_philox_exp1_f32(uint64_t seed, uint64_t offset, int64_t n, int log_e, float* out, void* stream) {
  if (n < 0 || (n & 3) || (log_e != 0 && log_e != 1) || (n > 0 && !out)) return PIPNET_ERR_ARG;
  if (!aligned16(out)) return PIPNET_ERR_ALIGN;
  if (n == 0) return PIPNET_OK;
  const int64_t nblk = n / 4;
  const int64_t g = (nblk + 255) / 256;
  hipLaunchKernelGGL(philox_exp1_kernel, dim3((unsigned)(g < 16384 ? g : 16384)), dim3(256), 0, (hipStream_t)stream,
                     seed, offset, nblk, log_e, out);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_count_gumbel_f32(const float* logits, int B, int HW, int P, float tau, const float* exp_noise,
                                       uint64_t seed, uint64_t offset, float* proto, int32_t* hist, void* stream) {
  return count_gumbel_launch(logits, B, HW, P, tau, exp_noise, seed, offset, nullptr, proto, hist, stream);
}

extern "C" int pipnet_count_gumbel_devseed_f32(const float* logits, int B, int HW, int P, float tau,
                                               uint64_t* seed_state, float* proto, int32_t* hist, void* stream) {
  if (!seed_state) return PIPNET_ERR_ARG;
  if (B <= 0) return count_gumbel_launch(logits, B, HW, P, tau, nullptr, 0, 0, seed_state + 1, proto, hist, stream);
  hipLaunchKernelGGL(seed_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, seed_state);
  PIPNET_CHECK_LAUNCH();
  return count_gumbel_launch(logits, B, HW, P, tau, nullptr, 0, 0, seed_state + 1, proto, hist, stream);
}

// Train-mode (soft) Gumbel head: proto = softmax((x - log E) / tau) [B,HW,P], sums [B,P] = spatial
// sums (the raw counts; zeroed here).  exp_noise as pipnet_count_gumbel_f32 (NCHW) or NULL (Philox).
extern "C" int pipnet_count_gumbel_soft_f32(const float* logits, int B, int HW, int P, float tau,
                                            const float* exp_noise, uint64_t seed, uint64_t offset, float* proto,
                                            float* sums, void* stream) {
  if (B < 0 || HW <= 0 || P <= 0 || (P & 3) || !(tau > 0.f) || !logits || !proto || !sums) return PIPNET_ERR_ARG;
  if (!aligned16(logits) || !aligned16(proto)) return PIPNET_ERR_ALIGN;
  if (B == 0) return PIPNET_OK;
  const int nj = nj_bucket(P);
  if (nj < 0) return PIPNET_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (!zero_fill(reinterpret_cast<uint32_t*>(sums), (int64_t)B * P, s)) return PIPNET_ERR_LAUNCH;
  const dim3 grid((HW + CG_PIX_PER_BLOCK - 1) / CG_PIX_PER_BLOCK, B);
  const float inv_tau = 1.0f / tau;
#define CG_CALL(N)                                                                                                \
  if (exp_noise)                                                                                                  \
    hipLaunchKernelGGL((count_gumbel_kernel<N, true, true>), grid, dim3(HEAD_THREADS), 0, s, logits, HW, P, inv_tau, \
                       exp_noise, seed, offset, nullptr, proto, nullptr, sums);                                    \
  else                                                                                                            \
    hipLaunchKernelGGL((count_gumbel_kernel<N, true, false>), grid, dim3(HEAD_THREADS), 0, s, logits, HW, P, inv_tau, \
                       exp_noise, seed, offset, nullptr, proto, nullptr, sums);
  PIPNET_NJ_SWITCH(nj, CG_CALL)
#undef CG_CALL
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_count_finish_f32(const int32_t* hist, const float* sums, int B, int P, int max_count,
                                       int do_round, float* counts_raw, float* clamped, void* stream) {
  if (B < 0 || P <= 0 || max_count < 0 || (!hist && !sums) || !clamped) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  const int64_t n = (int64_t)B * P;
  const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(count_finish_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, hist, sums, n,
                     (float)max_count, do_round, counts_raw, clamped);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_count_encode_f32(const float* x, int B, int P, int C, int kind, int do_round, const float* w,
                                       float* out, void* stream) {
  if (B < 0 || P <= 0 || C <= 0 || (kind != 0 && kind != 1) || !x || !out || (kind == 1 && !w)) return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  const int64_t n = (int64_t)B * P * C;
  const int blocks = (int)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
  hipLaunchKernelGGL(count_encode_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, (int64_t)B * P, C,
                     kind, do_round, w, out);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_amd_abi_version(void) { return PIPNET_AMD_ABI_VERSION; }

// sha256 over the library's sources (csrc/*.hip, csrc/*.hpp, include/*.h), computed by
// count_pipnet_amd/build.py and passed on the hipcc line; _lib.load() compares it with the
// tree it runs from, so a shipped binary built from other sources fails loudly.
#ifndef PIPNET_SRC_DIGEST
#define PIPNET_SRC_DIGEST "unknown"
#endif
extern "C" const char* pipnet_amd_source_digest(void) { return PIPNET_SRC_DIGEST; }

extern "C" const char* pipnet_amd_status_string(int status) {
  switch (status) {
    case PIPNET_OK: return "ok";
    case PIPNET_ERR_ARG: return "invalid argument (shape/size/configuration)";
    case PIPNET_ERR_ALIGN: return "pointer or leading dimension not 16-byte aligned";
    case PIPNET_ERR_LAUNCH: return "kernel launch failed";
    case PIPNET_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
  }
}
