// Shared device helpers for the gfx950 (MI355X, CDNA4) PIP-Net kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pipnet_amd.h"

#define PIPNET_DEV __device__ __forceinline__

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- wave64 reductions (butterfly over all 64 lanes) ----
PIPNET_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
PIPNET_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

PIPNET_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// Retire every outstanding vector-memory load with a wait hipcc's wait-count pass can see (an
// asm waitcnt is opaque to it).  Epilogues call it once, after their bias / residual preloads
// and before their row-guarded store loop: the pass cannot count stores issued inside
// `if (m < M)` branches, so without it every use of a preloaded register waited vmcnt(0) --
// for all the earlier stores of the loop as well (round 4, profiles/r04/epilogue_vmcnt_ab.txt).
PIPNET_DEV void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0F70); }   // vmcnt(0), gfx9 encoding
PIPNET_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// exact (erf) GELU, torch nn.GELU(approximate='none')
PIPNET_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

// GELU by Abramowitz & Stegun 7.1.28, erf(u) = 1 - (1 + a1 u + ... + a6 u^6)^-16 (|error| <
// 3e-7), rearranged branch-free: GELU(x) = relu(x) - |x|/2 * r with r = p(|x|/2)^-16 (the
// sqrt2 scalings folded into the coefficients): one transcendental (rcp) per element, the
// rest packed -- about 8.5 VALU issues per element.  |GELU error| < 1e-6 on [-10, 10]
// (fp32 emulation); p^16 overflows to inf for |x| > ~25, where r = 0 is exact.
PIPNET_DEV f32x2 gelu_pk16(f32x2 x) {
  const f32x2 hx = x * 0.5f;
  const f32x2 ahx = {fabsf(hx[0]), fabsf(hx[1])};
  f32x2 p = __builtin_elementwise_fma(ahx, (f32x2)0.00034451040f, (f32x2)0.0015645004f);
  p = __builtin_elementwise_fma(ahx, p, (f32x2)0.00060805720f);
  p = __builtin_elementwise_fma(ahx, p, (f32x2)0.026221010f);
  p = __builtin_elementwise_fma(ahx, p, (f32x2)0.084564020f);
  p = __builtin_elementwise_fma(ahx, p, (f32x2)0.099734694f);
  p = __builtin_elementwise_fma(ahx, p, (f32x2)1.0f);
  p = p * p;
  p = p * p;
  p = p * p;
  p = p * p;
  const f32x2 r = {__builtin_amdgcn_rcpf(p[0]), __builtin_amdgcn_rcpf(p[1])};
  return __builtin_elementwise_fma(-ahx, r, hx + ahx);
}

// fp32 -> (hi, lo) bf16 pair for the split-bf16 ("bf16x3") GEMMs: hi = RNE(x), lo =
// RNE(x - hi) (x - hi is exact in fp32), so x = hi + lo to ~2^-17 relative.
PIPNET_DEV void split_bf16(float x, __bf16& hi, __bf16& lo) {
  hi = (__bf16)x;
  lo = (__bf16)(x - (float)hi);
}

// Block-id remap: blocks b and b+8 share an XCD under round-robin dispatch (speed only,
// never correctness); give each XCD group a contiguous range of tile ids.  Bijective for
// any grid size (cdna_hip_programming.md section 5, "XCD swizzle must be bijective").
PIPNET_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = bid & 7, l = bid >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + l;
}

#define PIPNET_CHECK_LAUNCH()                                   \
  do {                                                          \
    hipError_t _e = hipGetLastError();                          \
    if (_e != hipSuccess) return PIPNET_ERR_LAUNCH;             \
  } while (0)

static inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
