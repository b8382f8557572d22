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
PIPNET_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// exact (erf) GELU, torch nn.GELU(approximate='none')
PIPNET_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }

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
