// Philox4x32-10 (Salmon et al., SC'11) -> one Exp(1) draw per element index: the hard Gumbel
// head's noise (head.hip count_gumbel_kernel; channels 4k..4k+3 of pixel row m draw Philox block
// offset + (m P + 4k) / 4).  A header of its own so that any kernel fusing the head draws the same
// noise (round 5 measured one such fusion, profiles/r05/fused_addon_gumbel.patch).
#pragma once
#include "common.hpp"

PIPNET_DEV uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
  const uint64_t p = (uint64_t)a * b;
  hi = (uint32_t)(p >> 32);
  return (uint32_t)p;
}

// One Philox4x32-10 block: four 32-bit words for counter `ctr` under key `seed`.
PIPNET_DEV void philox4(uint64_t seed, uint64_t ctr, uint32_t (&out)[4]) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0u, c3 = 0u;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, hi1;
    const uint32_t lo0 = mulhilo(0xD2511F53u, c0, hi0);
    const uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, hi1);
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0, out[1] = c1, out[2] = c2, out[3] = c3;
}

// E = -log u of the word's top 24 bits, u = (k + 1/2) 2^-24.  In fp32 the top value k = 2^24 - 1
// rounds to u = 1.0 (16777215.5 needs 25 bits; ties to even), so E would be 0 and log E = -inf --
// the soft head's z = +inf and its softmax NaN, once in 2^24 draws.  E is floored at
// 2^-25 (below every other draw's value, >= 8.9e-8), which changes only that one case.
// oracle/philox_ref.py restates this draw.
PIPNET_DEV float exp1_from_bits(uint32_t w) {
  const float u = ((float)(w >> 8) + 0.5f) * (1.0f / 16777216.0f);   // (0, 1]
  return fmaxf(-logf(u), 2.98023224e-8f);
}

// log E for E = -log u of the same 24-bit uniform, on the hardware log2 (v_log_f32):
// ln E = ln2 * log2(-log2 u) + ln(ln2).  The same floor E >= 2^-25, i.e. -log2 u >= 2^-25 / ln2;
// v_log_f32 returns 0 for u within a few ulp of 1 (and u = 1.0 exactly, above), which made log E =
// -inf, z = +inf and the
// pixel's one-hot value NaN (inf - inf in the exp-sum) about twice per C5 forward -- the inner
// value is clamped to that bound (every other draw unchanged).  For the hard Philox head only --
// its noise is this library's own draw; the injected-noise and soft paths keep the libm forms
// they share with the oracle.
PIPNET_DEV float log_exp1_from_bits_fast(uint32_t w) {
  const float u = ((float)(w >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float t = fmaxf(-__builtin_amdgcn_logf(u), 4.2995e-8f);
  return fmaf(__builtin_amdgcn_logf(t), 0.69314718f, -0.36651292f);
}

