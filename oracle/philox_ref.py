"""ORACLE -- CPU restatement of the HIP Gumbel head's Exp(1) noise draw (Philox4x32-10).

TEST INFRASTRUCTURE ONLY.  Only ``tests/`` (and ``__graft_entry__.smoke()``) may import this
module, and only as the checker -- the product draws its noise on the device
(``count_pipnet_amd/csrc/philox.hpp``) and never calls into ``oracle/``.

Why it exists.  The reference's hard Gumbel-softmax (``pipnet/count_pipnet_utils.py:23-38``:
``F.gumbel_softmax(x, tau, hard=True, dim=1)``) draws its noise as ``-torch.empty_like(x)
.exponential_().log()`` from torch's device RNG, whose stream is implementation-specific and
cannot be reproduced on another device.  The HIP path therefore draws Exp(1) from a
counter-based generator keyed by (seed, element index) -- fresh noise per call, as the
reference -- and this module restates that draw exactly (numpy uint32 arithmetic), so the
default (device-seeded) C5 forward can be checked element by element against the reference
algorithm fed the SAME Exp(1) values (``oracle.ref_cpu.gumbel_softmax_hard``).

Algorithm (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11;
Random123's philox4x32, 10 rounds).  Pinned by the published Random123 known-answer vectors
(``tests/test_philox_oracle.py``).  Layout, as ``csrc/head.hip`` count_gumbel_kernel and
``csrc/philox.hpp`` draw it:
  * the NHWC element (b, pix, c) of a [B, HW, P] head (P % 4 == 0) has linear index
    i = (b*HW + pix)*P + c and takes word i % 4 of the Philox block with counter
    ``offset + i // 4`` (64-bit, words 2-3 of the counter zero) under the 64-bit key ``seed``;
  * u = (float32(k) + 0.5f) * 2^-24 in fp32 with k = w >> 8 (round to nearest even: for
    k >= 2^23 the half is lost to the tie -- k + 1/2 needs 25 bits -- and the top value k = 2^24 - 1
    rounds to u = 1.0), E = -log(u), floored at 2^-25 (below every other draw, so the u = 1.0
    case cannot give E = 0 and log E = -inf).
"""
from __future__ import annotations

import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint64(0x9E3779B9)
W1 = np.uint64(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)
E_FLOOR = 2.0 ** -25


def philox4x32(ctr: np.ndarray, key: np.ndarray, rounds: int = 10) -> np.ndarray:
    """Philox4x32-R: ctr uint32 [..., 4], key uint32 [2] (or [..., 2]) -> uint32 [..., 4].
    One round: (hi0, lo0) = M0 * c0, (hi1, lo1) = M1 * c2;
    c = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0); then the key is bumped by the Weyl constants
    (csrc/philox.hpp:15-31)."""
    ctr = np.asarray(ctr, dtype=np.uint32)
    key = np.asarray(key, dtype=np.uint32)
    c0, c1, c2, c3 = (ctr[..., i].astype(np.uint64) for i in range(4))
    k0 = np.broadcast_to(key[..., 0], ctr.shape[:-1]).astype(np.uint64)
    k1 = np.broadcast_to(key[..., 1], ctr.shape[:-1]).astype(np.uint64)
    for _ in range(rounds):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0)
        k0 = (k0 + W0) & MASK32           # uint32 wrap-around
        k1 = (k1 + W1) & MASK32
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


def philox_blocks(seed: int, counters: np.ndarray) -> np.ndarray:
    """The device's philox4(seed, ctr) for 64-bit counters ``counters`` -> uint32 [n, 4]."""
    seed &= (1 << 64) - 1
    counters = np.asarray(counters, dtype=np.uint64)
    ctr = np.zeros(counters.shape + (4,), dtype=np.uint32)
    ctr[..., 0] = (counters & MASK32).astype(np.uint32)
    ctr[..., 1] = (counters >> np.uint64(32)).astype(np.uint32)
    key = np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)
    return philox4x32(ctr, key)


def exp1_from_words(w: np.ndarray) -> np.ndarray:
    """csrc/philox.hpp exp1_from_bits: the fp32 uniform of the word's top 24 bits, E = -log u
    (fp64 here; the device's libm logf is within an ulp), floored at 2^-25.  Returns float64."""
    u = (np.asarray(w, dtype=np.uint32) >> np.uint32(8)).astype(np.float32)
    u = (u + np.float32(0.5)) * np.float32(1.0 / 16777216.0)       # fp32 RNE, as the kernel
    return np.maximum(-np.log(u.astype(np.float64)), E_FLOOR)


def exp1_noise_nhwc(seed: int, offset: int, B: int, HW: int, P: int) -> np.ndarray:
    """The Exp(1) draw of a [B, HW, P] NHWC head with Philox key ``seed`` starting at block
    ``offset`` (count_gumbel_kernel's layout) -> float64 [B, HW, P]."""
    if P % 4:
        raise ValueError("the Philox head needs P % 4 == 0")
    n = B * HW * P
    words = philox_blocks(seed, np.uint64(offset) + np.arange(n // 4, dtype=np.uint64))
    return exp1_from_words(words.reshape(-1)).reshape(B, HW, P)


def exp1_noise_nchw(seed: int, offset: int, B: int, H: int, W: int, P: int) -> np.ndarray:
    """Same draw as an NCHW [B, P, H, W] map (the layout the reference's GumbelSoftmax and
    ``oracle.ref_cpu.gumbel_softmax_hard`` take)."""
    e = exp1_noise_nhwc(seed, offset, B, H * W, P)
    return np.ascontiguousarray(e.reshape(B, H, W, P).transpose(0, 3, 1, 2))
