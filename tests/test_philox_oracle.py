"""The Philox Exp(1) oracle (oracle/philox_ref.py) -- the restatement the device-seeded Gumbel head
is checked against (tests/test_gpu_philox.py) -- pinned on the CPU:

* Philox4x32-10 against the published Random123 known-answer vectors (kat_vectors, philox4x32 R=10:
  zero counter / key, all-ones, and the pi-digit counter / key);
* the draw's edge cases: the top uniform rounds to u = 1.0 in fp32 and is floored at E = 2^-25
  (csrc/philox.hpp exp1_from_bits), the smallest uniform gives E = -log(2^-25);
* the head's layout: element i of the NHWC stream = word i % 4 of block offset + i / 4, so a
  sub-batch starting at block offset b0*HW*P/4 continues the full batch's stream exactly (the
  two-stream split in count_pipnet.py);
* the draw is Exp(1) (mean / variance / an upper quantile on 4M samples).
"""
import numpy as np

from oracle import philox_ref as PR

KAT = [  # (ctr[4], key[2]) -> out[4]   Random123 kat_vectors, philox4x32 10 rounds
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox4x32_10_known_answers():
    for ctr, key, want in KAT:
        got = PR.philox4x32(np.array(ctr, dtype=np.uint32), np.array(key, dtype=np.uint32))
        assert [int(v) for v in got] == list(want), (ctr, key)
    # vectorised over counters = one call per counter
    ctrs = np.array([k[0] for k in KAT], dtype=np.uint32)
    keys = np.array([k[1] for k in KAT], dtype=np.uint32)
    got = PR.philox4x32(ctrs, keys)
    assert [[int(v) for v in r] for r in got] == [list(k[2]) for k in KAT]


def test_philox_blocks_64bit_counter():
    """The device forms ctr = (lo32, hi32, 0, 0) from a 64-bit counter and key = (lo32, hi32)
    from the 64-bit seed (csrc/philox.hpp philox4)."""
    seed = 0x299F31D0A4093822
    c = np.array([0x85A308D3243F6A88, 2 ** 32 - 1, 2 ** 32], dtype=np.uint64)
    got = PR.philox_blocks(seed, c)
    for i, cc in enumerate(c):
        ctr = np.array([int(cc) & 0xFFFFFFFF, int(cc) >> 32, 0, 0], dtype=np.uint32)
        ref = PR.philox4x32(ctr, np.array([0xA4093822, 0x299F31D0], dtype=np.uint32))
        assert np.array_equal(got[i], ref)


def test_exp1_edges():
    w = np.array([0xFFFFFFFF, 0xFFFFFF00, 0xFFFFFE00, 0x000000FF, 0], dtype=np.uint32)
    e = PR.exp1_from_words(w)
    # top 24 bits all ones: u = (2^24 - 1/2) 2^-24 rounds to 1.0 in fp32 -> floored
    assert e[0] == PR.E_FLOOR and e[1] == PR.E_FLOOR
    # k = 2^24 - 2: k + 1/2 ties to the even 2^24 - 2 (every k >= 2^23 loses its 1/2 this way), so
    # u = 1 - 2^-23 and E = 2^-23 to first order, above the floor
    assert abs(e[2] - 2.0 ** -23) < 1e-13 and e[2] > PR.E_FLOOR
    # smallest uniform: u = 2^-25 exactly -> E = 25 ln 2
    assert abs(e[3] - 25 * np.log(2.0)) < 1e-12 and e[3] == e[4]
    assert np.isfinite(np.log(e)).all()


def test_noise_layout_and_substream_offsets():
    seed, B, HW, P = 1234567, 3, 5, 8
    full = PR.exp1_noise_nhwc(seed, 0, B, HW, P)
    # the second image alone, starting at its own block offset (count_pipnet.py's split streams)
    one = PR.exp1_noise_nhwc(seed, 1 * HW * P // 4, 1, HW, P)
    assert np.array_equal(full[1:2], one)
    # element (b, pix, c) = word c % 4 of block (b*HW + pix)*P/4 + c/4
    words = PR.philox_blocks(seed, np.array([(2 * HW + 3) * P // 4 + 1], dtype=np.uint64))[0]
    assert np.array_equal(full[2, 3, 4:8], PR.exp1_from_words(words))
    nchw = PR.exp1_noise_nchw(seed, 0, B, 1, HW, P)
    assert nchw.shape == (B, P, 1, HW) and np.array_equal(nchw[:, :, 0, :], full.transpose(0, 2, 1))


def test_exp1_distribution():
    e = PR.exp1_noise_nhwc(99, 12345, 16, 256, 1024).ravel()         # 4M draws
    n = e.size
    assert abs(e.mean() - 1.0) < 5 * 1.0 / np.sqrt(n)
    assert abs(e.var() - 1.0) < 5 * np.sqrt(8.0 / n)
    q = np.mean(e > np.log(100.0))                                      # P(E > ln 100) = 1 %
    assert abs(q - 0.01) < 5 * np.sqrt(0.01 * 0.99 / n)
