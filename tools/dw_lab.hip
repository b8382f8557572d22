// Tuning lab for the depthwise 7x7 + LayerNorm kernel (not part of the product ABI):
// v0 = the register-tile kernel (convnext_dw.hpp), v1.. = row-ring variants (dw_ring_lab.hpp).
#include "../count_pipnet_amd/csrc/convnext_dw.hpp"
#include "dw_ring_lab.hpp"
#include "dw_lds_lab.hpp"
#include "dw_lnr_lab.hpp"
using namespace pipnet_dw;

extern "C" int lab_dw(int variant, const float* x, int B, int H, int W, int C, const float* wp, const float* bias,
                      const float* lnw, const float* lnb, float* y, void* stream, int min_wg, int min_rh) {
  hipStream_t s = (hipStream_t)stream;
#define V(ID, CC, TX, TY, MB, LPP) \
  if (variant == ID && C == CC) return launch_dw<CC, TX, TY, MB, false, LPP>(x, B, H, W, wp, bias, lnw, lnb, y, s);
#define R(ID, CC, TX, NS, MB, LPP)                                                                                 \
  if (variant == ID && C == CC)                                                                                     \
    return launch_dw_ring<CC, TX, NS, MB, false, LPP>(x, B, H, W, wp, bias, lnw, lnb, y, s, min_wg, min_rh);
  V(0, 96, 7, 1, 1, 16) V(0, 192, 7, 1, 1, 16) V(0, 384, 7, 1, 2, 32) V(0, 768, 13, 1, 1, 64)
  // v5-v7: tile kernel with the vectorised LayerNorm (LPP = C / 12) at other tiles
  V(5, 96, 7, 1, 1, 8) V(5, 192, 7, 1, 1, 16) V(5, 384, 7, 1, 2, 32) V(5, 768, 13, 1, 1, 64)
  V(6, 96, 7, 1, 2, 8) V(6, 192, 7, 1, 2, 16) V(6, 384, 14, 1, 1, 32) V(6, 768, 7, 1, 2, 64)
  V(7, 96, 14, 1, 1, 8) V(7, 192, 14, 1, 1, 16) V(7, 384, 7, 2, 1, 32) V(7, 768, 13, 1, 2, 64)
  // v8-v10: narrower column tiles for small maps (a row tile of G * TX pixels against W = 32 / 16)
  V(8, 96, 4, 1, 1, 8) V(8, 192, 4, 1, 1, 16) V(9, 96, 4, 2, 1, 8) V(9, 192, 4, 2, 1, 16)
  V(10, 96, 2, 2, 1, 8) V(10, 192, 2, 2, 1, 16)
  // v50-v53 (round 4): the v40-v43 tiles with the LayerNorm in registers (dw_lnr_lab.hpp)
#define LN(ID, CC, TX, TY) \
  if (variant == ID && C == CC) return launch_dw_lnr<CC, TX, TY, 1>(x, B, H, W, wp, bias, lnw, lnb, y, s);
  LN(50, 96, 7, 2) LN(50, 192, 7, 2) LN(50, 384, 7, 2) LN(50, 768, 7, 2)
  LN(51, 96, 7, 3) LN(51, 192, 7, 3) LN(51, 384, 7, 3) LN(51, 768, 7, 3)
  LN(52, 96, 4, 2) LN(52, 192, 4, 2) LN(52, 384, 4, 2) LN(52, 768, 4, 2)
  LN(53, 96, 4, 4) LN(53, 192, 4, 4) LN(53, 384, 4, 4) LN(53, 768, 13, 1)
#undef LN
  // v40-v43 (round 4): taller tiles now that each weight row is loaded once per workgroup
  V(40, 96, 7, 2, 1, 8) V(40, 192, 7, 2, 1, 16) V(40, 384, 7, 2, 1, 32) V(40, 768, 7, 2, 1, 64)
  V(41, 96, 7, 3, 1, 8) V(41, 192, 7, 3, 1, 16) V(41, 384, 7, 3, 1, 32) V(41, 768, 7, 3, 1, 64)
  V(42, 96, 4, 2, 1, 8) V(42, 192, 4, 2, 1, 16) V(42, 384, 4, 2, 1, 32) V(42, 768, 4, 2, 1, 64)
  V(43, 96, 4, 4, 1, 8) V(43, 192, 4, 4, 1, 16) V(43, 384, 4, 4, 1, 32) V(43, 768, 4, 4, 1, 64)
  R(1, 96, 4, 4, 2, 16) R(2, 96, 2, 4, 3, 16) R(3, 96, 4, 8, 1, 16) R(4, 96, 3, 4, 2, 16)
  R(1, 192, 4, 2, 2, 16) R(2, 192, 2, 2, 3, 16) R(3, 192, 4, 4, 1, 16) R(4, 192, 3, 2, 2, 16)
  R(1, 384, 4, 1, 2, 32) R(2, 384, 2, 1, 3, 32) R(3, 384, 4, 2, 1, 32) R(4, 384, 3, 1, 2, 32)
  R(1, 768, 2, 1, 1, 64) R(2, 768, 4, 1, 1, 64) R(3, 768, 2, 1, 1, 32) R(4, 768, 3, 1, 1, 64)
  // v30 / v31: LDS-staged kernel (dwconv7_ln_lds_kernel) with 16- / 32-wide column tiles
#define L(ID, CC, TWC) \
  if (variant == ID && C == CC) return launch_dw_lds<CC, TWC>(x, B, H, W, wp, bias, lnw, lnb, y, s);
  L(30, 96, 16) L(30, 192, 16) L(30, 384, 16) L(31, 96, 32) L(31, 192, 32) L(31, 384, 32)
#undef L
  // v32-v37: ablations of v30 (ABL bits: 1 no DMA after chunk 0, 2 no weight loads, 4 no row reads / FMAs)
#define LA(ID, CC, ABL) \
  if (variant == ID && C == CC) return launch_dw_lds<CC, 16, false, ABL>(x, B, H, W, wp, bias, lnw, lnb, y, s);
  LA(32, 96, 1) LA(33, 96, 2) LA(34, 96, 4) LA(35, 96, 3) LA(36, 96, 6) LA(37, 96, 5)
  LA(32, 384, 1) LA(33, 384, 2) LA(34, 384, 4) LA(35, 384, 3) LA(36, 384, 6) LA(37, 384, 5)
#undef LA
  // ablations of v1 (ABL bits: 1 no LayerNorm, 2 no FMAs, 4 no input loads)
#define A(ID, CC, TX, NS, MB, LPP, ABL)                                                                            \
  if (variant == ID && C == CC)                                                                                     \
    return launch_dw_ring<CC, TX, NS, MB, false, LPP, ABL>(x, B, H, W, wp, bias, lnw, lnb, y, s, min_wg, min_rh);
  A(11, 96, 4, 4, 2, 16, 1) A(12, 96, 4, 4, 2, 16, 2) A(14, 96, 4, 4, 2, 16, 4) A(13, 96, 4, 4, 2, 16, 3)
  A(16, 96, 4, 4, 2, 16, 6)
  A(11, 384, 4, 1, 2, 32, 1) A(12, 384, 4, 1, 2, 32, 2) A(14, 384, 4, 1, 2, 32, 4) A(13, 384, 4, 1, 2, 32, 3)
  A(16, 384, 4, 1, 2, 32, 6)
#undef A
  // v60-v69 (round 6): ablations of the PRODUCT kernels (dwconv7_ln_abl_kernel = the product body with
  // ABL bits: 1 no LN statistics, 2 one FMA per row, 4 no input loads, 8 no stores, 16 no weight
  // loads, 32 no LDS tile round trip) at the product's tiles: 384 -> (7, 3), 768 -> (13, 1), 96 -> (7, 2)
#define PA(ID, ABL)                                                                                                 \
  if (variant == ID && C == 384) return launch_dw_abl<384, 7, 3, 1, 32, ABL>(x, B, H, W, wp, bias, lnw, lnb, y, s); \
  if (variant == ID && C == 768) return launch_dw_abl<768, 13, 1, 1, 64, ABL>(x, B, H, W, wp, bias, lnw, lnb, y, s); \
  if (variant == ID && C == 96) return launch_dw_abl<96, 7, 2, 1, 8, ABL>(x, B, H, W, wp, bias, lnw, lnb, y, s);
  PA(60, 0) PA(61, 1) PA(62, 2) PA(63, 4) PA(64, 8) PA(65, 16) PA(66, 32) PA(67, 33) PA(68, 6) PA(69, 22)
  PA(70, 41) PA(71, 9) PA(72, 54) PA(73, 20)
#undef PA
#undef V
#undef R
  return 1;
}
