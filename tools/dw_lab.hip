// Tuning lab for the depthwise 7x7 + LayerNorm kernel (not part of the product ABI).
#include "../count_pipnet_amd/csrc/convnext_dw.hpp"
using namespace pipnet_dw;

extern "C" int lab_dw(int variant, const float* x, int B, int H, int W, int C, const float* wp, const float* bias,
                      const float* lnw, const float* lnb, float* y, void* stream) {
  hipStream_t s = (hipStream_t)stream;
#define V(ID, CC, TX, TY, MB, LPP) \
  if (variant == ID && C == CC) return launch_dw<CC, TX, TY, MB, false, LPP>(x, B, H, W, wp, bias, lnw, lnb, y, s);
  // v0 = the product's choice (LPP 64); v1-v4: lanes per LayerNorm pixel 32 / 16, TY 1 / 2
  V(0, 96, 7, 1, 1, 64) V(1, 96, 7, 1, 1, 32) V(2, 96, 7, 1, 1, 16) V(3, 96, 7, 2, 1, 16) V(4, 96, 14, 1, 1, 16)
  V(0, 192, 7, 1, 1, 64) V(1, 192, 7, 1, 1, 32) V(2, 192, 7, 1, 1, 16) V(3, 192, 7, 2, 1, 16) V(4, 192, 14, 1, 1, 16)
  V(0, 384, 7, 1, 2, 64) V(1, 384, 7, 1, 2, 32) V(2, 384, 7, 1, 2, 16) V(3, 384, 14, 1, 1, 16) V(4, 384, 7, 2, 2, 16)
  V(0, 768, 13, 1, 1, 64) V(1, 768, 13, 1, 1, 32) V(2, 768, 13, 1, 1, 16) V(3, 768, 7, 1, 2, 16) V(4, 768, 7, 1, 2, 32)
#undef V
  return 1;
}
