// Tuning lab for the fused narrow-stage CNBlock MLP (not part of the product library): the
// product kernel (count_pipnet_amd/csrc/mlp_f32.hip) with other (HC, waves, pixel groups)
// instantiations selected by mlp_lab_set().  Built by tools/mlp_lab.py.
#define PIPNET_MLP_LAB
#include "../count_pipnet_amd/csrc/mlp_f32.hip"

static int g_variant = 0;
extern "C" void mlp_lab_set(int v) { g_variant = v; }

bool pipnet_mlp_lab_variant(int C, const float* t, const float* W1, const float* b1, const float* W2, const float* b2,
                            const float* gamma, float* x, int M, hipStream_t s) {
#define V(ID, CC, HC, NW, PX) V2(ID, CC, HC, NW, PX, 1)
#define V2(ID, CC, HC, NW, PX, HS) \
  case ID: if (C != CC) return false; launch_mlp<CC, HC, NW, PX, HS>(t, W1, b1, W2, b2, gamma, x, M, s); return true;
  switch (g_variant) {
    V(1, 96, 32, 8, 2) V(2, 96, 32, 4, 2) V(4, 96, 32, 4, 1) V(5, 96, 16, 4, 2)
    V(11, 192, 32, 8, 1) V(12, 192, 32, 4, 1) V(13, 192, 16, 8, 1) V(14, 192, 16, 2, 1) V(15, 192, 16, 4, 1)
    V(7, 96, 32, 2, 1)
    // hidden split over 2 waves per pixel group (HS = 2)
    V2(21, 192, 16, 8, 1, 2) V2(24, 192, 16, 4, 1, 2) V2(25, 192, 16, 2, 1, 2)
    V2(31, 96, 32, 8, 1, 2) V2(32, 96, 16, 8, 1, 2) V2(33, 96, 32, 4, 1, 2)
    // ablations (ABL bits of cnblock_mlp_kernel): 1000 * shape + bits; shapes 1 = C2 stage 1 (96, 32, 4, 1),
    // 2 = C2 stage 2 (192, 16, 8, 1), 3 = C5 stage 1 (96, 32, 8, 1), 4 = C5 stage 2 (192, 16, 8, 1, HS 2)
#define A(B) \
  case 1000 + B: if (C != 96) return false; launch_mlp<96, 32, 4, 1, 1, B>(t, W1, b1, W2, b2, gamma, x, M, s); return true; \
  case 2000 + B: if (C != 192) return false; launch_mlp<192, 16, 8, 1, 1, B>(t, W1, b1, W2, b2, gamma, x, M, s); return true; \
  case 3000 + B: if (C != 96) return false; launch_mlp<96, 32, 8, 1, 1, B>(t, W1, b1, W2, b2, gamma, x, M, s); return true; \
  case 4000 + B: if (C != 192) return false; launch_mlp<192, 16, 8, 1, 2, B>(t, W1, b1, W2, b2, gamma, x, M, s); return true;
    A(0) A(1) A(2) A(4) A(8) A(16) A(3) A(12) A(18) A(32)
#undef A
    default: return false;
  }
#undef V
#undef V2
}
