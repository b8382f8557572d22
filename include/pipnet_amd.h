/*
 * pipnet_amd.h -- C-ABI of the MI355X-native PIP-Net / CountPIPNet inference path.
 *
 * The reference (TarasKutsyk/Count_PIPNet) has no native code and no FFI: its boundary is
 * the Python nn.Module contract of pipnet/pipnet.py and pipnet/count_pipnet.py
 * (SURVEY.md 8b).  These entry points are what a ctypes / torch-extension binding of that
 * forward binds: every op of the hot path's ATen sequence as one
 * stream-ordered call.  Plain pointers and sizes only (no torch types).
 *
 * Conventions
 *   - all tensors are float32 device pointers (HBM), activations NHWC ("channels_last"),
 *     the network input NCHW exactly as the reference receives it;
 *   - ``stream`` is a hipStream_t (NULL = default stream); calls only enqueue work;
 *   - the return value is a PIPNET_* status; the Python host layer raises RuntimeError
 *     on anything but PIPNET_OK (the reference raises Python exceptions).
 *   - re-entrant: no global mutable state; callers own every buffer.
 */
#ifndef PIPNET_AMD_H
#define PIPNET_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PIPNET_OK 0
#define PIPNET_ERR_ARG 1        /* bad shape / size / unsupported configuration */
#define PIPNET_ERR_ALIGN 2      /* pointer or leading dimension not 16-byte aligned */
#define PIPNET_ERR_LAUNCH 3     /* hipLaunchKernel failed (hipGetLastError) */
#define PIPNET_ERR_HIP 4        /* other HIP runtime error */

/* GEMM epilogues for pipnet_linear_f32 */
#define PIPNET_EPI_NONE 0       /* C = A W^T                                              */
#define PIPNET_EPI_BIAS 1       /* C = A W^T + b                                          */
#define PIPNET_EPI_BIAS_GELU 2  /* C = gelu_erf(A W^T + b)          (CNBlock Linear1+GELU) */
#define PIPNET_EPI_RESID 3      /* C = R + s * (A W^T + b)   (CNBlock Linear2*layer_scale+x)*/
#define PIPNET_EPI_MUL 4        /* C = (A W^T) * R          (BilinearIntermediate W(e)*V(e)) */
#define PIPNET_EPI_BIAS_RELU 5  /* C = relu(A W^T + b)            (ResNet conv+BN+ReLU)      */
#define PIPNET_EPI_BIAS_RESID_RELU 6 /* C = relu(A W^T + b + R) (Bottleneck conv3+BN+identity+ReLU) */
#define PIPNET_EPI_RESID_ROWSCALE 7  /* C = R + rs[m/g] * (s * (A W^T + b))  (pipnet_linear_rowscale_f32:
                                        CNBlock Linear2 with train-mode stochastic depth)              */
#define PIPNET_EPI_GELU_BWD 8        /* C = (A W^T) * gelu_erf'(R)   (training: d pre-GELU activation) */
/* split-bf16 ("bf16x3") epilogues of pipnet_conv2d_nhwc_s3 (fp32 results, see there) */
#define PIPNET_EPI_S3_GELU 9         /* g = gelu_erf(A W^T + b) stored as split planes [hi|lo] bf16    */
#define PIPNET_EPI_F32_BIAS 10       /* C = A W^T + b, fp32                                            */
#define PIPNET_EPI_F32_RESID 11      /* C = R + s * (A W^T + b), fp32 C and R (R may alias C)          */
#define PIPNET_EPI_DUAL_BIAS_RELU 12 /* columns < N1: C = A W^T + b; columns >= N1: C2 = relu(A W^T + b) (bf16 1x1 convs, pipnet_conv1x1_bf16_dual) */

/* ABI version: bumped whenever an exported signature changes.  2: pipnet_wgrad_conv_f32 gained
 * its `pad` argument (round 2).  3: the process-wide A/B switches (pipnet_gemm_persist /
 * _stream / _bk16x3 / _plain_store, pipnet_conv_bf16_rb, pipnet_head_bf16_quads) and
 * pipnet_linear_agelu_f32 are gone -- kernel selection is a fixed per-shape rule with no
 * mutable library state -- and the one-launch fused head pipnet_softmax_pool_linear_f32 / _bf16
 * (+ _part_floats) and pipnet_matmul2_f64acc_f32 are new (round 5).  A caller built against an older version must not bind this library.
 * Round 6 only ADDS entry points (pipnet_philox_exp1_f32, pipnet_conv2d_nhwc_bf16_plan,
 * pipnet_linear_f32_plan, pipnet_cnblock_mlp_plan); no signature changed. */
#define PIPNET_AMD_ABI_VERSION 3
int pipnet_amd_abi_version(void);
const char* pipnet_amd_status_string(int status);
/* sha256 (hex) of the sources this library was compiled from (build provenance). */
const char* pipnet_amd_source_digest(void);

/* Dense fp32 linear / 1x1 conv on MFMA (v_mfma_f32_32x32x2_f32, exact fp32):
 *   C[M,N] (ldc) = epi( A[M,K] (lda) * W[N,K]^T )
 * Replaces F.linear / nn.Linear (torchvision CNBlock block.3 / block.5),
 * the 1x1 add-on Conv2d (pipnet.py:99-104, count_pipnet.py:376-381) and the
 * Bilinear/LinearFull intermediate Linears (count_pipnet_utils.py:342-385, :387-444).
 * K % 4 == 0, lda/ldc/ldr % 4 == 0, pointers 16-B aligned.  bias/scale: [N] or NULL;
 * R (resid / other): [M,N] with leading dimension ldr (may alias C for in-place residual). */
int pipnet_linear_f32(const float* A, int64_t lda, const float* W, const float* bias,
                      const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                      int M, int N, int K, int epilogue, void* stream);

/* pipnet_linear_f32 with PIPNET_EPI_RESID_ROWSCALE: C = R + row_scale[m / rows_per_scale] *
 * (scale * (A W^T + bias)).  The CNBlock's Linear2 * layer_scale + residual under
 * torchvision's StochasticDepth("row") in train mode: rows_per_scale = H*W (one factor per
 * sample), row_scale[b] = keep_b / (1 - p) -- 0 leaves a dropped sample's rows equal to R. */
int pipnet_linear_rowscale_f32(const float* A, int64_t lda, const float* W, const float* bias, const float* scale,
                               const float* R, int64_t ldr, float* C, int64_t ldc, int M, int N, int K,
                               const float* row_scale, int rows_per_scale, void* stream);

/* Split-K variant for short-M products (M <= a few hundred rows, long K: the Bilinear /
 * LinearFull intermediate GEMMs at M = batch, count_pipnet_utils.py:342-385): the K range
 * is cut into `splits` slabs computed by separate workgroups into `workspace`
 * (splits * M * N floats), then one reduction kernel sums the slabs and applies the
 * epilogue.  N % 4 == 0, K % 32 == 0, splits <= K/32. */
int pipnet_linear_splitk_f32(const float* A, int64_t lda, const float* W, const float* bias,
                             const float* scale, const float* R, int64_t ldr, float* C, int64_t ldc,
                             int M, int N, int K, int epilogue, int splits, float* workspace,
                             void* stream);
/* BilinearIntermediate on the folded pair in one GEMM: Wpair = [W1; W2] ([2 Nh, K], the
 * pipnet_matmul2_f64acc_f32 output), C[M, Nh] = (A W2^T) * (A W1^T) elementwise, K split into
 * `splits` slabs (workspace: splits * M * 2 Nh floats) summed in slab order by the reduction that
 * also takes the product -- count_pipnet_utils.py:378-385 W(e) * V(e) with e folded in. */
int pipnet_linear_pair_mul_f32(const float* A, int64_t lda, const float* Wpair, float* C, int64_t ldc, int M, int Nh,
                               int K, int splits, float* workspace, void* stream);

/* ConvNeXt downsample conv, k=2, stride s in {1,2}, no padding, as implicit GEMM on MFMA.
 * x: [B,H,W,Cin] NHWC (already LayerNorm2d-normalised), w_packed: [Cout][2][2][Cin]
 * (torch weight [Cout,Cin,2,2] permuted), y: [B,OH,OW,Cout], OH=(H-2)/s+1.
 * Replaces features.{2,4,6}.1 of torchvision ConvNeXt with the stride patch of
 * features/convnext_features.py:5-15.  Cin % 32 == 0. */
int pipnet_conv2x2_f32(const float* x, int B, int H, int W, int Cin, const float* w_packed,
                       const float* bias, int Cout, int stride, float* y, void* stream);

/* General NHWC convolution as implicit GEMM on MFMA (ResNet backbones, eval BatchNorm
 * folded into w/bias by the caller):  y = epi(conv(x, w) + bias), epilogue one of
 * PIPNET_EPI_NONE / _BIAS / _BIAS_RELU / _BIAS_RESID_RELU (R: [B,OH,OW,Cout]).
 * x: [B,H,W,Cin] NHWC, w_packed: [Cout][KH][KW][Cin], y: [B,OH,OW,Cout] with
 * OH = (H + 2 pad - KH)/stride + 1.  Replaces the Conv2d+BatchNorm2d(+ReLU)(+identity)
 * sequences of features/resnet_features.py:77-124,126-229.  Cin % 4 == 0. */
int pipnet_conv2d_nhwc_f32(const float* x, int B, int H, int W, int Cin, const float* w_packed,
                           const float* bias, int Cout, int KH, int KW, int stride, int pad,
                           const float* R, int epilogue, float* y, void* stream);

/* MaxPool2d(k, stride, pad) on NHWC (ResNet stem, resnet_features.py:136). */
int pipnet_maxpool2d_nhwc_f32(const float* x, int B, int H, int W, int C, int k, int stride, int pad,
                              float* y, void* stream);

/* NCHW -> NHWC with the channel dimension zero-padded to Cpad (network input of the ResNet
 * stem, so every implicit-GEMM tap is a 16-byte vector). */
int pipnet_nchw_to_nhwc_f32(const float* x, int B, int C, int H, int W, int Cpad, float* y, void* stream);

/* ---- bf16 ResNet path (BASELINE C3 "ResNet50 ... bf16 inference") -------------------
 * Activations are bf16 NHWC (passed as void*: raw 16-bit bfloat16 storage), accumulation
 * fp32 on v_mfma_f32_32x32x16_bf16, folded-BN bias fp32, outputs rounded to nearest even.
 * Same epilogues and semantics as pipnet_conv2d_nhwc_f32; w_packed: [Cout][Kp] bf16 with
 * Kp = KH*KW*Cin rounded up to a multiple of 64 (taps [KH][KW][Cin], zero beyond).
 * Cin % 8 == 0, Cout % 8 == 0, x / w / y / R 16-byte aligned. */
int pipnet_conv2d_nhwc_bf16(const void* x, int B, int H, int W, int Cin, const void* w_packed,
                            const float* bias, int Cout, int KH, int KW, int stride, int pad,
                            const void* R, int epilogue, void* y, void* stream);

/* Same, with the workgroup tile forced (tuning / tests): tile 0 = 64x128 (32-deep K tiles,
 * 4 LDS stages), 1 = 128x128 and 2 = 256x256 (64-deep, 2 stages), 3 = 256x256 and
 * 4 = 128x128 (32-deep, 4 stages), 5 = 256x256 ping-pong on 16x16x32 MFMAs (Cin % 32 == 0
 * unless 1x1 stride 1), 6 = 256x64 (32-deep, 4 stages), -1 = automatic (what
 * pipnet_conv2d_nhwc_bf16 uses: tile 5 for every N >= 256 layer it can serve, tile 6 for
 * N <= 64, whatever M; the MFMA shape and K order never depend on the batch size, so
 * neither do the results). */
int pipnet_conv2d_nhwc_bf16_tile(const void* x, int B, int H, int W, int Cin, const void* w_packed,
                                 const float* bias, int Cout, int KH, int KW, int stride, int pad,
                                 const void* R, int epilogue, void* y, int tile, void* stream);

/* ---- CountPIPNet finetune phase (pipnet/train.py:75-140, main.py:333-343: classifier +
 * intermediate layer train) ------------------------------------------------------------
 * Train-mode (soft) Gumbel head, F.gumbel_softmax(hard=False) (count_pipnet_utils.py:34-35):
 * proto = softmax((x - log E) / tau) [B,HW,P] NHWC, sums [B,P] = spatial sums = the raw
 * counts (count_pipnet.py:88).  exp_noise / seed / offset as pipnet_count_gumbel_f32. */
int pipnet_count_gumbel_soft_f32(const float* logits, int B, int HW, int P, float tau, const float* exp_noise,
                                 uint64_t seed, uint64_t offset, float* proto, float* sums, void* stream);

/* dx = d_out relu(W)  (NonNegLinear input gradient; d_out [N,K], W [K,D], dx [N,D]). */
int pipnet_nonneg_linear_dx_f32(const float* d_out, const float* W, int N, int D, int K, float* dx, void* stream);

/* BilinearIntermediate backward front: du = g * v, dv = g * u (n elements). */
int pipnet_bilinear_bwd_prep_f32(const float* g, const float* u, const float* v, int64_t n, float* du, float* dv,
                                 void* stream);

/* LinearIntermediate backward (count_pipnet_utils.py:471-519, Linear(1, E, bias=False) over
 * the counts x [n = B*P]): g [n][E] -> dx [n] = g w (dx may be NULL) and dw [E] = g^T x
 * (accumulate adds); partial: pipnet_linear_inter_partials_floats(E) floats; E <= 16. */
int pipnet_linear_inter_partials_floats(int E);
int pipnet_linear_inter_bwd_f32(const float* x, int64_t n, int E, const float* g, const float* w, float* dx,
                                float* dw, int accumulate, float* partial, void* stream);

/* ---- split-bf16 ("bf16x3") fp32 path of the ConvNeXt backbone -------------------------
 * An fp32 operand x is carried as two bf16 values, hi = RNE(x) and lo = RNE(x - hi)
 * (x = hi + lo to ~2^-17 relative).  A product x.w is then hi.hi + lo.hi + hi.lo (the
 * lo.lo term, ~2^-16 relative, is dropped), accumulated in fp32 -- a bf16 GEMM over K' = 3K
 * whose A rows are read as [hi(x) | lo(x) | hi(x)] and whose weight rows are
 * [hi(w) | hi(w) | lo(w)] per tap.  Activations are stored as "split planes" [hi | lo]
 * (2 Cin bf16 per pixel = the fp32 bytes); the kernel reads the third K segment from the
 * hi plane again.  Per-product error ~1e-5 relative (fp32: 6e-8) at 3/16 of the fp32-MFMA
 * cost (v_mfma_f32_16x16x32_bf16 / 32x32x16_bf16 vs v_mfma_f32_32x32x2_f32).  Replaces the
 * same torchvision CNBlock Linears and downsample convs as pipnet_linear_f32 /
 * pipnet_conv2x2_f32.
 *   x: [B,H,W,2 Cin] split planes (Cin % 32 == 0), w_packed: [Cout][Kp] bf16 with taps
 *   [KH][KW][3 Cin] (Kp = KH*KW*3Cin rounded up to 32, zero beyond), bias / scale [Cout]
 *   fp32 or NULL.  epilogue PIPNET_EPI_S3_GELU: y = split planes [B,OH,OW,2 Cout] bf16 of
 *   gelu(conv + bias); PIPNET_EPI_F32_BIAS: y fp32 [B,OH,OW,Cout]; PIPNET_EPI_F32_RESID:
 *   y = R + scale * (conv + bias), fp32, R [B,OH,OW,Cout] (may equal y).  tile as
 *   pipnet_conv2d_nhwc_bf16_tile (only -1, 0, 4, 5). */
int pipnet_conv2d_nhwc_s3(const void* x, int B, int H, int W, int Cin, const void* w_packed,
                          const float* bias, const float* scale, const float* R, int Cout, int KH, int KW,
                          int stride, int pad, int epilogue, void* y, int tile, void* stream);

/* pipnet_dwconv7_ln_f32 writing its output as split planes [B,H,W,2C] bf16 [hi | lo] (the A
 * operand of the split-bf16 Linear1). */
int pipnet_dwconv7_ln_s3(const float* x, int B, int H, int W, int C, const float* w_packed,
                         const float* bias, const float* ln_w, const float* ln_b, void* y, void* stream);

/* pipnet_layernorm_f32 writing split planes [rows, 2C] bf16 (input of a split-bf16 downsample conv). */
int pipnet_layernorm_s3(const float* x, int64_t rows, int C, const float* w, const float* b, void* y,
                        void* stream);

/* MaxPool2d(k, stride, pad) on NHWC bf16 (C % 8 == 0). */
int pipnet_maxpool2d_nhwc_bf16(const void* x, int B, int H, int W, int C, int k, int stride, int pad,
                               void* y, void* stream);

/* fp32 NCHW -> bf16 NHWC (round to nearest even), channels zero-padded to Cpad (% 8 == 0). */
int pipnet_nchw_to_nhwc_bf16(const float* x, int B, int C, int H, int W, int Cpad, void* y, void* stream);

/* Two 1x1 stride-1 bf16 convs over the same input in one launch (a ResNet stage's first
 * Bottleneck: the downsample conv + BN and conv1 + BN + ReLU, resnet_features.py:95-117):
 * w_packed = [N1 + N2, Kp] (rows 0..N1-1 the first conv), bias [N1 + N2];
 *   y1[M,N1] = x W1^T + b1,   y2[M,N2] = relu(x W2^T + b2).
 * x: [M, Cin] bf16 (NHWC pixels), N1 % 256 == 0, N2 % 256 == 0.  Each output equals the
 * single-conv launch bit for bit (same tile, same K order); the input is read once. */
int pipnet_conv1x1_bf16_dual(const void* x, int64_t M, int Cin, const void* w_packed, const float* bias, int N1,
                             void* y1, int N2, void* y2, void* stream);

/* ResNet stem input for a 3-channel k7 s2 p3 conv run as a 4x4 stride-1 conv: fp32 NCHW [B,3,H,W]
 * -> bf16 2x2 space-to-depth image [B, SH, SW, 16], SH = (H-1)/2 + 4, SW = (W-1)/2 + 4,
 * y[b][i][j][(2 bi + bj) * 4 + c] = x[b][c][2(i-2)+bi][2(j-2)+bj] (zero outside the image and for
 * c = 3).  The matching weights are W'[o][a][a'][(2 bi + bj) * 4 + c] = w[o][c][2a+bi-1][2a'+bj-1]. */
int pipnet_nchw_to_s2d_bf16(const float* x, int B, int H, int W, void* y, void* stream);
/* ResNet stem (4x4 stride-1 conv over the s2d image, 16 -> 64 channels, + bias + ReLU) fused
 * with MaxPool2d(3, 2, 1) -- replaces the conv1 / bn1 / relu / maxpool sequence of
 * resnet_features.py:161-164 in the bf16 build.  s2d: [B][SH][SW][16] bf16 from
 * pipnet_nchw_to_s2d_bf16; w: packed [64][256] bf16 (the regrouped 4x4x16 stem weight, BN
 * folded); bias: [64] fp32; y: [B][PH][PW][64] bf16, PH = (SH - 4) / 2 + 1.  SW - 3 <= 112.
 * Bitwise equal to pipnet_conv2d_nhwc_bf16 (4x4, EPI_BIAS_RELU) + pipnet_maxpool2d_nhwc_bf16. */
int pipnet_stem_pool_bf16(const void* s2d, int B, int SH, int SW, const void* w, const float* bias, void* y,
                          void* stream);

/* pipnet_softmax_pool_f32 reading bf16 logits (fp32 softmax, fp32 proto / pooled out). */
int pipnet_softmax_pool_bf16(const void* feat, int B, int HW, int P, int pool_mode, float* proto,
                             float* pooled, void* stream);

/* The whole PIP-Net head in ONE kernel launch (pipnet.py:33-37; replaces pipnet_softmax_pool_f32
 * (pool_mode 0) + pipnet_nonneg_linear_f32): per-pixel softmax over P channels, proto written
 * once, spatial max into pooled [B,P], then -- in the last workgroup to finish image b (an
 * arrival ticket) -- x' = where(pooled < thresh, 0, pooled) when apply_thresh, else pooled,
 * written to x_out [B,P] (may be NULL), and out [B,K] = x' relu(W)^T + bias, W [K,P] read at
 * call time.  Bitwise equal to the two-kernel path.  W 16-B aligned when P % 4 == 0.  _bf16:
 * bf16 logits.
 * part: pipnet_softmax_pool_linear_part_floats(B, HW, P) (= B * P) floats of scratch for the
 * running maxima, tickets: int32 [B] arrival counters -- BOTH must be ZERO on entry: zero them once
 * at allocation; every completed call leaves part[0 .. B*P) and tickets[0 .. B) zero again, so no
 * memset is needed between calls.  Calls that may run concurrently (different streams) need
 * separate part / tickets buffers. */
int64_t pipnet_softmax_pool_linear_part_floats(int B, int HW, int P);
int pipnet_softmax_pool_linear_f32(const float* feat, int B, int HW, int P, float* proto, float* pooled,
                                   const float* W, const float* bias, int K, int apply_thresh, float thresh,
                                   float* x_out, float* out, float* part, int32_t* tickets, void* stream);
int pipnet_softmax_pool_linear_bf16(const void* feat, int B, int HW, int P, float* proto, float* pooled,
                                    const float* W, const float* bias, int K, int apply_thresh, float thresh,
                                    float* x_out, float* out, float* part, int32_t* tickets, void* stream);

/* ---- eval_pipnet metric loop (pipnet/test.py:67-131,266-319) -------
 * One evaluation batch, entirely on the device (no host sync):
 *   pooled [B,P] (clamped presence / counts), out [B,K] logits, W [K,P] the prototype->class
 *   weights the reference multiplies with (PIP-Net: the sparsified classification weight;
 *   CountPIPNet: get_prototype_importance_per_class stacked), ys [B] int64 labels,
 *   multiplier -> normalization_multiplier (device scalar, may be NULL = 1), thr = 1e-3.
 * Writes ys_pred [B] (torch.max index) and score [B] (amax softmax(log1p(out^m))); adds into
 * cm [K,K] int64 (cm[y][pred]), acc[5] fp64 running sums of the per-batch means
 * {true-class local size, all-class local size, prototypes per class, almost-nonzeros,
 * top-1}, *abstained (images whose max logit is 0).  workspace: int32 [5B + K]. */
int pipnet_eval_batch_f32(const float* pooled, const float* out, const float* W, int B, int P, int K,
                          const int64_t* ys, const float* multiplier, float thr, int32_t* ys_pred,
                          float* score, int64_t* cm, double* acc, int64_t* abstained, int32_t* workspace,
                          void* stream);

/* In-place classifier sparsification of eval_pipnet (test.py:71-73): w = max(w - delta, 0). */
int pipnet_weight_sparsify_f32(float* w, int64_t n, float delta, void* stream);

/* ConvNeXt stem: Conv2d(3,96,k4,s4,bias) + LayerNorm2d(96, eps 1e-6)  (features.0).
 * x: [B,3,H,W] NCHW (the reference's own input layout), w: [96,3,4,4] as torch stores it,
 * y: [B,H/4,W/4,96] NHWC.  H, W multiples of 4; x, w, b, ln_w, ln_b, y 16-byte aligned. */
int pipnet_convnext_stem_f32(const float* x, int B, int H, int W, const float* w, const float* b,
                             const float* ln_w, const float* ln_b, float* y, void* stream);

/* CNBlock front half: depthwise Conv2d 7x7 pad 3 (+bias) + LayerNorm(C, eps 1e-6).
 * x, y: [B,H,W,C] NHWC, w_packed: [49][C] (torch [C,1,7,7] transposed).
 * C in {96,192,384,768}. */
int pipnet_dwconv7_ln_f32(const float* x, int B, int H, int W, int C, const float* w_packed,
                          const float* bias, const float* ln_w, const float* ln_b, float* y,
                          void* stream);

/* Row LayerNorm over the last dim (LayerNorm2d on NHWC), eps 1e-6: y = LN(x) * w + b. */
int pipnet_layernorm_f32(const float* x, int64_t rows, int C, const float* w, const float* b,
                         float* y, void* stream);

/* PIP-Net head, part 1 (pipnet.py:33-34): per-pixel softmax over P prototype channels
 * (nn.Softmax(dim=1)), proto written once (NHWC), fused spatial pooling:
 *   pool_mode 0 -> pooled[b,p] = max over pixels (AdaptiveMaxPool2d(1)+Flatten)
 *   pool_mode 1 -> pooled[b,p] = sum over pixels (CountPIPNet softmax activation, :88)
 * feat, proto: [B,HW,P]; pooled: [B,P] (zeroed by this call before accumulation). */
int pipnet_softmax_pool_f32(const float* feat, int B, int HW, int P, int pool_mode, float* proto,
                            float* pooled, void* stream);

/* Fused CNBlock MLP of the narrow ConvNeXt stages (torchvision CNBlock block.3-5 + layer_scale +
 * residual; the Linear / GELU / Linear of features.1 and features.3):
 *   x[M,C] += gamma * (W2 gelu_erf(W1 t + b1) + b2)        in place on x
 * t: [M,C] (dwconv7 + LayerNorm output), W1: [4C,C], b1: [4C], W2: [C,4C], b2 / gamma: [C];
 * C = 96 or 192; exact fp32 (v_mfma_f32_16x16x4_f32), the 4C-wide hidden activation never
 * leaves the registers.  All pointers 16-B aligned. */
int pipnet_cnblock_mlp_f32(const float* t, const float* W1, const float* b1, const float* W2, const float* b2,
                           const float* gamma, float* x, int64_t M, int C, void* stream);
/* Same, told the layer's feature-map size hw = H*W per image (0 = unknown, as above): C = 192 on
 * maps of <= 256 pixels splits the hidden dimension over two waves per 16-pixel group (another
 * fixed summation order, chosen by hw only, so a pixel's result never depends on M). */
int pipnet_cnblock_mlp_hw_f32(const float* t, const float* W1, const float* b1, const float* W2, const float* b2,
                              const float* gamma, float* x, int64_t M, int C, int hw, void* stream);

/* NonNegLinear (pipnet.py:54-71, count_pipnet.py:176-224): out = x' relu(W)^T + b with
 * x' = where(x < thresh, 0, x) when apply_thresh (pipnet.py:36, inference) else x.
 * x: [B,D], W: [K,D] read at call time (callers mutate it in place, test.py:73),
 * bias [K] or NULL, x_out: [B,D] receives x' (may be NULL), out: [B,K]. */
int pipnet_nonneg_linear_f32(const float* x, int B, int D, const float* W, const float* bias,
                             int K, int apply_thresh, float thresh, float* x_out, float* out,
                             void* stream);

/* CountPIPNet Gumbel-softmax (eval, hard=True) + spatial count (count_pipnet_utils.py:36-38,
 * count_pipnet.py:88): per pixel z = (x - log E)/tau, one-hot at argmax written as the
 * straight-through value (1 - y) + y, all other channels exactly 0, and hist[b,p] += 1.
 * E ~ Exp(1) is read from exp_noise ([B,P,HW], the NCHW layout of torch's draw) when
 * non-NULL, else generated in-kernel by Philox4x32-10 keyed by (seed, offset + element/4):
 * one 128-bit block feeds channels 4k..4k+3 of a pixel.
 * logits, proto: [B,HW,P], 16-byte aligned, P % 4 == 0; hist: [B,P] int32 (zeroed by this call). */
int pipnet_count_gumbel_f32(const float* logits, int B, int HW, int P, float tau,
                            const float* exp_noise, uint64_t seed, uint64_t offset, float* proto,
                            int32_t* hist, void* stream);

/* Same, graph-replayable: the Philox key is device memory.  seed_state: uint64[2] on the
 * device ([0] a splitmix64 counter, [1] the key); each call first advances the counter and
 * derives a new key on the stream (fresh noise per call, as the reference draws fresh
 * noise), so a captured hipGraph replays with new noise every time. */
int pipnet_count_gumbel_devseed_f32(const float* logits, int B, int HW, int P, float tau,
                                    uint64_t* seed_state, float* proto, int32_t* hist, void* stream);

/* The Gumbel heads' Exp(1) noise on its own (parity tests; oracle/philox_ref.py restates it):
 * out[i] for i < n (n % 4 == 0) = the draw count_gumbel_kernel uses for element i of its NHWC
 * [B,HW,P] stream under (seed, offset): word i % 4 of Philox4x32-10 block offset + i/4, E = -log u
 * with u = (top 24 bits + 1/2) 2^-24 floored at E >= 2^-25.  log_e = 0: E (the soft head's libm
 * form); log_e = 1: log E on the hard head's hardware-log form.  Replaces the
 * `-torch.empty_like(x).exponential_().log()` draw inside F.gumbel_softmax (count_pipnet_utils.py:36-38). */
int pipnet_philox_exp1_f32(uint64_t seed, uint64_t offset, int64_t n, int log_e, float* out, void* stream);

/* fp32 GEMM variant plan: the variant pipnet_linear_f32 (and the conv / rowscale forms) launch for an
 * M x N x K product with dense 16-B aligned operands, PIPNET_EPI_* epilogue and A-operand gather
 * (0 dense / linear, 1 the 2x2 patch conv, 2 the general NHWC conv) -- 0 K-tail kernel, 1 BK16
 * 128-row, 2 BK32 64-row, 3 BK32 128-row, 5 BK32 192 x 384 on 12 waves -- or -PIPNET_ERR_ARG
 * (profiling labels). */
int pipnet_linear_f32_plan(int M, int N, int K, int epilogue, int aload);

/* fused CNBlock MLP plan: the instantiation pipnet_cnblock_mlp_hw_f32 launches for M pixels of C
 * channels on maps of hw pixels per image (0 = unknown), as HC * 100 + NW * 10 + HS
 * (cnblock_mlp_kernel<C, HC, NW, 1, HS>), or -PIPNET_ERR_ARG (profiling labels). */
int pipnet_cnblock_mlp_plan(int64_t M, int C, int hw);

/* bf16 conv tile plan: the tile id pipnet_conv2d_nhwc_bf16_tile takes for this shape / epilogue
 * (tile -1 = the automatic choice, >= 0 validated), or -PIPNET_ERR_ARG.  The library's own rule,
 * exported so that profiling labels never mirror it (kernels.bf16_conv_kernel_name). */
int pipnet_conv2d_nhwc_bf16_plan(int B, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad,
                                 int epilogue, int tile);

/* Count finish (count_pipnet.py:88-97): counts_raw = float(hist) (or sums when hist is
 * NULL), clamped = clamp(round?(counts), 0, max_count) -- round when do_round.
 * sums: [B,P] float (softmax activation path) used when hist == NULL. */
int pipnet_count_finish_f32(const int32_t* hist, const float* sums, int B, int P, int max_count,
                            int do_round, float* counts_raw, float* clamped, void* stream);

/* Elementwise count encodings into [B, P*C] (p-major):
 *   kind 0 (OneHotEncoder, count_pipnet_utils.py:141-185): one-hot at clamp(int(x)-1,0,C-1)
 *          where x > 0.1, x rounded first when do_round (ModifiedSTEFunction :201-217);
 *   kind 1 (LinearIntermediate, :471-539): out[b,p*C+c] = x[b,p] * w[c]. */
int pipnet_count_encode_f32(const float* x, int B, int P, int C, int kind, int do_round,
                            const float* w, float* out, void* stream);

/* ---- evaluation input transform ----------------------------------
 * transform_no_augment of util/data.py (:264-269, :314-321, :500-505, :537-542, :568-574):
 * Resize((out_h, out_w)) [+ Grayscale(3)] + ToTensor + Normalize(mean, std), applied to a
 * ragged batch of decoded RGB images (ImageFolder's pil_loader: Image.open().convert('RGB')).
 * Resize restates Pillow's ImagingResample(BILINEAR) integer arithmetic exactly (torchvision
 * forwards a PIL image's Resize to it), so the uint8 resized image is bit-identical to
 * Pillow's and the fp32 output to ToTensor/Normalize of it.
 *
 * pipnet_resize_plan (host only): sizes_host [B][2] = (h, w) per image -> kmax (taps per
 *   output coordinate) and the device workspace size in bytes.
 * pipnet_resize_normalize_rgb8: pixels = the B images packed HWC uint8 (image b at byte
 *   offsets[b], device), sizes [B][2] int32 (device), mean3/std3 host float[3], workspace
 *   (device, from pipnet_resize_plan), out [B,3,out_h,out_w] fp32 NCHW, out_u8 optional
 *   [B,out_h,out_w,3] uint8 copy of the resized (and grayscaled) image, NULL to skip. */
int pipnet_resize_plan(const int32_t* sizes_host, int B, int out_h, int out_w, int* kmax,
                       int64_t* workspace_bytes);
int pipnet_resize_normalize_rgb8(const uint8_t* pixels, const int64_t* offsets, const int32_t* sizes,
                                 int B, int out_h, int out_w, int kmax, int grayscale,
                                 const float* mean3, const float* std3, int32_t* workspace,
                                 float* out, uint8_t* out_u8, void* stream);

/* ---- training step, finetune phase (pipnet/train.py:75-140) ----
 * The batch is cat([xs1, xs2]) (train.py:84): N = 2*Bh rows, proto features NHWC
 * [N][HW][P] (rows n and Bh*HW + n are the two views of one pixel), pooled [N][P],
 * out [N][K], ys int64 [Bh] (row r's label is ys[r % Bh], train.py:155).
 *
 * pipnet_train_align_partial_f32: align_loss (train.py:259-265) partial sums, one double
 *   per workgroup into partial[pipnet_train_align_partials()].  P % 4 == 0 needs pf
 *   16-byte aligned.
 * pipnet_train_loss_f32 (train.py:154-250): stats[8] = {align, tanh, class, total loss,
 *   correct count, w_align, w_tanh, w_class}; mode 0 train, 1 pretrain (no class term, no
 *   d_out), 2 finetune (loss = w_class * class).  mult = normalization_multiplier (device
 *   float[1]); enforce = enforce_weight_sparsity (class input log1p(out^mult)).
 *   d_out [N][K] = d loss / d out (w_class * d class).
 * pipnet_nonneg_linear_bwd_f32 (pipnet.py:54-71 backward): dW = (W > 0) * d_out^T x,
 *   db = sum_r d_out (db may be NULL).  x [N][D], W/dW [K][D].
 * pipnet_adamw_step_f32: torch.optim.AdamW on one tensor at optimizer step ``step`` (1-based),
 *   hyper-parameters in double as torch's param_groups hold them (the float constants the
 *   kernel uses -- 1 - lr*wd, 1 - beta1, 1 - beta2, lr/(1 - beta1^t), sqrt(1 - beta2^t) --
 *   are derived from them in double, as torch does), then if post != 0
 *   p = max(p - post_delta, post_floor) (train.py:134-140's clamps).
 * pipnet_clamp_min_f32: x = max(x, lo) (normalization_multiplier clamp, train.py:137). */
int pipnet_train_align_partials(void);
int pipnet_train_align_partial_f32(const float* pf, int Bh, int HW, int P, double* partial, void* stream);
int pipnet_train_loss_f32(const double* align_partial, int Bh, int HW, const float* pooled, const float* out,
                          const int64_t* ys, int P, int K, const float* mult, int enforce, float tanh_coeff,
                          float w_align, float w_tanh, float w_class, int mode, float* d_out, float* stats,
                          void* stream);
int pipnet_nonneg_linear_bwd_f32(const float* d_out, const float* x, int N, int D, const float* W, int K,
                                 float* dW, float* db, void* stream);
int pipnet_adamw_step_f32(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                          double lr, double beta1, double beta2, double eps, double weight_decay, int64_t step,
                          int post, float post_delta, float post_floor, void* stream);
int pipnet_clamp_min_f32(float* x, int64_t n, float lo, void* stream);

/* ---- backward building blocks (trainable ConvNeXt stages) ----
 * pipnet_wgrad_f32: C[N1][N2] (ldc) = (accumulate ? C : 0) + sum_m A[m][n1] B[m][n2]
 *   (A [M][N1] lda, B [M][N2] ldb, both pixel-major as the forward stores activations):
 *   the weight gradient dW = dY^T X of a Linear / 1x1 conv.  fp32 MFMA, deterministic
 *   (fixed pixel slabs, fixed-order reduction).  N1, N2, lda, ldb % 4 == 0, A/B 16-B
 *   aligned; workspace: pipnet_wgrad_workspace_bytes(M, N1, N2) bytes (needed unless the
 *   call runs as a single slab without accumulate; pass it whenever that size is > 0).
 * pipnet_colsum_f32: out[n] = (accumulate ? out[n] : 0) + sum_m A[m][n] (bias gradients);
 *   workspace of pipnet_colsum_workspace_bytes(N) bytes. */
int64_t pipnet_wgrad_workspace_bytes(int M, int N1, int N2);
int pipnet_wgrad_f32(const float* A, int64_t lda, const float* B, int64_t ldb, int M, int N1, int N2, float* C,
                     int64_t ldc, int accumulate, float* workspace, void* stream);
/* pipnet_wgrad_conv2x2_f32: weight gradient of the 2x2 downsample conv (stride 1 or 2):
 *   dW[co][(ky*2+kx)*Cin + ci] (+)= sum_{b,oy,ox} dY[b,oy,ox,co] x[b, oy*s+ky, ox*s+kx, ci]
 *   (the packed layout of pipnet_conv2x2_f32's weights); dY NHWC [B,OH,OW,Cout], x NHWC
 *   [B,H,W,Cin]; workspace: pipnet_wgrad_workspace_bytes(B*OH*OW, Cout, 4*Cin) bytes. */
int pipnet_wgrad_conv2x2_f32(const float* dY, const float* x, int B, int H, int W, int Cin, int stride, int Cout,
                             float* dW, int accumulate, float* workspace, void* stream);
/* pipnet_wgrad_conv_f32: weight gradient of a KHxKW conv, stride s, zero padding p (the
 * ConvNeXt stem, Conv2d(3, 96, 4, 4) with Cin zero-padded to 4; the ResNet 3x3 / strided 1x1
 * convs, features/resnet_features.py:17-28): dY NHWC [B][OH][OW][Cout], x NHWC [B][H][W][Cin]
 * -> dW [Cout][KH][KW][Cin] (accumulate adds); OH = (H + 2p - KH) / s + 1; workspace:
 * pipnet_wgrad_workspace_bytes(B*OH*OW, Cout, KH*KW*Cin). */
int pipnet_wgrad_conv_f32(const float* dY, const float* x, int B, int H, int W, int Cin, int KH, int KW, int stride,
                          int pad, int Cout, float* dW, int accumulate, float* workspace, void* stream);
int pipnet_colsum_workspace_bytes(int N);
int pipnet_colsum_f32(const float* A, int64_t lda, int M, int N, float* out, int accumulate, float* workspace,
                      void* stream);

/* ---- training backward of the trainable ConvNeXt suffix + PIP-Net head ----
 * Per-channel parameter gradients go through ``partial`` (device scratch of
 * pipnet_train_partials_floats(C) floats) and a fixed-order reduction; ``accumulate``
 * adds into the output instead of overwriting.  M = pixels (B*H*W), rows of C channels.
 * pipnet_gelu_fwd_f32: g = gelu_erf(h) (train forward keeps h for the backward).
 * pipnet_resid_scale_f32: out = x + row_scale[m / rows_per_scale] * (ls * y2)
 *   (CNBlock output with layer scale and stochastic depth; row_scale may be NULL).
 * pipnet_ls_bwd_f32: its backward w.r.t. y2 (dy2 = dy * ls * r), ls and the Linear2 bias.
 * pipnet_ln_bwd_f32: LayerNorm(C, eps 1e-6) backward from the pre-norm input z:
 *   dz (NULL to skip), d_gamma, d_beta.
 * pipnet_dwconv7_plain_f32: y (+)= [bias] + depthwise 7x7 pad 3 of x, w_packed [49][C]
 *   (the input gradient uses the spatially flipped taps, no bias, accumulate = 1).
 * pipnet_dwconv7_wgrad_f32: depthwise 7x7 weight ([49][C] packed) and bias gradients.
 * pipnet_head_bwd_f32: d loss / d logits of the PIP-Net head (softmax over P, max-pool over
 *   HW) for the align (w_align), tanh (w_tanh) and -- when d_out != NULL -- classifier terms
 *   (pipnet/train.py:154-265); proto NHWC [2Bh][HW][P], pooled [2Bh][P], W [K][P];
 *   argmax_ws int32 [2Bh*P], dpool_ws float [2Bh*P]. */
int64_t pipnet_train_partials_floats(int C);
int pipnet_gelu_fwd_f32(const float* h, float* g, int64_t n, void* stream);
int pipnet_resid_scale_f32(const float* x, const float* y2, const float* ls, const float* row_scale,
                           int rows_per_scale, int64_t M, int C, float* out, void* stream);
int pipnet_ls_bwd_f32(const float* dy, const float* y2, const float* ls, const float* row_scale, int rows_per_scale,
                      int64_t M, int C, float* dy2, float* d_ls, float* d_b2, int accumulate, float* partial,
                      void* stream);
int pipnet_ln_bwd_f32(const float* z, const float* dt, const float* gamma, int64_t M, int C, float* dz,
                      float* d_gamma, float* d_beta, int accumulate, float* partial, void* stream);
int pipnet_dwconv7_plain_f32(const float* x, int B, int H, int W, int C, const float* w_packed, const float* bias,
                             int accumulate, float* y, void* stream);
int pipnet_dwconv7_wgrad_f32(const float* dz, const float* x, int B, int H, int W, int C, float* dw_packed,
                             float* db, int accumulate, float* partial, void* stream);
int pipnet_head_bwd_f32(const float* proto, const float* pooled, int Bh, int HW, int P, const float* d_out,
                        const float* W, int K, float w_align, float w_tanh, float tanh_coeff, int32_t* argmax_ws,
                        float* dpool_ws, float* d_logits, void* stream);

/* ---- CountPIPNet pretrain / joint backward (pipnet/train.py:75-140 with is_count_pipnet;
 * count_pipnet.py:70-110, count_pipnet_utils.py:41-84, 188-321) ----------------------------
 * pipnet_count_ste_bwd_f32: d counts_raw from d clamped through STE_Round (identity) and
 *   ClampSTE(0, max_count) -- gated = 1 ("Gated": pass where the clamp input, rint(counts)
 *   with use_ste, the raw counts without, lies in [0, max_count]), 0 ("Identity").
 * pipnet_onehot_ste_bwd_f32: ModifiedSTEFunction.backward over rows = B*P of the encoding
 *   gradient g [rows][M]; x = the encoder input (clamped counts); strategy 0 = None/'none',
 *   1 = 'current_grad', 2 = 'max_grad'; flag_ws one int of workspace.  Reproduces the
 *   reference's effective behaviour (zero-count rows and the non-all-positive rows of a
 *   'max_grad' batch get 0: its chained mask assignments write temporaries).
 * pipnet_count_head_bwd_f32: d logits of the count head -- counts = spatial sums of
 *   proto = softmax((logits + g) * inv_tau) -- for the align (w_align), tanh (w_tanh on
 *   tanh_coeff * counts) terms plus d_counts_in (NULL or [2Bh][P], the classifier chain);
 *   proto NHWC [2Bh][HW][P], dcnt_ws float [2Bh*P]. */
int pipnet_count_ste_bwd_f32(const float* counts, int64_t n, int max_count, int use_ste, int gated,
                             const float* d_clamped, float* d_counts, void* stream);
int pipnet_onehot_ste_bwd_f32(const float* x, int64_t rows, int M, const float* g, int strategy, int respect_active,
                              int* flag_ws, float* dx, void* stream);
int pipnet_count_head_bwd_f32(const float* proto, const float* counts, int Bh, int HW, int P, const float* d_counts_in,
                              float w_align, float w_tanh, float tanh_coeff, float inv_tau, float* dcnt_ws,
                              float* d_logits, void* stream);

/* fp64-accumulated product for inference-time weight folds (csrc/fold_f64.hip):
 *   C[M,N] (ldc) = RNE_f32( sum_k double(A[m,k]) * double(B[k,n]) ), A [M,K] (lda) and B [K,N]
 *   (ldb) row-major fp32, products and sums in fp64 on v_mfma_f64_16x16x4_f64, any sizes.
 * Replaces the float64 torch matmul of the BilinearIntermediate fold (the embedding folded into
 * W and V: W(embed(x)) * V(embed(x)) = (W E) x * (V E) x, count_pipnet_utils.py:378-385) --
 * run once per weight version, off the steady-state forward. */
int pipnet_matmul_f64acc_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                             int M, int N, int K, void* stream);
/* Two such products sharing B in one launch: C0 = A0 B, C1 = A1 B (A0, A1 [M,K] with one lda; C0, C1
 * [M,N] with one ldc).  The fold of W and V against the same embedding E (count_pipnet_utils.py:
 * 378-385) as one grid of 2 x ceil(M/128) x ceil(N/128) tiles. */
int pipnet_matmul2_f64acc_f32(const float* A0, const float* A1, int64_t lda, const float* B, int64_t ldb,
                              float* C0, float* C1, int64_t ldc, int M, int N, int K, void* stream);

/* ---- ResNet training step (csrc/bn_ops.hip): BatchNorm2d in train mode ------------------
 * Replaces the autograd of nn.BatchNorm2d(C) under net.train() in the ResNet Bottleneck /
 * stem (features/resnet_features.py:77-119, 137-140; pipnet/train.py:14), NHWC rows
 * x[M][C], M = B*H*W, C % 4 == 0 (and C/4 >= 64 or dividing 256), 16-B aligned operands.
 * pipnet_bn_stats_f32: mean / invstd of the batch (two-pass biased variance, eps), and when
 *   running_mean / running_var are given the momentum update with the unbiased variance
 *   (torch semantics); M >= 2 (torch: "Expected more than 1 value per channel").
 * pipnet_bn_apply_f32: y = gamma (x - mean) invstd + beta [+ residual] [ReLU].
 * pipnet_bn_backward_f32: g = dy [* (relu_out > 0)]; d_beta = sum g, d_gamma = sum g xhat,
 *   dx = gamma invstd (g - d_beta/M - xhat d_gamma/M) (dx NULL: parameters only); d_masked
 *   (optional) receives g -- the identity-path gradient of a residual block.
 *   workspace: pipnet_bn_workspace_floats(C) floats, for both calls.
 * pipnet_stride_scatter_f32: out[B][H][W][C] (+)= in[B][OH][OW][C] placed on the stride
 *   lattice (zeros elsewhere): the input gradient of a stride-s 1x1 conv, and the
 *   zero-inserted gradient a stride-s 3x3 conv's input gradient is convolved from. */
int64_t pipnet_bn_workspace_floats(int C);
int pipnet_bn_stats_f32(const float* x, int64_t M, int C, float eps, float momentum, float* mean, float* invstd,
                        float* running_mean, float* running_var, float* workspace, void* stream);
int pipnet_bn_apply_f32(const float* x, int64_t M, int C, const float* mean, const float* invstd, const float* gamma,
                        const float* beta, const float* residual, int relu, float* y, void* stream);
int pipnet_bn_backward_f32(const float* x, const float* dy, const float* relu_out, int64_t M, int C,
                           const float* mean, const float* invstd, const float* gamma, float* dx, float* d_masked,
                           float* d_gamma, float* d_beta, float* workspace, void* stream);
int pipnet_stride_scatter_f32(const float* in, int B, int OH, int OW, int C, int H, int W, int stride, int accumulate,
                              float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PIPNET_AMD_H */
