// eval_pipnet metric loop on the GPU (reference pipnet/test.py:67-131,
// 266-319).  The reference materialises scores = pooled * W as a [K, B, P] tensor per batch
// and syncs the host ~B+5 times per batch (.item(), a Python loop over GPU scalars for the
// confusion matrix).  Here one batch is three small launches that never leave the device:
//
//   eval_image_kernel   (one workgroup per image)  argmax / max score (torch.max, first
//                       index), softmax(log1p(out^m)) confidence, abstain flag, top-1 hit,
//                       confusion-matrix atomic, and the per-image explanation sizes
//                       (|pooled*W| > thr for the predicted class / any class, |pooled| > thr)
//   eval_class_kernel   (one workgroup per class)  prototypes with relu(pooled*W - thr)
//                       mean > 0 over the batch (= some image has pooled*W > thr)
//   eval_reduce_kernel  (one workgroup)            per-batch float32 means, accumulated in
//                       fp64 exactly as the reference's running Python floats
//
// Float semantics follow the reference on the CPU: products pooled*W in fp32, means as
// fp32 sum / n (torch's CPU mean = sum().div_(n); the counts are exact integers), running
// totals in double.
#include "common.hpp"

namespace {

constexpr int EVT = 256;

PIPNET_DEV void block_argmax(float& v, int& idx, float* sv, int* si) {
  // (max value, first index among equal maxima); NaN never wins (torch.max would return it,
  // but the head never produces NaN)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) v = ov, idx = oi;
  }
  if (lane == 0) sv[w] = v, si[w] = idx;
  __syncthreads();
  v = sv[0];
  idx = si[0];
  for (int i = 1; i < EVT / 64; ++i)
    if (sv[i] > v || (sv[i] == v && si[i] < idx)) v = sv[i], idx = si[i];
  __syncthreads();
}

PIPNET_DEV float block_sum_f(float x, float* s) {
  x = wave_sum(x);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < EVT / 64; ++i) t += s[i];
  __syncthreads();
  return t;
}

PIPNET_DEV float block_max_f(float x, float* s) {
  x = wave_max(x);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  float t = s[0];
  for (int i = 1; i < EVT / 64; ++i) t = fmaxf(t, s[i]);
  __syncthreads();
  return t;
}

PIPNET_DEV int block_sum_i(int x, int* s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = x;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < EVT / 64; ++i) t += s[i];
  __syncthreads();
  return t;
}

// ws layout (int32): [0,B) predicted-class size, [B,2B) any-class size, [2B,3B) almost-nz,
// [3B,4B) top-1 hit, [4B,5B) abstained flag, [5B,5B+K) prototypes per class
__global__ __launch_bounds__(EVT) void eval_image_kernel(const float* __restrict__ pooled,
                                                         const float* __restrict__ out,
                                                         const float* __restrict__ W, int B, int P, int K,
                                                         const int64_t* __restrict__ ys,
                                                         const float* __restrict__ mult, float thr,
                                                         int32_t* __restrict__ ys_pred, float* __restrict__ score,
                                                         int64_t* __restrict__ cm, int32_t* __restrict__ ws) {
  __shared__ float sv[EVT / 64];
  __shared__ int si[EVT / 64];
  const int b = blockIdx.x;
  const float* o = out + (int64_t)b * K;
  // torch.max(out, dim=1): value and first index of the maximum
  float mv = -INFINITY;
  int mi = 0x7fffffff;
  for (int k = threadIdx.x; k < K; k += EVT) {
    const float v = o[k];
    if (v > mv || (v == mv && k < mi)) mv = v, mi = k;
  }
  block_argmax(mv, mi, sv, si);
  const int pred = mi;
  // amax(softmax(log1p(out ** m))) = 1 / sum_k exp(z_k - max z)
  const float m = mult ? *mult : 1.0f;
  float zm = -INFINITY;
  for (int k = threadIdx.x; k < K; k += EVT) zm = fmaxf(zm, log1pf(powf(o[k], m)));
  zm = block_max_f(zm, sv);
  float se = 0.f;
  for (int k = threadIdx.x; k < K; k += EVT) se += expf(log1pf(powf(o[k], m)) - zm);
  se = block_sum_f(se, sv);
  // explanation sizes over prototypes
  const float* pl = pooled + (int64_t)b * P;
  const float* wp = W + (int64_t)pred * P;
  int n_pred = 0, n_any = 0, n_nz = 0;
  for (int p = threadIdx.x; p < P; p += EVT) {
    const float pv = pl[p];
    n_nz += fabsf(pv) > thr;
    n_pred += fabsf(pv * wp[p]) > thr;
    int any = 0;
    for (int k = 0; k < K && !any; ++k) any = fabsf(pv * W[(int64_t)k * P + p]) > thr;
    n_any += any;
  }
  n_pred = block_sum_i(n_pred, si);
  n_any = block_sum_i(n_any, si);
  n_nz = block_sum_i(n_nz, si);
  if (threadIdx.x == 0) {
    const int64_t y = ys[b];
    ys_pred[b] = pred;
    score[b] = 1.0f / se;
    ws[b] = n_pred;
    ws[B + b] = n_any;
    ws[2 * B + b] = n_nz;
    ws[3 * B + b] = (int64_t)pred == y;
    ws[4 * B + b] = mv == 0.f;
    if (y >= 0 && y < K) atomicAdd(reinterpret_cast<unsigned long long*>(cm + y * K + pred), 1ull);
  }
}

__global__ __launch_bounds__(EVT) void eval_class_kernel(const float* __restrict__ pooled,
                                                         const float* __restrict__ W, int B, int P, int K,
                                                         float thr, int32_t* __restrict__ ws) {
  __shared__ int si[EVT / 64];
  const int k = blockIdx.x;
  int n = 0;
  for (int p = threadIdx.x; p < P; p += EVT) {
    const float w = W[(int64_t)k * P + p];
    int hit = 0;
    for (int b = 0; b < B && !hit; ++b) hit = pooled[(int64_t)b * P + p] * w - thr > 0.f;
    n += hit;
  }
  n = block_sum_i(n, si);
  if (threadIdx.x == 0) ws[5 * B + k] = n;
}

// acc[0] local_size_for_true_class, [1] local_size_for_all_classes, [2] prototypes_per_class,
// [3] almost_nonzeros, [4] top1 -- running sums of per-batch float32 means; abstained += count
__global__ __launch_bounds__(EVT) void eval_reduce_kernel(const int32_t* __restrict__ ws, int B, int K,
                                                          double* __restrict__ acc, int64_t* __restrict__ abstained) {
  __shared__ int si[EVT / 64];
  int s[6] = {0, 0, 0, 0, 0, 0};
  for (int b = threadIdx.x; b < B; b += EVT)
#pragma unroll
    for (int j = 0; j < 5; ++j) s[j] += ws[j * B + b];
  for (int k = threadIdx.x; k < K; k += EVT) s[5] += ws[5 * B + k];
#pragma unroll
  for (int j = 0; j < 6; ++j) s[j] = block_sum_i(s[j], si);
  if (threadIdx.x == 0) {
    const float fb = (float)B;
    acc[0] += (double)((float)s[0] / fb);
    acc[1] += (double)((float)s[1] / fb);
    acc[2] += (double)((float)s[5] / (float)K);
    acc[3] += (double)((float)s[2] / fb);
    acc[4] += (double)((float)s[3] / fb);
    *abstained += s[4];
  }
}

__global__ __launch_bounds__(256) void sparsify_kernel(float* __restrict__ w, int64_t n, float delta) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    w[i] = fmaxf(w[i] - delta, 0.f);
}

}  // namespace

extern "C" int pipnet_eval_batch_f32(const float* pooled, const float* out, const float* W, int B, int P, int K,
                                     const int64_t* ys, const float* multiplier, float thr, int32_t* ys_pred,
                                     float* score, int64_t* cm, double* acc, int64_t* abstained, int32_t* workspace,
                                     void* stream) {
  if (B < 0 || P <= 0 || K <= 0 || !pooled || !out || !W || !ys || !ys_pred || !score || !cm || !acc ||
      !abstained || !workspace)
    return PIPNET_ERR_ARG;
  if (B == 0) return PIPNET_OK;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(eval_image_kernel, dim3(B), dim3(EVT), 0, s, pooled, out, W, B, P, K, ys, multiplier, thr,
                     ys_pred, score, cm, workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(eval_class_kernel, dim3(K), dim3(EVT), 0, s, pooled, W, B, P, K, thr, workspace);
  PIPNET_CHECK_LAUNCH();
  hipLaunchKernelGGL(eval_reduce_kernel, dim3(1), dim3(EVT), 0, s, workspace, B, K, acc, abstained);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}

extern "C" int pipnet_weight_sparsify_f32(float* w, int64_t n, float delta, void* stream) {
  if (n < 0 || !w) return PIPNET_ERR_ARG;
  if (n == 0) return PIPNET_OK;
  const int64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(sparsify_kernel, dim3((unsigned)(g < 4096 ? g : 4096)), dim3(256), 0, (hipStream_t)stream, w, n,
                     delta);
  PIPNET_CHECK_LAUNCH();
  return PIPNET_OK;
}
