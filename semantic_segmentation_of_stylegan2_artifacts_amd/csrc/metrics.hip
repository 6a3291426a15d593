// Validation metrics of scripts/validation_functions.py on the GPU, one pass over the
// logits: per image p = sigmoid(logit), pred_bin = p > threshold, gt = label > 0 and
//   soft sums   sum(p*g), sum(p^2), sum(g^2), sum(p), sum(g)            (:289-304)
//   soft confusion  sum((1-g)p), sum(g(1-p)), sum((1-p)(1-g))            (:219-222, :291-294)
//   binary confusion tp, fp, fn, tn                                      (:208-213, :266-269)
// from which the host forms soft / binary Dice and IoU, recall, precision, accuracy and FPR
// (calculate_metrics_fake :247-309, calculate_metrics_real :201-244) -- no per-image D2H of
// the prediction, no medpy.  Per (image, block) f32 partials (binary counts exact: <= 2^24
// per block), then per-image totals in double, in a fixed order (deterministic).
#include "common.h"

namespace {

constexpr int NQ = 12;  // quantities per partial row

template <typename T>
__global__ void __launch_bounds__(256) metrics_partial_kernel(const T* logits, const float* label, long N,
                                                              int nblk, float thr, float* part) {
  const int b = blockIdx.y;
  const T* x = logits + (long)b * N;
  const float* t = label + (long)b * N;
  float acc[NQ];
#pragma unroll
  for (int k = 0; k < NQ; ++k) acc[k] = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long)nblk * 256) {
    const float p = 1.f / (1.f + __expf(-to_f32(x[i])));
    const float g = t[i] > 0.f ? 1.f : 0.f;  // ground_truth = label > 0 (validation_functions.py:108)
    const float pb = p > thr ? 1.f : 0.f;
    acc[0] += p * g;
    acc[1] += p * p;
    acc[2] += g;  // g*g == g
    acc[3] += p;
    acc[4] += (1.f - g) * p;
    acc[5] += g * (1.f - p);
    acc[6] += (1.f - p) * (1.f - g);
    acc[7] += pb * g;                  // tp
    acc[8] += pb * (1.f - g);          // fp
    acc[9] += (1.f - pb) * g;          // fn
    acc[10] += (1.f - pb) * (1.f - g); // tn
  }
  __shared__ float red[4][NQ];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const float s = group_sum<64>(acc[k]);
    if (lane == 0) red[wv][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < NQ) {
    const int k = threadIdx.x;
    part[((long)b * nblk + blockIdx.x) * NQ + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// one wave per (image, quantity): lanes stride the partial rows, fixed-order double tree
__global__ void __launch_bounds__(256) metrics_final_kernel(const float* part, int B, int nblk, double* out) {
  const int lane = threadIdx.x & 63;
  const int wq = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wq >= B * NQ) return;
  const int b = wq / NQ, q = wq - (wq / NQ) * NQ;
  double v = 0.0;
  for (int k = lane; k < nblk; k += 64) v += (double)part[((long)b * nblk + k) * NQ + q];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) out[(long)b * NQ + q] = v;
}

}  // namespace

extern "C" {

int msu_metrics_nblk(long N) {
  long nb = (N + 256 * 16 - 1) / (256 * 16);
  if (nb > 256) nb = 256;
  return (int)(nb < 1 ? 1 : nb);
}

// logits [B, N] (f32, bf16 or f16), label [B, N] f32; part [B * nblk * 12] f32 scratch;
// out [B, 12] f64: sum(p g), sum(p^2), sum(g), sum(p), soft fp, soft fn, soft tn, tp, fp, fn,
// tn, 0.
int msu_seg_metrics(int dtype, const void* logits, const float* label, int B, long N, float threshold,
                    float* part, int nblk, double* out, void* stream) {
  if (B <= 0 || N <= 0 || nblk <= 0) return -2;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)nblk, (unsigned)B);
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(metrics_partial_kernel<T>, grid, dim3(256), 0, st, (const T*)logits,
                                            label, N, nblk, threshold, part));
  hipLaunchKernelGGL(metrics_final_kernel, dim3((unsigned)((B * NQ + 3) / 4)), dim3(256), 0, st, part, B, nblk, out);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
