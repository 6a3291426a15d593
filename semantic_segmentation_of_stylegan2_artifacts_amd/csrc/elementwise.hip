// Streaming kernels of the MS-UNet step: GELU fwd/bwd (torchvision MLP activation,
// FinalPatchExpand_X4_V2.act), the 4x4/s4 patch-embed im2col (PatchEmbed.proj,
// model_parts.py:211,222), DynamicLoss fwd/bwd (loss/DynamicLoss.py:82-111) and the fused
// AdamW step over flat parameter buffers (trainer.py:143-152, torch.optim.AdamW semantics).
// All HBM-bound: vectorised 4-wide, grid-stride, f32 math.  GELU: libm erff for f32 (the
// parity path), the one-exp / one-rcp erf of common.h for bf16 (|error| <= 1.5e-7, far below
// bf16 rounding; libm erff made the bf16 kernels VALU-bound).
#include <type_traits>

#include "common.h"

#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace {

template <typename T>
__global__ void __launch_bounds__(256) gelu_fwd_kernel(const T* x, T* y, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float v[4];
    Vec4<T>::load(x + 4 * i, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = (sizeof(T) == 2 && !(MSU_EXP & 1)) ? gelu_fast(v[e]) : gelu_f(v[e]);
    Vec4<T>::store(y + 4 * i, v);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) gelu_bwd_kernel(const T* x, const T* dy, T* dx, long n4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    float v[4], d[4];
    Vec4<T>::load(x + 4 * i, v);
    Vec4<T>::load(dy + 4 * i, d);
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] *= (sizeof(T) == 2 && !(MSU_EXP & 1)) ? gelu_grad_fast(v[e]) : gelu_grad_f(v[e]);
    Vec4<T>::store(dx + 4 * i, d);
  }
}

// out = a + b * scale[sample] (a may be null: out = b * scale[sample]): the residual add with
// StochasticDepth's per-sample scale (torchvision SwinTransformerBlock: x + stochastic_depth(f(x)))
// in one pass, and its backward for the branch (dy * scale[sample]).
template <typename T>
__global__ void __launch_bounds__(256) residual_kernel(const T* a, const T* b, const float* scale, T* out,
                                                       long n4, long per_sample4) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const float s = scale[i / per_sample4];
    float vb[4], va[4] = {0.f, 0.f, 0.f, 0.f};
    Vec4<T>::load(b + 4 * i, vb);
    if (a) Vec4<T>::load(a + 4 * i, va);
#pragma unroll
    for (int e = 0; e < 4; ++e) vb[e] = fmaf(vb[e], s, va[e]);
    Vec4<T>::store(out + 4 * i, vb);
  }
}

// img [B, Cin, H, W] f32 -> cols [B*(H/p)*(W/p), Cin*p*p] in (c, ky, kx) order = conv weight order
template <typename T>
__global__ void __launch_bounds__(256) patchify_kernel(const float* img, T* out, int B, int Cin,
                                                       int H, int W, int p) {
  const int Ho = H / p, Wo = W / p;
  const int K = Cin * p * p;
  const long total = (long)B * Ho * Wo * K;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long tok = i / K;
    const int k = (int)(i - tok * K);
    const int c = k / (p * p), r = k - c * p * p, ky = r / p, kx = r - (r / p) * p;
    const long b = tok / ((long)Ho * Wo);
    const int t = (int)(tok - b * Ho * Wo);
    const int oy = t / Wo, ox = t - (t / Wo) * Wo;
    out[i] = from_f32<T>(img[((b * Cin + c) * H + oy * p + ky) * (long)W + ox * p + kx]);
  }
}

// ---------------------------------------------------------------- DynamicLoss
// Per (sample, block) partial sums, for both the raw target and the >127.5-binarised one
// (the reference binarises iff target.max() > 1 over the WHOLE batch, DynamicLoss.py:87-88).
// part layout [B][nblk][12]: raw {bce, tp, fp, fn, tsum}, bin {bce, tp, fp, fn, tsum}, tmax, pad
constexpr int NS = 12;

template <typename T>
__global__ void __launch_bounds__(256) dynloss_partial_kernel(const T* logits, const float* target,
                                                              long N, int nblk, float* part) {
  const int b = blockIdx.y;
  const T* x = logits + (long)b * N;
  const float* t = target + (long)b * N;
  float acc[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) acc[k] = 0.f;
  acc[10] = -INFINITY;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < N; i += (long)nblk * 256) {
    const float xv = to_f32(x[i]);
    const float tr = t[i];
    const float p = 1.f / (1.f + __expf(-xv));
    const float sp = fmaxf(xv, 0.f) + log1pf(__expf(-fabsf(xv)));  // softplus(x) = max(x,0)+log1p(e^-|x|)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const float tv = m == 0 ? tr : (tr > 127.5f ? 1.f : 0.f);
      acc[m * 5 + 0] += sp - xv * tv;
      acc[m * 5 + 1] += p * tv;
      acc[m * 5 + 2] += p * (1.f - tv);
      acc[m * 5 + 3] += (1.f - p) * tv;
      acc[m * 5 + 4] += tv;
    }
    acc[10] = fmaxf(acc[10], tr);
  }
  __shared__ float red[4][11];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const float s = group_sum<64>(acc[k]);
    if (lane == 0) red[wv][k] = s;
  }
  const float mx = group_max<64>(acc[10]);
  if (lane == 0) red[wv][10] = mx;
  __syncthreads();
  if (threadIdx.x < 11) {
    const int k = threadIdx.x;
    float v = red[0][k];
    for (int w = 1; w < 4; ++w) v = k == 10 ? fmaxf(v, red[w][k]) : v + red[w][k];
    part[((long)b * nblk + blockIdx.x) * NS + k] = v;
  }
}

// One block: finalise per-sample loss terms.  coef[b] = {w_bce, has_tv, num, den}; flags[0]=binarise
// Per-sample totals over the nblk partial rows: one wave per (sample, quantity), lanes
// stride over the partial rows, fixed-order double-precision shuffle tree (deterministic).
MSU_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(512) dynloss_final_kernel(const float* part, int B, int nblk, long N,
                                                            float alpha, float beta, float mix,
                                                            float smooth, float* loss, float* flag,
                                                            float* coef, float* zero_out) {
  __shared__ int binarise;
  __shared__ double sums[64][5];  // B <= 64
  __shared__ float wmax[8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float mx = -INFINITY;
  for (long i = threadIdx.x; i < (long)B * nblk; i += 512) mx = fmaxf(mx, part[i * NS + 10]);
  mx = group_max<64>(mx);
  if (lane == 0) wmax[wave] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = wmax[0];
    for (int w = 1; w < 8; ++w) m = fmaxf(m, wmax[w]);
    binarise = m > 1.f;
  }
  __syncthreads();
  const int o = binarise ? 5 : 0;
  for (int bq = wave; bq < B * 5; bq += 8) {
    const int b = bq / 5, q = bq - (bq / 5) * 5;
    double v = 0.0;
    for (int k = lane; k < nblk; k += 64) v += part[((long)b * nblk + k) * NS + o + q];
    v = wave_sum_d(v);
    if (lane == 0) sums[b][q] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double total = 0.0;
    for (int b = 0; b < B; ++b) {
      const double* s = sums[b];
      const double bce = s[0] / (double)N;
      float* c = coef + 4 * b;
      if (s[4] != 0.0) {
        const double num = s[1] + smooth;
        const double den = s[1] + alpha * s[2] + beta * s[3] + smooth;
        total += (1.0 - mix) * bce + mix * (1.0 - num / den);
        c[0] = (float)((1.0 - mix) / (double)N);
        c[1] = 1.f;
        c[2] = (float)num;
        c[3] = (float)den;
      } else {
        total += bce;
        c[0] = (float)(1.0 / (double)N);
        c[1] = 0.f; c[2] = 1.f; c[3] = 1.f;
      }
    }
    loss[0] = (float)(total / B);
    flag[0] = (float)binarise;
    if (zero_out) zero_out[0] = 0.f;  // the trainer's non-finite flag, reset for this step
  }
}

template <typename T>
__global__ void __launch_bounds__(256) dynloss_bwd_kernel(const T* logits, const float* target,
                                                          const float* coef, const float* flag,
                                                          const float* gout, long N, int B,
                                                          float alpha, float beta, float mix,
                                                          float* dlogits) {
  const long total = N * B;
  const bool bin = flag[0] != 0.f;
  const float g = gout ? gout[0] / B : 1.f / B;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int b = (int)(i / N);
    const float* c = coef + 4 * b;
    const float xv = to_f32(logits[i]);
    float tv = target[i];
    if (bin) tv = tv > 127.5f ? 1.f : 0.f;
    const float p = 1.f / (1.f + __expf(-xv));
    float d = c[0] * (p - tv);
    if (c[1] != 0.f) {
      const float num = c[2], den = c[3];
      const float dti = (tv * den - num * (tv + alpha * (1.f - tv) - beta * tv)) / (den * den);
      d -= mix * dti * p * (1.f - p);
    }
    dlogits[i] = g * d;
  }
}

// ---------------------------------------------------------------- AdamW (torch semantics)
__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, long n,
                                                    float lr, float b1, float b2, float eps, float wd,
                                                    float bc1, float bc2_sqrt, const float* inv_scale,
                                                    const float* found_inf) {
  if (found_inf && found_inf[0] != 0.f) return;
  const float is = inv_scale ? inv_scale[0] : 1.f;
  const float step_size = lr / bc1;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float gi = g[i] * is;
    float pi = p[i] * (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    pi -= step_size * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
  }
}

// Device-resident hyper-parameters (hyper = {lr, step}, f64): the launch carries no per-step
// host scalar, so a step can be replayed from a HIP graph and a skipped step (found_inf, the
// GradScaler rule of trainer.py:315-316) leaves the step count where it was.  Every scalar is
// formed in double and rounded once, and the update follows torch.optim.AdamW's operation
// order (param.mul_(1 - lr*wd); exp_avg.lerp_(g, 1 - b1); exp_avg_sq.mul_(b2).addcmul_(g, g,
// 1 - b2); param.addcdiv_(exp_avg, sqrt(exp_avg_sq) / sqrt(bc2) + eps, -lr / bc1)).
// S: the 16-bit shadow written with the updated parameter (void: none); ZERO: the gradient is
// zeroed after it was read (also on a skipped step) -- the step's gradient reset and bf16 shadow
// refresh in the same pass instead of a fill and a re-read of the parameters
template <typename S, bool ZERO>
__global__ void __launch_bounds__(256) adamw_dev_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, long n,
                                                        const double* hyper, double b1, double b2, float eps,
                                                        double wd, const float* inv_scale,
                                                        const float* found_inf, S* __restrict__ shadow) {
#pragma clang fp contract(off)
  if (found_inf && found_inf[0] != 0.f) {
    if constexpr (ZERO)
      for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) g[i] = 0.f;
    return;
  }
  const double lr = hyper[0];
  const double step = hyper[1];
  const float decay = (float)(1.0 - lr * wd);
  const float w1 = (float)(1.0 - b1);
  const float b2f = (float)b2, w2 = (float)(1.0 - b2);
  const float neg_step_size = (float)(-(lr / (1.0 - pow(b1, step))));
  const float bc2_sqrt = (float)sqrt(1.0 - pow(b2, step));
  const float is = inv_scale ? inv_scale[0] : 1.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const float gi = inv_scale ? g[i] * is : g[i];
    const float pi = p[i] * decay;
    float mi = m[i];
    mi = w1 < 0.5f ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);  // ATen lerp
    const float vi = v[i] * b2f + w2 * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = __fsqrt_rn(vi) / bc2_sqrt + eps;
    const float pn = pi + neg_step_size * (mi / denom);
    p[i] = pn;
    if constexpr (!std::is_void_v<S>) shadow[i] = from_f32<S>(pn);  // the cast copy_shadow made
    if constexpr (ZERO) g[i] = 0.f;
  }
}

// hyper[1] += 1 unless the step is skipped (one thread)
__global__ void step_advance_kernel(double* hyper, const float* found_inf) {
  if (threadIdx.x == 0 && !(found_inf && found_inf[0] != 0.f)) hyper[1] = hyper[1] + 1.0;
}

// any non-finite in x0[0:n0] or x1[0:n1] -> flag[0] = 1 (flag zeroed by the caller)
__global__ void __launch_bounds__(256) nonfinite2_kernel(const float* x0, long n0, const float* x1, long n1,
                                                         float* flag) {
  bool bad = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n0 + n1; i += (long)gridDim.x * 256)
    bad |= !isfinite(i < n0 ? x0[i] : x1[i - n0]);
  if (__any(bad) && (threadIdx.x & 63) == 0) flag[0] = 1.f;
}

// any non-finite in x -> flag[0] = 1 (flag must be zeroed by the caller)
__global__ void __launch_bounds__(256) nonfinite_kernel(const float* x, long n, float* flag) {
  bool bad = false;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x & 63) == 0) flag[0] = 1.f;
}

template <typename T>
__global__ void __launch_bounds__(256) cast_kernel(const float* x, T* y, long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    y[i] = from_f32<T>(x[i]);
}

// Refine-conv weight in the layouts the implicit-GEMM conv reads (ops.py _refine_impl /
// _refine_backward; the reference's nn.Conv2d weight [Cout][Cin][3][3], model_parts.py:447-448):
// flip 0: out[t][co][ci] = W[co][ci][t], ci padded with zeros to P = roundup(Cin, 32);
// flip 1: out[t][ci][co] = W[co][ci][8 - t], co padded to P = roundup(Cout, 32).
// One thread per output element (<= 9 x 192 x 224 per conv: one launch, read once, L2-resident).
template <typename T>
__global__ void __launch_bounds__(256) conv_weight_kernel(const float* w, T* out, int Cout, int Cin,
                                                          int flip, int P, long n) {
  long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int inner = (int)(i % P);
  long r = i / P;
  int outer = (int)(r % (flip ? Cin : Cout));
  int t = (int)(r / (flip ? Cin : Cout));
  int co = flip ? inner : outer, ci = flip ? outer : inner;
  float v = 0.f;
  if (co < Cout && ci < Cin) v = w[((long)co * Cin + ci) * 9 + (flip ? 8 - t : t)];
  out[i] = from_f32<T>(v);
}

// Batched 16-bit transpose: entry e = {src offset, dst offset, N, K, first tile} (int64, in
// elements of the two flat bases) turns src[N][K] into dst[K][N]; a block moves one 64 x 64
// tile through LDS with 16-B loads and stores (N, K multiples of 8).  Entries are found by a
// binary search over their first tiles (ascending).
__global__ void __launch_bounds__(256) transpose16_multi_kernel(const uint16_t* __restrict__ src,
                                                                uint16_t* __restrict__ dst,
                                                                const long long* __restrict__ tab, int nent) {
  __shared__ uint16_t t[64][64 + 8];
  const int tile = blockIdx.x;
  int lo = 0, hi = nent - 1;
  while (lo < hi) {  // last entry whose first tile <= tile
    const int mid = (lo + hi + 1) >> 1;
    if (tab[5 * mid + 4] <= tile) lo = mid; else hi = mid - 1;
  }
  const long long* e = tab + 5 * lo;
  const uint16_t* s = src + e[0];
  uint16_t* d = dst + e[1];
  const int N = (int)e[2], K = (int)e[3];
  const int r = tile - (int)e[4];
  const int tk = (K + 63) / 64;
  const int n0 = (r / tk) * 64, k0 = (r % tk) * 64;
  const int c8 = (threadIdx.x & 7) * 8;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rr = (threadIdx.x >> 3) + 32 * i;
    if (n0 + rr < N && k0 + c8 < K) {
      const uint4 v = *reinterpret_cast<const uint4*>(s + (long)(n0 + rr) * K + k0 + c8);
      const uint16_t* pv = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[c8 + j][rr] = pv[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kk = (threadIdx.x >> 3) + 32 * i;
    if (k0 + kk < K && n0 + c8 < N)
      *reinterpret_cast<uint4*>(d + (long)(k0 + kk) * N + n0 + c8) = *reinterpret_cast<const uint4*>(&t[kk][c8]);
  }
}

inline unsigned grid_for(long n, long per_block = 256, long cap = 8192) {
  long nb = (n + per_block - 1) / per_block;
  if (nb > cap) nb = cap;
  return (unsigned)(nb < 1 ? 1 : nb);
}

}  // namespace

extern "C" {

int msu_gelu_fwd(int dtype, const void* x, void* y, long n, void* stream) {
  if (n % 4) return -2;
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(gelu_fwd_kernel<T>, dim3(grid_for(n / 4)), dim3(256), 0, st,
                                            (const T*)x, (T*)y, n / 4));
  return MSU_CHECK_LAUNCH();
}

int msu_gelu_bwd(int dtype, const void* x, const void* dy, void* dx, long n, void* stream) {
  if (n % 4) return -2;
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(gelu_bwd_kernel<T>, dim3(grid_for(n / 4)), dim3(256), 0, st,
                                            (const T*)x, (const T*)dy, (T*)dx, n / 4));
  return MSU_CHECK_LAUNCH();
}

int msu_residual(int dtype, const void* a, const void* b, const float* scale, void* out, long n, long per_sample,
                 void* stream) {
  if (n % 4 || per_sample % 4 || per_sample <= 0 || scale == nullptr) return -2;
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(residual_kernel<T>, dim3(grid_for(n / 4)), dim3(256), 0, st,
                                            (const T*)a, (const T*)b, scale, (T*)out, n / 4, per_sample / 4));
  return MSU_CHECK_LAUNCH();
}

int msu_patchify(int dtype, const float* img, void* out, int B, int Cin, int H, int W, int p,
                 void* stream) {
  if (H % p || W % p) return -2;
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)B * Cin * H * W;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(patchify_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, img,
                                            (T*)out, B, Cin, H, W, p));
  return MSU_CHECK_LAUNCH();
}

int msu_dynloss_nblk(long N) {
  long nb = (N + 256 * 16 - 1) / (256 * 16);
  if (nb > 256) nb = 256;
  return (int)(nb < 1 ? 1 : nb);
}

// loss[0] = loss value, flag[0] = binarised flag; coef [B*4]; part [B*nblk*12]; zero_out (nullable)
// is set to 0 by the same single-block launch
int msu_dynloss_fwd3(int dtype, const void* logits, const float* target, int B, long N,
                     float alpha, float beta, float mix, float* part, int nblk, float* loss, float* flag,
                     float* coef, float* zero_out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(dynloss_partial_kernel<T>, dim3(nblk, B), dim3(256), 0, st,
                                            (const T*)logits, target, N, nblk, part));
  if (B > 64) return -2;
  hipLaunchKernelGGL(dynloss_final_kernel, dim3(1), dim3(512), 0, st, part, B, nblk, N, alpha, beta,
                     mix, 1e-6f, loss, flag, coef, zero_out);
  return MSU_CHECK_LAUNCH();
}

int msu_dynloss_fwd2(int dtype, const void* logits, const float* target, int B, long N,
                     float alpha, float beta, float mix, float* part, int nblk, float* loss, float* flag,
                     float* coef, void* stream) {
  return msu_dynloss_fwd3(dtype, logits, target, B, N, alpha, beta, mix, part, nblk, loss, flag, coef, nullptr,
                          stream);
}

// loss[0] = loss value, loss[1] = binarised flag
int msu_dynloss_fwd(int dtype, const void* logits, const float* target, int B, long N,
                    float alpha, float beta, float mix, float* part, int nblk, float* loss,
                    float* coef, void* stream) {
  return msu_dynloss_fwd2(dtype, logits, target, B, N, alpha, beta, mix, part, nblk, loss, loss + 1, coef, stream);
}

int msu_dynloss_bwd2(int dtype, const void* logits, const float* target, const float* coef,
                     const float* flag, const float* gout, int B, long N, float alpha, float beta,
                     float mix, float* dlogits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long n = (long)B * N;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(dynloss_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st,
                                            (const T*)logits, target, coef, flag, gout, N, B, alpha, beta, mix,
                                            dlogits));
  return MSU_CHECK_LAUNCH();
}

int msu_dynloss_bwd(int dtype, const void* logits, const float* target, const float* coef,
                    const float* loss, const float* gout, int B, long N, float alpha, float beta,
                    float mix, float* dlogits, void* stream) {
  return msu_dynloss_bwd2(dtype, logits, target, coef, loss + 1, gout, B, N, alpha, beta, mix, dlogits, stream);
}

int msu_adamw(float* p, const float* g, float* m, float* v, long n, float lr, float beta1,
              float beta2, float eps, float weight_decay, int step, const float* inv_scale,
              const float* found_inf, void* stream) {
  if (n == 0) return 0;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n, 256, 16384)), dim3(256), 0, (hipStream_t)stream,
                     p, g, m, v, n, lr, beta1, beta2, eps, weight_decay, (float)bc1,
                     (float)sqrt(bc2), inv_scale, found_inf);
  return MSU_CHECK_LAUNCH();
}

int msu_adamw_dev(float* p, const float* g, float* m, float* v, long n, const double* hyper, double beta1,
                  double beta2, double eps, double weight_decay, const float* inv_scale, const float* found_inf,
                  void* stream) {
  if (n == 0) return 0;
  if (hyper == nullptr) return -2;
  hipLaunchKernelGGL((adamw_dev_kernel<void, false>), dim3(grid_for(n, 256, 16384)), dim3(256), 0,
                     (hipStream_t)stream, p, const_cast<float*>(g), m, v, n, hyper, beta1, beta2, (float)eps,
                     weight_decay, inv_scale, found_inf, (void*)nullptr);
  return MSU_CHECK_LAUNCH();
}

int msu_adamw_dev2(float* p, float* g, float* m, float* v, long n, const double* hyper, double beta1, double beta2,
                   double eps, double weight_decay, const float* inv_scale, const float* found_inf, void* shadow,
                   int shadow_dtype, int zero_grad, void* stream) {
  if (n == 0) return 0;
  if (hyper == nullptr || (shadow != nullptr && !msu_is16(shadow_dtype))) return -2;
  const dim3 grid(grid_for(n, 256, 16384));
  hipStream_t st = (hipStream_t)stream;
#define MSU_ADAMW(S, Z)                                                                                         \
  hipLaunchKernelGGL((adamw_dev_kernel<S, Z>), grid, dim3(256), 0, st, p, g, m, v, n, hyper, beta1, beta2,      \
                     (float)eps, weight_decay, inv_scale, found_inf, (S*)shadow)
  if (shadow == nullptr) {
    if (zero_grad) MSU_ADAMW(void, true);
    else MSU_ADAMW(void, false);
  } else {
    MSU_DISPATCH16(shadow_dtype, T, if (zero_grad) MSU_ADAMW(T, true); else MSU_ADAMW(T, false));
  }
#undef MSU_ADAMW
  return MSU_CHECK_LAUNCH();
}

int msu_step_advance(double* hyper, const float* found_inf, void* stream) {
  if (hyper == nullptr) return -2;
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, hyper, found_inf);
  return MSU_CHECK_LAUNCH();
}

int msu_nonfinite2(const float* x0, long n0, const float* x1, long n1, float* flag, void* stream) {
  if (n0 + n1 == 0) return 0;
  hipLaunchKernelGGL(nonfinite2_kernel, dim3(grid_for(n0 + n1, 256, 16384)), dim3(256), 0, (hipStream_t)stream,
                     x0, n0, x1, n1, flag);
  return MSU_CHECK_LAUNCH();
}

int msu_nonfinite(const float* x, long n, float* flag, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, flag);
  return MSU_CHECK_LAUNCH();
}

int msu_cast(int dtype, const float* x, void* y, long n, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(cast_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, x, (T*)y, n));
  return MSU_CHECK_LAUNCH();
}

int msu_conv3x3_weight(int dtype, const float* W, void* out, int Cout, int Cin, int flip, void* stream) {
  if (Cout <= 0 || Cin <= 0) return 0;
  int P = ((flip ? Cout : Cin) + 31) / 32 * 32;
  long n = 9L * (flip ? Cin : Cout) * P;
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH(dtype, T, hipLaunchKernelGGL(conv_weight_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                                            st, W, (T*)out, Cout, Cin, flip, P, n));
  return MSU_CHECK_LAUNCH();
}

int msu_transpose16_multi(const void* src, void* dst, const long long* table, int nent, int ntiles,
                          void* stream) {
  if (nent <= 0 || ntiles <= 0) return 0;
  hipLaunchKernelGGL(transpose16_multi_kernel, dim3(ntiles), dim3(256), 0, (hipStream_t)stream,
                     (const uint16_t*)src, (uint16_t*)dst, table, nent);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
