// Deterministic column reduction of per-block partial rows: out[i] (+)= sum_p part[p*stride + i].
// Block = (256/PL) columns x PL part-lanes; each part-lane walks parts p = ly, ly+PL, ...
// in a fixed order with 8 loads in flight, then the PL lane partials are added in a fixed
// order through LDS.  Narrow reductions (LayerNorm affine, biases: a few hundred columns,
// ~1000 parts) use 32 part-lanes so enough loads are in flight; wide ones (weight-gradient
// slabs) 8 part-lanes for coalescing.
#pragma once
#include "common.h"

namespace {

template <int PL>
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ part, int nparts, long n,
                                                     long stride, float* __restrict__ out, int accumulate) {
  constexpr int NC = 256 / PL;
  __shared__ float red[PL][NC + 1];
  const int lx = threadIdx.x % NC, ly = threadIdx.x / NC;
  const long i = (long)blockIdx.x * NC + lx;
  float s = 0.f;
  if (i < n) {
    int p = ly;
    for (; p + 7 * PL < nparts; p += 8 * PL) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)(p + u * PL) * stride + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; p < nparts; p += PL) s += part[(long)p * stride + i];
  }
  red[ly][lx] = s;
  __syncthreads();
  if (ly == 0 && i < n) {
    float t = red[0][lx];
#pragma unroll
    for (int k = 1; k < PL; ++k) t += red[k][lx];
    out[i] = accumulate ? out[i] + t : t;
  }
}

inline void colsum(const float* part, int nparts, long n, long stride, float* out, int accumulate,
                   hipStream_t st) {
  if (n <= 4096)
    hipLaunchKernelGGL(colsum_kernel<32>, dim3((unsigned)((n + 7) / 8)), dim3(256), 0, st, part, nparts, n,
                       stride, out, accumulate);
  else
    hipLaunchKernelGGL(colsum_kernel<8>, dim3((unsigned)((n + 31) / 32)), dim3(256), 0, st, part, nparts, n,
                       stride, out, accumulate);
}

}  // namespace
