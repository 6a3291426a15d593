// Deterministic column reduction of per-block partial rows: out[i] (+)= sum_p part[p*stride + i].
// Block = 32 columns x 8 part-lanes; each part-lane walks parts p = ly, ly+8, ... (fixed
// order), then the 8 lane partials are added in fixed order through LDS.  Coalesced over
// columns, parallel over parts (the serial one-thread-per-column form was 30 ms/step).
#pragma once
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ part, int nparts, long n,
                                                     long stride, float* __restrict__ out, int accumulate) {
  __shared__ float red[8][33];
  const int lx = threadIdx.x & 31, ly = threadIdx.x >> 5;
  const long i = (long)blockIdx.x * 32 + lx;
  float s = 0.f;
  if (i < n) {
    int p = ly;
    for (; p + 24 < nparts; p += 32) {
      const float a = part[(long)p * stride + i];
      const float b = part[(long)(p + 8) * stride + i];
      const float c = part[(long)(p + 16) * stride + i];
      const float d = part[(long)(p + 24) * stride + i];
      s += a; s += b; s += c; s += d;
    }
    for (; p < nparts; p += 8) s += part[(long)p * stride + i];
  }
  red[ly][lx] = s;
  __syncthreads();
  if (ly == 0 && i < n) {
    float t = red[0][lx];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][lx];
    out[i] = accumulate ? out[i] + t : t;
  }
}

inline void colsum(const float* part, int nparts, long n, long stride, float* out, int accumulate,
                   hipStream_t st) {
  hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((n + 31) / 32)), dim3(256), 0, st, part, nparts, n,
                     stride, out, accumulate);
}

}  // namespace
