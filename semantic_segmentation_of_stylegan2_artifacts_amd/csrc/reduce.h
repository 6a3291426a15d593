// Deterministic column reduction of per-block partial rows: out[i] (+)= sum_p part[p*stride + i].
// The output may be a column slice of a wider row-major matrix: element i goes to
// out[(i / rowlen) * ldo + i % rowlen] (rowlen = n, ldo = n: contiguous).
// Block = (256/PL) column groups (V = 4 floats each, 16-B loads, when aligned) x PL part-lanes;
// each part-lane walks parts p = ly, ly+PL, ... in a fixed order with 8 loads in flight, then
// the PL lane partials are added in a fixed order through LDS.  Narrow reductions (LayerNorm
// affine, biases: a few hundred columns, ~1000 parts) use 32 part-lanes so enough loads are in
// flight; wide ones (weight-gradient slabs) 8 part-lanes.  Several reductions over the same
// parts (a weight slab and its bias) share one launch.
#pragma once
#include "common.h"

namespace {

// Up to three independent reductions over the same number of parts in one launch (a weight
// slab and its bias, LayerNorm gamma / beta, ...): blocks [bend[j-1], bend[j]) serve segment j.
struct ColSegs {
  const float* part[3];
  float* out[3];
  long n[3];
  long stride[3];
  long rowlen[3], ldo[3];
  int bend[3];
  int nseg;
};

// V = floats per thread (4: 16-B loads; needs n, stride and pointers 16-B aligned)
template <int PL, int V>
__global__ void __launch_bounds__(256) colsum_kernel(ColSegs sg, int nparts, int accumulate) {
  constexpr int NC = 256 / PL;
  typedef float vec __attribute__((ext_vector_type(V)));
  __shared__ vec red[PL][NC + (V == 1 ? 1 : 0)];
  int seg = 0;
  if (sg.nseg > 1 && (int)blockIdx.x >= sg.bend[0]) seg = (sg.nseg > 2 && (int)blockIdx.x >= sg.bend[1]) ? 2 : 1;
  const float* __restrict__ part = sg.part[seg];
  float* __restrict__ out = sg.out[seg];
  const long n = sg.n[seg], stride = sg.stride[seg];
  const int b0 = seg == 0 ? 0 : sg.bend[seg - 1];
  const int lx = threadIdx.x % NC, ly = threadIdx.x / NC;
  const long i = ((long)((int)blockIdx.x - b0) * NC + lx) * V;
  vec s = {};
  if (i < n) {
    int p = ly;
    for (; p + 7 * PL < nparts; p += 8 * PL) {
      vec v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const vec*>(part + (long)(p + u * PL) * stride + i);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; p < nparts; p += PL) s += *reinterpret_cast<const vec*>(part + (long)p * stride + i);
  }
  red[ly][lx] = s;
  __syncthreads();
  if (ly == 0 && i < n) {
    vec t = red[0][lx];
#pragma unroll
    for (int k = 1; k < PL; ++k) t += red[k][lx];
    const long rl = sg.rowlen[seg];
    const long oi = rl == n ? i : (i / rl) * sg.ldo[seg] + (i - (i / rl) * rl);
    vec* o = reinterpret_cast<vec*>(out + oi);
    *o = accumulate ? *o + t : t;
  }
}

// segs: {part, n, stride, out[, rowlen, ldo]} x nseg (nseg <= 3), all over nparts parts
struct ColSeg {
  const float* part;
  long n;
  long stride;
  float* out;
  long rowlen = 0;  // 0: contiguous output
  long ldo = 0;
};

inline void colsum_multi(const ColSeg* segs, int nseg, int nparts, int accumulate, hipStream_t st) {
  bool v4 = true;
  long total = 0;
  for (int j = 0; j < nseg; ++j) {
    const long rl = segs[j].rowlen > 0 ? segs[j].rowlen : segs[j].n;
    const long lo = segs[j].rowlen > 0 ? segs[j].ldo : segs[j].n;
    v4 = v4 && segs[j].n % 4 == 0 && segs[j].stride % 4 == 0 && rl % 4 == 0 && lo % 4 == 0 &&
         ((uintptr_t)segs[j].part & 15) == 0 && ((uintptr_t)segs[j].out & 15) == 0;
    total += segs[j].n;
  }
  const int V = v4 ? 4 : 1;
  // narrow reductions (LayerNorm affine, biases: ~1000 parts) want many part-lanes in flight:
  // with 128 part-lanes a 1024-part reduction is one round of 8 loads per thread
  const int PL = total / V <= 256 ? 128 : (total / V <= 1024 ? 32 : 8);
  const int NC = 256 / PL;
  ColSegs sg{};
  int blocks = 0;
  for (int j = 0; j < nseg; ++j) {
    sg.part[j] = segs[j].part;
    sg.out[j] = segs[j].out;
    sg.n[j] = segs[j].n;
    sg.stride[j] = segs[j].stride;
    sg.rowlen[j] = segs[j].rowlen > 0 ? segs[j].rowlen : segs[j].n;
    sg.ldo[j] = segs[j].rowlen > 0 ? segs[j].ldo : segs[j].n;
    blocks += (int)((segs[j].n / V + NC - 1) / NC);
    sg.bend[j] = blocks;
  }
  sg.nseg = nseg;
  if (blocks == 0) return;
  if (V == 4) {
    if (PL == 128) hipLaunchKernelGGL((colsum_kernel<128, 4>), dim3(blocks), dim3(256), 0, st, sg, nparts, accumulate);
    else if (PL == 32) hipLaunchKernelGGL((colsum_kernel<32, 4>), dim3(blocks), dim3(256), 0, st, sg, nparts, accumulate);
    else hipLaunchKernelGGL((colsum_kernel<8, 4>), dim3(blocks), dim3(256), 0, st, sg, nparts, accumulate);
  } else {
    if (PL == 128) hipLaunchKernelGGL((colsum_kernel<128, 1>), dim3(blocks), dim3(256), 0, st, sg, nparts, accumulate);
    else if (PL == 32) hipLaunchKernelGGL((colsum_kernel<32, 1>), dim3(blocks), dim3(256), 0, st, sg, nparts, accumulate);
    else hipLaunchKernelGGL((colsum_kernel<8, 1>), dim3(blocks), dim3(256), 0, st, sg, nparts, accumulate);
  }
}

inline void colsum(const float* part, int nparts, long n, long stride, float* out, int accumulate,
                   hipStream_t st) {
  const ColSeg s{part, n, stride, out};
  colsum_multi(&s, 1, nparts, accumulate, st);
}

}  // namespace
