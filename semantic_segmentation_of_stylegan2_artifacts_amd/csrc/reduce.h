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
#include <mutex>

#include "common.h"

// in-kernel tail reductions on (1, default) / off (0: colsum launches); msu_tail_reduce_mode
extern int g_msu_tail_on;

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
__global__ void __launch_bounds__(256) colsum_kernel(ColSegs sg, int nparts, int accmask) {
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
    *o = (accmask >> seg) & 1 ? *o + t : t;  // bit j: segment j adds to its output
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

// accumulate != 0: every segment adds to its output; acc_mask >= 0 instead picks them (bit j: segment j)
inline void colsum_multi(const ColSeg* segs, int nseg, int nparts, int accumulate, hipStream_t st,
                         int acc_mask = -1) {
  const int accmask = acc_mask >= 0 ? acc_mask : (accumulate ? 7 : 0);
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
    if (PL == 128) hipLaunchKernelGGL((colsum_kernel<128, 4>), dim3(blocks), dim3(256), 0, st, sg, nparts, accmask);
    else if (PL == 32) hipLaunchKernelGGL((colsum_kernel<32, 4>), dim3(blocks), dim3(256), 0, st, sg, nparts, accmask);
    else hipLaunchKernelGGL((colsum_kernel<8, 4>), dim3(blocks), dim3(256), 0, st, sg, nparts, accmask);
  } else {
    if (PL == 128) hipLaunchKernelGGL((colsum_kernel<128, 1>), dim3(blocks), dim3(256), 0, st, sg, nparts, accmask);
    else if (PL == 32) hipLaunchKernelGGL((colsum_kernel<32, 1>), dim3(blocks), dim3(256), 0, st, sg, nparts, accmask);
    else hipLaunchKernelGGL((colsum_kernel<8, 1>), dim3(blocks), dim3(256), 0, st, sg, nparts, accmask);
  }
}

inline void colsum(const float* part, int nparts, long n, long stride, float* out, int accumulate,
                   hipStream_t st) {
  const ColSeg s{part, n, stride, out};
  colsum_multi(&s, 1, nparts, accumulate, st);
}

// ------------------------------------------------------------------ batched reductions
// Many independent partial-row reductions in one launch (deferred LayerNorm parameter
// gradients: a stage's worth of LayerNorm backwards hand over their [nparts][2C] partials instead
// of each summing them in its own tail): segment j sums part_j[q * stride_j + i] over q in
// [0, nparts_j) for i < n_j into out_j (+= with accumulate), in a fixed order (deterministic).
// Block = 32 part-lanes x 8 float4 column lanes (32 columns).
constexpr int CB_MAX = 48, CB_PL = 32, CB_NC = 8;
struct ColBatch {
  const float* part[CB_MAX];
  float* out[CB_MAX];
  long stride[CB_MAX];
  int n[CB_MAX];
  int nparts[CB_MAX];
  int bend[CB_MAX];  // prefix sums of the segments' block counts
  int nseg;
  int accumulate;
};

__global__ void __launch_bounds__(256) colsum_batch_kernel(ColBatch cb) {
  int seg = 0;
  while (seg + 1 < cb.nseg && (int)blockIdx.x >= cb.bend[seg]) ++seg;
  const int b0 = seg == 0 ? 0 : cb.bend[seg - 1];
  const float* __restrict__ part = cb.part[seg];
  const long stride = cb.stride[seg];
  const int n = cb.n[seg], np = cb.nparts[seg];
  const int lx = threadIdx.x % CB_NC, ly = threadIdx.x / CB_NC;
  const int i = (((int)blockIdx.x - b0) * CB_NC + lx) * 4;
  float4 s = {0.f, 0.f, 0.f, 0.f};
  if (i < n) {
    int q = ly;
    for (; q + 3 * CB_PL < np; q += 4 * CB_PL) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(part + (long)(q + u * CB_PL) * stride + i);
#pragma unroll
      for (int u = 0; u < 4; ++u) { s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w; }
    }
    for (; q < np; q += CB_PL) {
      const float4 v = *reinterpret_cast<const float4*>(part + (long)q * stride + i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  __shared__ float4 red[CB_PL][CB_NC];
  red[ly][lx] = s;
  __syncthreads();
  if (ly == 0 && i < n) {
    float4 t = red[0][lx];
#pragma unroll
    for (int k = 1; k < CB_PL; ++k) { t.x += red[k][lx].x; t.y += red[k][lx].y; t.z += red[k][lx].z; t.w += red[k][lx].w; }
    float4* o = reinterpret_cast<float4*>(cb.out[seg] + i);
    if (cb.accumulate) { const float4 v = *o; t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w; }
    *o = t;
  }
}

// ------------------------------------------------------------------ in-kernel tail reduction
// The partial rows a kernel's blocks write, summed by the kernel itself instead of a colsum
// launch.  A colsum launch queued behind the other stream's kernels waited for free CUs: the
// LayerNorm parameter reductions took 15-43 us each on the main stream in the step for ~5 us of
// work, the weight-gradient slab reductions up to 1 ms on the side stream (r05a profile).
// Two levels, in a fixed order (deterministic, whatever the arrival order): part rows form groups
// of TAIL_GS consecutive indices; the block drawing the last ticket of its group sums the group's
// rows in index order into the group's first row; the block finishing the last group sums those
// rows in group order and emits the result.
// Hand-off (cdna_hip_programming.md "In-launch split-K reduction", its write-through form): the
// partial rows are stored write-through (sc1: tail_st), every wave drains its stores (vmcnt(0)),
// barrier, lane 0 draws a relaxed agent-scope ticket; the last arriver: lane 0 agent-scope acquire
// + vmcnt(0), barrier, plain loads.  (An agent-scope release fence in every block instead wrote
// back the whole L2 -- the kernel's dx too -- per block: the step ran 2.7 % slower, r05h.)
// Counters: one region per stream (launches on one stream never overlap; a captured graph keeps
// the regions of its capture streams), zero at load and left zero by every launch: the block
// drawing a counter's last ticket resets it.
constexpr int TAIL_GS = 32, TAIL_SLOTS = 64, TAIL_WORDS = 2048;
__device__ int g_tail_cnt[TAIL_SLOTS * TAIL_WORDS];

// the counter region of stream st (-1: every region taken; the caller falls back to colsum)
inline int tail_slot(hipStream_t st) {
  static std::mutex mu;
  static hipStream_t owner[TAIL_SLOTS];
  static int used = 0;
  if (!g_msu_tail_on) return -1;
  std::lock_guard<std::mutex> lk(mu);
  for (int i = 0; i < used; ++i)
    if (owner[i] == st) return i;
  if (used == TAIL_SLOTS) return -1;
  owner[used] = st;
  return used++;
}

// write-through store of a partial-row value (4 B per lane: the natural width of these writers)
MSU_DEV void tail_st(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
MSU_DEV void tail_st4(float* p, float4 v) {
  tail_st(p, v.x);
  tail_st(p + 1, v.y);
  tail_st(p + 2, v.z);
  tail_st(p + 3, v.w);
}

// true (in every thread) in the block that drew the last of `total` tickets at *cnt, after the
// acquire; the block's partial rows stored by tail_st; flag: one int of the kernel's LDS
// (kernels staging by LDS-DMA keep one LDS array)
MSU_DEV bool tail_ticket(int* cnt, int total, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == total - 1;
    if (last) {
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every ticket drawn
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// Sum rows part[q * stride + i] (i < n) over q in [0, nparts), this block having written row p
// (by tail_st): emit(i, float4) receives columns i .. i + 3 of the total in the block that
// finishes it.  n % 4 == 0, stride % 4 == 0, part 16-B aligned; groups of gs rows; cnt: the
// ceil(nparts / gs) + 1 counters of this reduction (in g_tail_cnt + slot * TAIL_WORDS).
template <typename Emit>
MSU_DEV void tail_reduce(float* part, int p, int nparts, int n, long stride, int* cnt, int* flag, Emit&& emit,
                         int gs = TAIL_GS) {
  const int g = p / gs, ng = (nparts + gs - 1) / gs;
  const int q0 = g * gs, q1 = min(nparts, q0 + gs);
  if (!tail_ticket(cnt + g, q1 - q0, flag)) return;
  for (int i = 4 * (int)threadIdx.x; i < n; i += 4 * (int)blockDim.x) {
    const float* r = part + (long)q0 * stride + i;
    float4 s = *reinterpret_cast<const float4*>(r);
#pragma unroll 8
    for (int q = 1; q < q1 - q0; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(r + (long)q * stride);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    if (ng == 1) emit(i, s);
    else tail_st4(part + (long)q0 * stride + i, s);
  }
  if (ng == 1 || !tail_ticket(cnt + ng, ng, flag)) return;
  for (int i = 4 * (int)threadIdx.x; i < n; i += 4 * (int)blockDim.x) {
    const float* r = part + i;
    float4 s = *reinterpret_cast<const float4*>(r);
#pragma unroll 8
    for (int h = 1; h < ng; ++h) {
      const float4 v = *reinterpret_cast<const float4*>(r + (long)h * gs * stride);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    emit(i, s);
  }
}

MSU_DEV void acc_store4(float* o, float4 s, int accumulate) {
  if (accumulate) {
    const float4 v = *reinterpret_cast<const float4*>(o);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  *reinterpret_cast<float4*>(o) = s;
}

}  // namespace
