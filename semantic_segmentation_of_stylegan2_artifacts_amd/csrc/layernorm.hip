// Row LayerNorm family (eps, per-row f32 mean/rstd saved for backward) with fused input
// addressing.  Replaces every nn.LayerNorm on the MS-UNet path:
//   * plain            block norm1/norm2, PatchEmbed.norm, norm, norm_up
//                      (model_parts.py:213,224,740-741; torchvision block)
//   * residual add     x + dp[b]*branch -> LN (torchvision block residual + StochasticDepth,
//                      fused with the following norm)
//   * 2x2 merge gather PatchMerging x0..x3 cat + norm (model_parts.py:87-94)
//   * 2x2 d2s          PatchExpand rearrange + norm (model_parts.py:403-405)
//   * head             FinalPatchExpand_X4_V2.norm + 1x1 output conv (model_parts.py:475,846)
// One row is owned by TPR lanes; each lane holds KMAX 4-wide chunks in registers.
#include <stdlib.h>

#include "common.h"
#include "reduce.h"

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace {

enum InMode { IN_PLAIN = 0, IN_ADD = 1, IN_MERGE = 2, IN_D2S2 = 3 };

// 16-byte row chunks: 4 f32 or 8 16-bit elements per lane access
template <typename T> struct VecW;
template <> struct VecW<float> {
  static constexpr int W = 4;
  static MSU_DEV void load(const float* p, float (&v)[4]) { Vec4<float>::load(p, v); }
  static MSU_DEV void store(float* p, const float (&v)[4]) { Vec4<float>::store(p, v); }
};
template <typename T> struct VecW16 {
  static constexpr int W = 8;
  static MSU_DEV void load(const T* p, float (&v)[8]) {
    const uint4 q = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = Fmt16<T>::lo(w[i]);
      v[2 * i + 1] = Fmt16<T>::hi(w[i]);
    }
  }
  static MSU_DEV void store(T* p, const float (&v)[8]) {
    uint4 q;
    q.x = pack2<T>(v[0], v[1]);
    q.y = pack2<T>(v[2], v[3]);
    q.z = pack2<T>(v[4], v[5]);
    q.w = pack2<T>(v[6], v[7]);
    *reinterpret_cast<uint4*>(p) = q;
  }
};
template <> struct VecW<bf16_t> : VecW16<bf16_t> {};
template <> struct VecW<f16_t> : VecW16<f16_t> {};
template <int VW> MSU_DEV void load_f32(const float* p, float (&v)[VW]) {
#pragma unroll
  for (int i = 0; i < VW; i += 4) {
    const float4 q = *reinterpret_cast<const float4*>(p + i);
    v[i] = q.x; v[i + 1] = q.y; v[i + 2] = q.z; v[i + 3] = q.w;
  }
}

struct LnArgs {
  const void* x;      // IN_PLAIN/MERGE/D2S2: source; IN_ADD: residual stream a
  const void* b;      // IN_ADD: branch output (may be null)
  const float* bscale;  // IN_ADD: per-sample stochastic-depth scale (null = 1)
  void* s_out;        // IN_ADD: a + scale*b (null = not stored)
  const float* gamma;
  const float* beta;
  void* y;
  float* mean;
  float* rstd;
  long rows;
  int C;              // normalised width (row length of y)
  int H, W;           // MERGE: input grid; D2S2: input grid (output grid is 2H x 2W)
  int Cin;            // MERGE: input channels (C = 4*Cin)
  long rows_per_sample;
  float eps;
};

// element offset of column `col` of logical row `r` in the source tensor
template <int MODE>
MSU_DEV long src_off(const LnArgs& a, long r, int col) {
  if constexpr (MODE == IN_MERGE) {
    const int H2 = a.H >> 1, W2 = a.W >> 1;
    const long b = r / ((long)H2 * W2);
    const int rem = (int)(r - b * (long)H2 * W2);
    const int i = rem / W2, j = rem - (rem / W2) * W2;
    const int q = col / a.Cin, off = col - q * a.Cin;
    const int dy = q & 1, dx = q >> 1;  // x0 (0,0) x1 (1,0) x2 (0,1) x3 (1,1)
    return (((b * a.H + 2 * i + dy) * a.W) + 2 * j + dx) * (long)a.Cin + off;
  } else if constexpr (MODE == IN_D2S2) {
    const int OH = a.H * 2, OW = a.W * 2;
    const long b = r / ((long)OH * OW);
    const int rem = (int)(r - b * (long)OH * OW);
    const int oh = rem / OW, ow = rem - (rem / OW) * OW;
    const long tok = (b * a.H + (oh >> 1)) * a.W + (ow >> 1);
    return tok * (4L * a.C) + (long)(((oh & 1) * 2 + (ow & 1)) * a.C) + col;
  } else {
    return r * (long)a.C + col;
  }
}

template <typename T>
MSU_DEV void unpack16(const uint4 q, float (&v)[8]) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = Fmt16<T>::lo(w[i]);
    v[2 * i + 1] = Fmt16<T>::hi(w[i]);
  }
}

template <typename T, int MODE, int TPR, int KMAX, bool PFF = true>
__global__ void __launch_bounds__(256) ln_fwd_kernel(LnArgs a) {
  constexpr int VW = VecW<T>::W;  // elements per 16-B chunk
  const int lane = threadIdx.x % TPR;
  const int grp = threadIdx.x / TPR;
  constexpr int GPB = 256 / TPR;
  const int nchunk = a.C / VW;
  const T* X = reinterpret_cast<const T*>(a.x);
  const T* Bv = reinterpret_cast<const T*>(a.b);
  // 16-bit rows of one chunk per lane: the group's next row is loaded while this one is
  // normalised (same arithmetic as the plain loop below; see ln_bwd_kernel)
  if constexpr (KMAX == 1 && VW == 8 && PFF) {
    const int ch = lane;
    const bool act = ch < nchunk;
    float g[VW], bt[VW];
    if (act) {
      load_f32<VW>(a.gamma + ch * VW, g);
      load_f32<VW>(a.beta + ch * VW, bt);
    }
    const long stride = (long)gridDim.x * GPB;
    long r = (long)blockIdx.x * GPB + grp;
    uint4 qx{}, qb{};
    float qsc = 1.f;
    auto fetch = [&](long rr) __attribute__((always_inline)) {
      if constexpr (MODE == IN_ADD) {
        if (a.bscale) qsc = a.bscale[rr / a.rows_per_sample];
      }
      if (act) {
        const long off = src_off<MODE>(a, rr, ch * VW);
        qx = *reinterpret_cast<const uint4*>(X + off);
        if constexpr (MODE == IN_ADD) {
          if (Bv) qb = *reinterpret_cast<const uint4*>(Bv + off);
        }
      }
    };
    if (r < a.rows) fetch(r);
    for (; r < a.rows; r += stride) {
      const uint4 cx = qx, cb = qb;
      const float sc = qsc;
      if (r + stride < a.rows) fetch(r + stride);
      float v[VW];
      float sum = 0.f;
      if (act) {
        unpack16<T>(cx, v);
        if constexpr (MODE == IN_ADD) {
          if (Bv) {
            float w[VW];
            unpack16<T>(cb, w);
#pragma unroll
            for (int e = 0; e < VW; ++e) v[e] += sc * w[e];
          }
#pragma unroll
          for (int e = 0; e < VW; ++e) v[e] = to_f32(from_f32<T>(v[e]));
          if (a.s_out) VecW<T>::store(reinterpret_cast<T*>(a.s_out) + src_off<MODE>(a, r, ch * VW), v);
        }
#pragma unroll
        for (int e = 0; e < VW; ++e) sum += v[e];
      }
      sum = group_sum<TPR>(sum);
      const float mu = sum / a.C;
      float var = 0.f;
      if (act) {
#pragma unroll
        for (int e = 0; e < VW; ++e) { const float d = v[e] - mu; var += d * d; }
      }
      var = group_sum<TPR>(var);
      const float rs = rsqrtf(var / a.C + a.eps);
      if (act) {
        float o[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) o[e] = (v[e] - mu) * rs * g[e] + bt[e];
        VecW<T>::store(reinterpret_cast<T*>(a.y) + r * (long)a.C + ch * VW, o);
      }
      if (lane == 0) { a.mean[r] = mu; a.rstd[r] = rs; }
    }
  } else
  for (long r = (long)blockIdx.x * GPB + grp; r < a.rows; r += (long)gridDim.x * GPB) {
    float v[KMAX][VW];
    float sum = 0.f;
    float sc = 1.f;
    if constexpr (MODE == IN_ADD) {
      if (a.bscale) sc = a.bscale[r / a.rows_per_sample];
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        const long off = src_off<MODE>(a, r, ch * VW);
        VecW<T>::load(X + off, v[k]);
        if constexpr (MODE == IN_ADD) {
          if (Bv) {
            float w[VW];
            VecW<T>::load(Bv + off, w);
#pragma unroll
            for (int e = 0; e < VW; ++e) v[k][e] += sc * w[e];
          }
          // round the residual stream to storage precision first: the stored value is
          // what later layers (and backward) see, so normalise exactly that value
#pragma unroll
          for (int e = 0; e < VW; ++e) v[k][e] = to_f32(from_f32<T>(v[k][e]));
          if (a.s_out) VecW<T>::store(reinterpret_cast<T*>(a.s_out) + off, v[k]);
        }
#pragma unroll
        for (int e = 0; e < VW; ++e) sum += v[k][e];
      }
    }
    sum = group_sum<TPR>(sum);
    const float mu = sum / a.C;
    float var = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
#pragma unroll
        for (int e = 0; e < VW; ++e) { const float d = v[k][e] - mu; var += d * d; }
      }
    }
    var = group_sum<TPR>(var);
    const float rs = rsqrtf(var / a.C + a.eps);
    T* Y = reinterpret_cast<T*>(a.y);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        float o[VW], g[VW], bt[VW];
        load_f32<VW>(a.gamma + ch * VW, g);
        load_f32<VW>(a.beta + ch * VW, bt);
#pragma unroll
        for (int e = 0; e < VW; ++e) o[e] = (v[k][e] - mu) * rs * g[e] + bt[e];
        VecW<T>::store(Y + r * (long)a.C + ch * VW, o);
      }
    }
    if (lane == 0) { a.mean[r] = mu; a.rstd[r] = rs; }
  }
}

struct LnBwdArgs {
  const void* dy;       // [rows, C]
  const void* x;        // the normalised input (IN_ADD: the stored s; others: source)
  const void* dres;     // extra gradient into s (IN_ADD / IN_PLAIN; null = none)
  const float* gamma;
  const float* mean;
  const float* rstd;
  void* dx;             // gradient wrt the normalised input (scattered for MERGE / D2S2)
  void* db;             // IN_ADD: gradient wrt branch = dx * bscale (null = not needed)
  const float* bscale;
  float* part;          // [gridDim.x, 2, C] partial dgamma / dbeta
  long rows;
  int C, H, W, Cin;
  long rows_per_sample;
  // the partials summed in the kernel (reduce.h tail_reduce) into dgamma / dbeta (+= when
  // accumulate): the counter region of the launch stream, or -1 (a colsum launch after it)
  int tail = -1;
  int accumulate = 0;
  float* dgamma = nullptr;
  float* dbeta = nullptr;
  // more extra gradients into s, summed with dres in f32 before the one rounding (only with
  // dres; the skip-gradient handoff: a stage input's other readers)
  const void* dres2 = nullptr;
  const void* dres3 = nullptr;
};

template <typename T, int MODE, int TPR, int KMAX, bool PFB = true>
__global__ void __launch_bounds__(256) ln_bwd_kernel(LnBwdArgs a) {
  // no implicit contraction: the two row loops below (prefetching / plain) fuse exactly the
  // multiply-adds written as fmaf, so they agree bitwise (tools/ln_pf_check.py)
#pragma clang fp contract(off)
  constexpr int VW = VecW<T>::W;  // elements per 16-B chunk
  const int lane = threadIdx.x % TPR;
  const int grp = threadIdx.x / TPR;
  constexpr int GPB = 256 / TPR;
  const int nchunk = a.C / VW;
  const T* X = reinterpret_cast<const T*>(a.x);
  const T* DY = reinterpret_cast<const T*>(a.dy);
  float accg[KMAX][VW], accb[KMAX][VW];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int e = 0; e < VW; ++e) { accg[k][e] = 0.f; accb[k][e] = 0.f; }
  LnArgs fa;
  fa.C = a.C; fa.H = a.H; fa.W = a.W; fa.Cin = a.Cin;
  constexpr bool HAS_RES = MODE == IN_ADD || MODE == IN_PLAIN;
  // 16-bit rows of one chunk per lane (every C <= 512 of the path): the group's next row is
  // loaded while this one is reduced and stored, so a group waits one memory round trip per
  // row only where the prefetch has not landed (the arithmetic, and so the result, is the
  // plain loop's below).  A/B switch: the plain loop, template-selected by launch_bwd
  if constexpr (KMAX == 1 && VW == 8 && PFB) {
    const int ch = lane;
    const bool act = ch < nchunk;
    float gg[VW];
    if (act) load_f32<VW>(a.gamma + ch * VW, gg);
    const long stride = (long)gridDim.x * GPB;
    long r = (long)blockIdx.x * GPB + grp;
    struct RowSet {
      uint4 x{}, d{}, r{}, r2{}, r3{};
      float mu = 0.f, rs = 0.f;
    };
    auto fetch = [&](RowSet& q, long rr) __attribute__((always_inline)) {
      q.mu = a.mean[rr];
      q.rs = a.rstd[rr];
      if (act) {
        const long off = src_off<MODE>(fa, rr, ch * VW);
        q.x = *reinterpret_cast<const uint4*>(X + off);
        q.d = *reinterpret_cast<const uint4*>(DY + rr * (long)a.C + ch * VW);
        if constexpr (HAS_RES) {
          if (a.dres) q.r = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.dres) + off);
          if (a.dres2) q.r2 = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.dres2) + off);
          if (a.dres3) q.r3 = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.dres3) + off);
        }
      }
    };
    auto work = [&](const RowSet& c, long r) __attribute__((always_inline)) {
      float xh[VW], g[VW];
      float s1 = 0.f, s2 = 0.f;
      if (act) {
        float xv[VW], dv[VW];
        unpack16<T>(c.x, xv);
        unpack16<T>(c.d, dv);
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          xh[e] = (xv[e] - c.mu) * c.rs;
          g[e] = dv[e] * gg[e];
          s1 += g[e];
          s2 = __builtin_fmaf(g[e], xh[e], s2);
          accg[0][e] = __builtin_fmaf(dv[e], xh[e], accg[0][e]);
          accb[0][e] += dv[e];
        }
      }
      s1 = group_sum<TPR>(s1) / a.C;
      s2 = group_sum<TPR>(s2) / a.C;
      float sc = 1.f;
      if constexpr (MODE == IN_ADD) {
        if (a.bscale) sc = a.bscale[r / a.rows_per_sample];
      }
      if (act) {
        float o[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) o[e] = __builtin_fmaf(-xh[e], s2, g[e] - s1);
        const long off = src_off<MODE>(fa, r, ch * VW);
        bool res = false;
        if constexpr (HAS_RES) res = a.dres != nullptr;
        if (res) {
          float dr[VW];
          unpack16<T>(c.r, dr);
#pragma unroll
          for (int e = 0; e < VW; ++e) o[e] = __builtin_fmaf(c.rs, o[e], dr[e]);
          if (a.dres2) {
            unpack16<T>(c.r2, dr);
#pragma unroll
            for (int e = 0; e < VW; ++e) o[e] += dr[e];
          }
          if (a.dres3) {
            unpack16<T>(c.r3, dr);
#pragma unroll
            for (int e = 0; e < VW; ++e) o[e] += dr[e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < VW; ++e) o[e] *= c.rs;
        }
        VecW<T>::store(reinterpret_cast<T*>(a.dx) + off, o);
        if constexpr (MODE == IN_ADD) {
          if (a.db) {
#pragma unroll
            for (int e = 0; e < VW; ++e) o[e] *= sc;
            VecW<T>::store(reinterpret_cast<T*>(a.db) + off, o);
          }
        }
      }
    };
    if constexpr ((MSU_EXP & 256) != 0) {
      // ablation: two rows ahead (two register sets, the loop unrolled by two)
      RowSet q0, q1;
      if (r < a.rows) fetch(q0, r);
      if (r + stride < a.rows) fetch(q1, r + stride);
      for (; r < a.rows; r += 2 * stride) {
        work(q0, r);
        if (r + 2 * stride < a.rows) fetch(q0, r + 2 * stride);
        if (r + stride >= a.rows) break;
        work(q1, r + stride);
        if (r + 3 * stride < a.rows) fetch(q1, r + 3 * stride);
      }
    } else {
      RowSet nxt;
      if (r < a.rows) fetch(nxt, r);
      for (; r < a.rows; r += stride) {
        const RowSet cur = nxt;
        if (r + stride < a.rows) fetch(nxt, r + stride);
        work(cur, r);
      }
    }
  } else
  for (long r = (long)blockIdx.x * GPB + grp; r < a.rows; r += (long)gridDim.x * GPB) {
    const float mu = a.mean[r], rs = a.rstd[r];
    float xh[KMAX][VW], g[KMAX][VW];
    // the residual gradient is loaded with x and dy: one memory round trip per row, not two
    float dr[KMAX][VW];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        float xv[VW], dv[VW], gg[VW];
        const long off = src_off<MODE>(fa, r, ch * VW);
        VecW<T>::load(X + off, xv);
        VecW<T>::load(DY + r * (long)a.C + ch * VW, dv);
        if constexpr (HAS_RES) {
          if (a.dres) VecW<T>::load(reinterpret_cast<const T*>(a.dres) + off, dr[k]);
        }
        load_f32<VW>(a.gamma + ch * VW, gg);
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          xh[k][e] = (xv[e] - mu) * rs;
          g[k][e] = dv[e] * gg[e];
          s1 += g[k][e];
          s2 = __builtin_fmaf(g[k][e], xh[k][e], s2);
          accg[k][e] = __builtin_fmaf(dv[e], xh[k][e], accg[k][e]);
          accb[k][e] += dv[e];
        }
      }
    }
    s1 = group_sum<TPR>(s1) / a.C;
    s2 = group_sum<TPR>(s2) / a.C;
    float sc = 1.f;
    if constexpr (MODE == IN_ADD) {
      if (a.bscale) sc = a.bscale[r / a.rows_per_sample];
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        float o[VW];
#pragma unroll
        for (int e = 0; e < VW; ++e) o[e] = __builtin_fmaf(-xh[k][e], s2, g[k][e] - s1);
        const long off = src_off<MODE>(fa, r, ch * VW);
        bool res = false;
        if constexpr (HAS_RES) res = a.dres != nullptr;
        if (res) {
#pragma unroll
          for (int e = 0; e < VW; ++e) o[e] = __builtin_fmaf(rs, o[e], dr[k][e]);
          const void* more[2] = {a.dres2, a.dres3};
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            if (more[q]) {
              float d2[VW];
              VecW<T>::load(reinterpret_cast<const T*>(more[q]) + off, d2);
#pragma unroll
              for (int e = 0; e < VW; ++e) o[e] += d2[e];
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < VW; ++e) o[e] *= rs;
        }
        VecW<T>::store(reinterpret_cast<T*>(a.dx) + off, o);
        if constexpr (MODE == IN_ADD) {
          if (a.db) {
#pragma unroll
            for (int e = 0; e < VW; ++e) o[e] *= sc;
            VecW<T>::store(reinterpret_cast<T*>(a.db) + off, o);
          }
        }
      }
    }
  }
  // parameter-gradient partials: the row groups of a wave hold the same columns in the
  // same lanes -> fixed xor-shuffle tree over the groups, then the 4 waves' rows are summed
  // through LDS in a fixed order (deterministic)
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int e = 0; e < VW; ++e)
#pragma unroll
      for (int o = TPR; o < 64; o <<= 1) {
        accg[k][e] += __shfl_xor(accg[k][e], o, 64);
        accb[k][e] += __shfl_xor(accb[k][e], o, 64);
      }
  __shared__ float red[2][4][TPR * KMAX * VW];  // [g/b][wave][column]
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < TPR) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
#pragma unroll
        for (int e = 0; e < VW; ++e) {
          red[0][wave][ch * VW + e] = accg[k][e];
          red[1][wave][ch * VW + e] = accb[k][e];
        }
      }
    }
  }
  __syncthreads();
  float* P = a.part + (long)blockIdx.x * 2 * a.C;
  for (int i = threadIdx.x; i < a.C; i += 256) {
    tail_st(P + i, ((red[0][0][i] + red[0][1][i]) + red[0][2][i]) + red[0][3][i]);
    tail_st(P + a.C + i, ((red[1][0][i] + red[1][1][i]) + red[1][2][i]) + red[1][3][i]);
  }
  if (a.tail >= 0) {
    __shared__ int tail_flag;
    tail_reduce(a.part, blockIdx.x, gridDim.x, 2 * a.C, 2L * a.C, g_tail_cnt + a.tail * TAIL_WORDS, &tail_flag,
                [&](int i, float4 v) {
                  acc_store4(i < a.C ? a.dgamma + i : a.dbeta + (i - a.C), v, a.accumulate);
                });
  }
}

template <typename T, int MODE>
int launch_fwd(const LnArgs& a, hipStream_t st, int max_blocks) {
  const int nchunk = a.C / VecW<T>::W;
  auto go = [&](auto kern, int tpr) {
    const long gpb = 256 / tpr;
    long nb = (a.rows + gpb - 1) / gpb;
    if (nb > max_blocks) nb = max_blocks;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(256), 0, st, a);
    return MSU_CHECK_LAUNCH();
  };
  // rows of <= 64 chunks (C <= 512 bf16) read by 16 / 32 / 64 lanes (one 16-B chunk per lane,
  // whole rows per load instruction) instead of 4 lanes x 4 chunks: bench 153.5 vs 152.8 img/s
  // up to C = 128, +0.25 % more up to C = 512 (r01, 3 of 3 pairs); the next row of a group
  // prefetched (r04y: +0.2 %)
  if (nchunk <= 16) return go(ln_fwd_kernel<T, MODE, 16, 1>, 16);
  if constexpr ((MSU_EXP & 8) != 0) {  // ablation: C = 192 rows as 8 lanes x 3 chunks
    if (nchunk <= 24 && nchunk > 16) return go(ln_fwd_kernel<T, MODE, 8, 3>, 8);
  }
  if (nchunk <= 32) return go(ln_fwd_kernel<T, MODE, 32, 1>, 32);
  if (nchunk <= 64) return go(ln_fwd_kernel<T, MODE, 64, 1>, 64);
  if (nchunk <= 4 * 4) return go(ln_fwd_kernel<T, MODE, 4, 4>, 4);
  if (nchunk <= 8 * 4) return go(ln_fwd_kernel<T, MODE, 8, 4>, 8);
  if (nchunk <= 16 * 4) return go(ln_fwd_kernel<T, MODE, 16, 4>, 16);
  if (nchunk <= 32 * 4) return go(ln_fwd_kernel<T, MODE, 32, 4>, 32);
  if (nchunk <= 64 * 4) return go(ln_fwd_kernel<T, MODE, 64, 4>, 64);
  if (nchunk <= 64 * 8) return go(ln_fwd_kernel<T, MODE, 64, 8>, 64);
  return -2;
}

template <typename T, int MODE>
int launch_bwd(const LnBwdArgs& a, hipStream_t st, int nblocks) {
  const int nchunk = a.C / VecW<T>::W;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nblocks), dim3(256), 0, st, a);
    return MSU_CHECK_LAUNCH();
  };
  // one chunk per lane up to C = 512 (see launch_fwd), next row prefetched (r04x: +0.45 %)
  if (nchunk <= 16) return go(ln_bwd_kernel<T, MODE, 16, 1>);
  if (nchunk <= 32) return go(ln_bwd_kernel<T, MODE, 32, 1>);
  if (nchunk <= 64) return go(ln_bwd_kernel<T, MODE, 64, 1>);
  if (nchunk <= 4 * 3) return go(ln_bwd_kernel<T, MODE, 4, 3>);  // C = 96 bf16: no idle slot
  if (nchunk <= 4 * 4) return go(ln_bwd_kernel<T, MODE, 4, 4>);
  if (nchunk <= 8 * 4) return go(ln_bwd_kernel<T, MODE, 8, 4>);
  if (nchunk <= 16 * 4) return go(ln_bwd_kernel<T, MODE, 16, 4>);
  if (nchunk <= 32 * 4) return go(ln_bwd_kernel<T, MODE, 32, 4>);
  if (nchunk <= 64 * 4) return go(ln_bwd_kernel<T, MODE, 64, 4>);
  if (nchunk <= 64 * 8) return go(ln_bwd_kernel<T, MODE, 64, 8>);
  return -2;
}

template <int MODE>
int fwd_dispatch(int dtype, const LnArgs& a, hipStream_t st) {
  if (a.C % (msu_is16(dtype) ? 8 : 4) != 0 || a.C > 2048) return -2;
  if (a.rows == 0) return 0;
  // grid cap 4096 blocks: with the next row prefetched (r04y) a group needs several rows to
  // overlap loads with the normalisation; at 16384 the C >= 192 launches ran one row per group
  // (r05af alone: 131072 x 192 add-LN 43.3 vs 51.5 us, 32768 x 384 22.9 vs 25.0; step 172.3 vs
  // 171.8 img/s, 3 of 3 pairs, r05ag; r01, before the prefetch, had 16384 ahead of 4096)
  constexpr int cap = (MSU_EXP & 16) ? 2048 : ((MSU_EXP & 64) ? 1024 : ((MSU_EXP & 32) ? 16384 : 4096));
  MSU_DISPATCH(dtype, T, return launch_fwd<T, MODE>(a, st, cap));
  return -3;
}

template <int MODE>
int bwd_dispatch(int dtype, const LnBwdArgs& a, float* dgamma, float* dbeta, int nparts, int accumulate,
                 hipStream_t st) {
  if (a.C % (msu_is16(dtype) ? 8 : 4) != 0 || a.C > 2048) return -2;
  if (a.rows == 0) return 0;
  int rc = -3;
  // the parameter-gradient partials summed by the kernel's last blocks (16-B aligned rows and
  // outputs), else by a colsum launch after it
  const bool al = ((uintptr_t)a.part & 15) == 0 && ((uintptr_t)dgamma & 15) == 0 && ((uintptr_t)dbeta & 15) == 0;
  LnBwdArgs b = a;
  b.tail = al && nparts <= TAIL_GS * (TAIL_WORDS - 1) ? tail_slot(st) : -1;
  b.accumulate = accumulate;
  b.dgamma = dgamma;
  b.dbeta = dbeta;
  // dgamma and dbeta null: only the [nparts][2C] partials are written (the caller reduces them
  // later, msu_colsum_batch: the deferred LayerNorm parameter gradients)
  const bool partials_only = dgamma == nullptr && dbeta == nullptr;
  if (partials_only || (MSU_EXP & 128) != 0) b.tail = -1;  // (128: ablation, no reduction)
  MSU_DISPATCH(dtype, T, rc = launch_bwd<T, MODE>(b, st, nparts));
  if (rc || b.tail >= 0 || partials_only || (MSU_EXP & 128)) return rc;
  if (dbeta == dgamma + a.C) {  // contiguous [dgamma | dbeta]: one reduction launch
    colsum(a.part, nparts, 2L * a.C, 2L * a.C, dgamma, accumulate, st);
  } else {
    const ColSeg segs[2] = {{a.part, a.C, 2L * a.C, dgamma}, {a.part + a.C, a.C, 2L * a.C, dbeta}};
    colsum_multi(segs, 2, nparts, accumulate, st);
  }
  return MSU_CHECK_LAUNCH();
}

// ----------------------------------------------------------------------------- head
// FinalPatchExpand_X4_V2.norm (model_parts.py:475) fused with the bias-free 1x1 `output`
// conv (:751, :846) for num_classes == 1: logit[r] = sum_c LN(z[r])_c * w_c (f32 logits).
template <typename T, int KMAX>
__global__ void __launch_bounds__(256) head_fwd_kernel(const T* z, const float* gamma, const float* beta,
                                                       const float* w, float* logit, float* mean,
                                                       float* rstd, long rows, int C, float eps) {
  constexpr int TPR = 8, GPB = 32;
  const int lane = threadIdx.x % TPR, grp = threadIdx.x / TPR;
  const int nchunk = C >> 2;
  for (long r = (long)blockIdx.x * GPB + grp; r < rows; r += (long)gridDim.x * GPB) {
    float v[KMAX][4];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        Vec4<T>::load(z + r * (long)C + ch * 4, v[k]);
#pragma unroll
        for (int e = 0; e < 4; ++e) sum += v[k][e];
      }
    }
    const float mu = group_sum<TPR>(sum) / C;
    float var = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { const float d = v[k][e] - mu; var += d * d; }
      }
    }
    const float rs = rsqrtf(group_sum<TPR>(var) / C + eps);
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = ch * 4 + e;
          dot += ((v[k][e] - mu) * rs * gamma[c] + beta[c]) * w[c];
        }
      }
    }
    dot = group_sum<TPR>(dot);
    if (lane == 0) { logit[r] = dot; mean[r] = mu; rstd[r] = rs; }
  }
}

template <typename T, int KMAX>
__global__ void __launch_bounds__(256) head_bwd_kernel(const float* dlogit, const T* z, const float* gamma,
                                                       const float* beta, const float* w,
                                                       const float* mean, const float* rstd, T* dz,
                                                       float* part /* [grid, 3, C] */, long rows, int C) {
  constexpr int TPR = 8, GPB = 32;
  const int lane = threadIdx.x % TPR, grp = threadIdx.x / TPR;
  const int nchunk = C >> 2;
  float ag[KMAX][4], ab[KMAX][4], aw[KMAX][4];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) { ag[k][e] = 0.f; ab[k][e] = 0.f; aw[k][e] = 0.f; }
  for (long r = (long)blockIdx.x * GPB + grp; r < rows; r += (long)gridDim.x * GPB) {
    const float mu = mean[r], rs = rstd[r], dl = dlogit[r];
    float xh[KMAX][4], g[KMAX][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        float xv[4];
        Vec4<T>::load(z + r * (long)C + ch * 4, xv);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = ch * 4 + e;
          const float dy = dl * w[c];
          xh[k][e] = (xv[e] - mu) * rs;
          g[k][e] = dy * gamma[c];
          s1 += g[k][e];
          s2 += g[k][e] * xh[k][e];
          ag[k][e] += dy * xh[k][e];
          ab[k][e] += dy;
          aw[k][e] += dl * (xh[k][e] * gamma[c] + beta[c]);
        }
      }
    }
    s1 = group_sum<TPR>(s1) / C;
    s2 = group_sum<TPR>(s2) / C;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int ch = lane + k * TPR;
      if (ch < nchunk) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (g[k][e] - s1 - xh[k][e] * s2);
        Vec4<T>::store(dz + r * (long)C + ch * 4, o);
      }
    }
  }
  __shared__ float red[3][256 / 4][4];
  for (int gsel = 0; gsel < GPB; ++gsel) {
    if (grp == gsel) {
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const int ch = lane + k * TPR;
        if (ch < nchunk) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (gsel == 0) { red[0][ch][e] = ag[k][e]; red[1][ch][e] = ab[k][e]; red[2][ch][e] = aw[k][e]; }
            else { red[0][ch][e] += ag[k][e]; red[1][ch][e] += ab[k][e]; red[2][ch][e] += aw[k][e]; }
          }
        }
      }
    }
    __syncthreads();
  }
  float* P = part + (long)blockIdx.x * 3 * C;
  for (int i = threadIdx.x; i < C; i += 256) {
    P[i] = red[0][i >> 2][i & 3];
    P[C + i] = red[1][i >> 2][i & 3];
    P[2 * C + i] = red[2][i >> 2][i & 3];
  }
}

// 16-bit, C % 32 == 0: 4 lanes per row, 16-B loads (KC chunks of 8 channels per lane), the
// lane's gamma*w / beta*w slices held in registers, two rows per iteration for ILP.
template <typename T, int KC>
__global__ void __launch_bounds__(256) head_fwd16_kernel(const T* z, const float* gamma, const float* beta,
                                                         const float* w, float* logit, float* mean,
                                                         float* rstd, long rows, float eps) {
  constexpr int TPR = 4, C = 32 * KC, RPB = 256 / TPR;
  const int lane = threadIdx.x % TPR, grp = threadIdx.x / TPR;
  float gw[KC][8];
  float bwsum = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = (lane + TPR * k) * 8 + e;
      gw[k][e] = gamma[c] * w[c];
      bwsum += beta[c] * w[c];
    }
  bwsum = group_sum<TPR>(bwsum);
  for (long r0 = ((long)blockIdx.x * RPB + grp) * 2; r0 < rows; r0 += (long)gridDim.x * RPB * 2) {
    float v[2][KC][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const long r = r0 + h < rows ? r0 + h : r0;
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const u32x4 q = *reinterpret_cast<const u32x4*>(z + r * C + (lane + TPR * k) * 8);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[h][k][2 * i] = Fmt16<T>::lo(q[i]);
          v[h][k][2 * i + 1] = Fmt16<T>::hi(q[i]);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) sum += v[h][k][e];
      const float mu = group_sum<TPR>(sum) * (1.0f / C);
      float var = 0.f, dot = 0.f;
#pragma unroll
      for (int k = 0; k < KC; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[h][k][e] - mu;
          var += d * d;
          dot += d * gw[k][e];
        }
      const float rs = rsqrtf(group_sum<TPR>(var) * (1.0f / C) + eps);
      dot = group_sum<TPR>(dot) * rs + bwsum;
      if (lane == 0 && r0 + h < rows) {
        logit[r0 + h] = dot;
        mean[r0 + h] = mu;
        rstd[r0 + h] = rs;
      }
    }
  }
}

// dgamma_c = w_c A_c, dbeta_c = w_c D, dw_c = gamma_c A_c + beta_c D with A_c = sum_r dl xh_c,
// D = sum_r dl: per block only A (per channel) and D are accumulated, reduced over the
// block's 64 row groups in fixed order through LDS, and expanded into the [3][C] partial.
// PF: the group's next row (z chunks, mean, rstd, dlogit) is loaded while this one is reduced
// and stored -- a group walks ~128 rows per launch at 1024^2; the arithmetic is the plain loop's
// (no implicit contraction; 0 of 61 tensors differ from the plain loop, r04ab)
template <typename T, int KC, bool PF = true>
__global__ void __launch_bounds__(256) head_bwd16_kernel(const float* dlogit, const T* z, const float* gamma,
                                                         const float* beta, const float* w, const float* mean,
                                                         const float* rstd, T* dz,
                                                         float* part /* [grid, 3, C] */, long rows) {
#pragma clang fp contract(off)
  constexpr int TPR = 4, C = 32 * KC, RPB = 256 / TPR;
  __shared__ float redA[RPB][C + 1];
  __shared__ float redD[RPB];
  const int lane = threadIdx.x % TPR, grp = threadIdx.x / TPR;
  float gw[KC][8], acc[KC][8];
  float adl = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = (lane + TPR * k) * 8 + e;
      gw[k][e] = gamma[c] * w[c];
      acc[k][e] = 0.f;
    }
  const long stride = (long)gridDim.x * RPB;
  long r = (long)blockIdx.x * RPB + grp;
  u32x4 nq[KC];
  float nmu = 0.f, nrs = 0.f, ndl = 0.f;
  auto fetch = [&](long rr) __attribute__((always_inline)) {
    nmu = mean[rr];
    nrs = rstd[rr];
    ndl = dlogit[rr];
#pragma unroll
    for (int k = 0; k < KC; ++k) nq[k] = *reinterpret_cast<const u32x4*>(z + rr * C + (lane + TPR * k) * 8);
  };
  if (PF && r < rows) fetch(r);
  for (; r < rows; r += stride) {
    if constexpr (!PF) fetch(r);
    const float mu = nmu, rs = nrs, dl = ndl;
    u32x4 cq[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) cq[k] = nq[k];
    if constexpr (PF) {
      if (r + stride < rows) fetch(r + stride);
    }
    float xh[KC][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const u32x4 q = cq[k];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xh[k][2 * i] = (Fmt16<T>::lo(q[i]) - mu) * rs;
        xh[k][2 * i + 1] = (Fmt16<T>::hi(q[i]) - mu) * rs;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float g = dl * gw[k][e];
        s1 += g;
        s2 = __builtin_fmaf(g, xh[k][e], s2);
        acc[k][e] = __builtin_fmaf(dl, xh[k][e], acc[k][e]);
      }
    }
    adl += dl;
    s1 = group_sum<TPR>(s1) * (1.0f / C);
    s2 = group_sum<TPR>(s2) * (1.0f / C);
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rs * __builtin_fmaf(-xh[k][e], s2, dl * gw[k][e] - s1);
      *reinterpret_cast<u32x4*>(dz + r * C + (lane + TPR * k) * 8) =
          u32x4{pack2<T>(o[0], o[1]), pack2<T>(o[2], o[3]), pack2<T>(o[4], o[5]), pack2<T>(o[6], o[7])};
    }
  }
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) redA[grp][(lane + TPR * k) * 8 + e] = acc[k][e];
  if (lane == 0) redD[grp] = adl;
  __syncthreads();
  float D = 0.f;
  for (int g = 0; g < RPB; ++g) D += redD[g];
  float* P = part + (long)blockIdx.x * 3 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    float A = 0.f;
    for (int g = 0; g < RPB; ++g) A += redA[g][c];
    P[c] = w[c] * A;
    P[C + c] = w[c] * D;
    P[2 * C + c] = gamma[c] * A + beta[c] * D;
  }
}

}  // namespace

int g_msu_tail_on = 1;

extern "C" {

int msu_head_fwd(int dtype, const void* z, const float* gamma, const float* beta, const float* w,
                 float* logit, float* mean, float* rstd, long rows, int C, float eps, void* stream) {
  if (C % 4 || C > 256) return -2;
  if (rows == 0) return 0;
  long nb = (rows + 31) / 32;
  if (nb > 8192) nb = 8192;
  hipStream_t st = (hipStream_t)stream;
  if (msu_is16(dtype) && (C == 96 || C == 128)) {
    long g = (rows + 127) / 128;
    if (g > 4096) g = 4096;
    MSU_DISPATCH16(dtype, T,
      if (C == 96) hipLaunchKernelGGL((head_fwd16_kernel<T, 3>), dim3(g), dim3(256), 0, st, (const T*)z, gamma, beta, w, logit, mean, rstd, rows, eps);
      else hipLaunchKernelGGL((head_fwd16_kernel<T, 4>), dim3(g), dim3(256), 0, st, (const T*)z, gamma, beta, w, logit, mean, rstd, rows, eps));
    return MSU_CHECK_LAUNCH();
  }
  MSU_DISPATCH(dtype, T,
    if (C <= 128) hipLaunchKernelGGL((head_fwd_kernel<T, 4>), dim3(nb), dim3(256), 0, st, (const T*)z, gamma, beta, w, logit, mean, rstd, rows, C, eps);
    else hipLaunchKernelGGL((head_fwd_kernel<T, 8>), dim3(nb), dim3(256), 0, st, (const T*)z, gamma, beta, w, logit, mean, rstd, rows, C, eps));
  return MSU_CHECK_LAUNCH();
}

// grads: dgamma, dbeta, dw (each [C]); part [nparts, 3, C]
int msu_head_bwd2(int dtype, const float* dlogit, const void* z, const float* gamma,
                  const float* beta, const float* w, const float* mean, const float* rstd, void* dz,
                  float* part, int nparts, float* dgamma, float* dbeta, float* dw, long rows, int C,
                  int accumulate, void* stream) {
  if (C % 4 || C > 256) return -2;
  if (rows == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (msu_is16(dtype) && (C == 96 || C == 128)) {
    MSU_DISPATCH16(dtype, T,
      if (C == 96) hipLaunchKernelGGL((head_bwd16_kernel<T, 3>), dim3(nparts), dim3(256), 0, st, dlogit, (const T*)z, gamma, beta, w, mean, rstd, (T*)dz, part, rows);
      else hipLaunchKernelGGL((head_bwd16_kernel<T, 4>), dim3(nparts), dim3(256), 0, st, dlogit, (const T*)z, gamma, beta, w, mean, rstd, (T*)dz, part, rows));
  } else {
    MSU_DISPATCH(dtype, T,
      if (C <= 128) hipLaunchKernelGGL((head_bwd_kernel<T, 4>), dim3(nparts), dim3(256), 0, st, dlogit, (const T*)z, gamma, beta, w, mean, rstd, (T*)dz, part, rows, C);
      else hipLaunchKernelGGL((head_bwd_kernel<T, 8>), dim3(nparts), dim3(256), 0, st, dlogit, (const T*)z, gamma, beta, w, mean, rstd, (T*)dz, part, rows, C));
  }
  if (dbeta == dgamma + C && dw == dgamma + 2 * C) {  // contiguous [dgamma | dbeta | dw]
    colsum(part, nparts, 3L * C, 3L * C, dgamma, accumulate, st);
  } else {
    const ColSeg segs[3] = {{part, C, 3L * C, dgamma}, {part + C, C, 3L * C, dbeta}, {part + 2 * C, C, 3L * C, dw}};
    colsum_multi(segs, 3, nparts, accumulate, st);
  }
  return MSU_CHECK_LAUNCH();
}

int msu_head_bwd(int dtype, const float* dlogit, const void* z, const float* gamma,
                 const float* beta, const float* w, const float* mean, const float* rstd, void* dz,
                 float* part, int nparts, float* dgamma, float* dbeta, float* dw, long rows, int C,
                 void* stream) {
  return msu_head_bwd2(dtype, dlogit, z, gamma, beta, w, mean, rstd, dz, part, nparts, dgamma, dbeta, dw, rows, C,
                       0, stream);
}

int msu_ln_part_blocks(long rows, int C) {
  // >= 16 rows per block (the per-block parameter-gradient reduction amortises) and enough
  // blocks to fill the CUs at the deep stages (8192 rows x 768: 512 blocks, not 64).  Cap 1024
  // (512 / 256: 168.2 / 162.5 vs 170.0 img/s, r04t); C >= 384 (stages 2-3, whose partials are 2C
  // wide and whose reductions run on the main stream): 512 (170.5 / 170.4 vs 169.8 / 169.8 with
  // 1024, 256: 168.7 / 168.6; r04v)
  constexpr long cap = (MSU_EXP & 2) ? 4096 : ((MSU_EXP & 1) ? 2048 : 1024);
  constexpr long cap_deep = (MSU_EXP & 2) ? 2048 : ((MSU_EXP & 1) ? 1024 : 512);
  long nb = (rows + 15) / 16;
  if (nb > cap) nb = cap;
  if (C >= 384 && nb > cap_deep) nb = cap_deep;
  return nb < 1 ? 1 : (int)nb;
}

int msu_layernorm_fwd(int dtype, int mode, const void* x, const void* b, const float* bscale,
                      long rows_per_sample, void* s_out, const float* gamma, const float* beta,
                      void* y, float* mean, float* rstd, long rows, int C, int H, int W, int Cin,
                      float eps, void* stream) {
  LnArgs a{x, b, bscale, s_out, gamma, beta, y, mean, rstd, rows, C, H, W, Cin,
           rows_per_sample > 0 ? rows_per_sample : 1, eps};
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case IN_PLAIN: return fwd_dispatch<IN_PLAIN>(dtype, a, st);
    case IN_ADD: return fwd_dispatch<IN_ADD>(dtype, a, st);
    case IN_MERGE: return fwd_dispatch<IN_MERGE>(dtype, a, st);
    case IN_D2S2: return fwd_dispatch<IN_D2S2>(dtype, a, st);
  }
  return -3;
}

int msu_layernorm_bwd(int dtype, int mode, const void* dy, const void* x, const void* dres,
                      const float* gamma, const float* mean, const float* rstd, void* dx,
                      void* db, const float* bscale, long rows_per_sample, float* part,
                      int nparts, float* dgamma, float* dbeta, long rows, int C, int H, int W,
                      int Cin, int accumulate, void* stream) {
  LnBwdArgs a{dy, x, dres, gamma, mean, rstd, dx, db, bscale, part, rows, C, H, W, Cin,
              rows_per_sample > 0 ? rows_per_sample : 1};
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case IN_PLAIN: return bwd_dispatch<IN_PLAIN>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
    case IN_ADD: return bwd_dispatch<IN_ADD>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
    case IN_MERGE: return bwd_dispatch<IN_MERGE>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
    case IN_D2S2: return bwd_dispatch<IN_D2S2>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
  }
  return -3;
}

int msu_layernorm_bwd3(int dtype, int mode, const void* dy, const void* x, const void* dres,
                       const void* dres2, const void* dres3, const float* gamma, const float* mean,
                       const float* rstd, void* dx, void* db, const float* bscale, long rows_per_sample,
                       float* part, int nparts, float* dgamma, float* dbeta, long rows, int C, int H, int W,
                       int Cin, int accumulate, void* stream) {
  if ((dres2 || dres3) && (!dres || (mode != IN_PLAIN && mode != IN_ADD) || (dres3 && !dres2))) return -3;
  LnBwdArgs a{dy, x, dres, gamma, mean, rstd, dx, db, bscale, part, rows, C, H, W, Cin,
              rows_per_sample > 0 ? rows_per_sample : 1};
  a.dres2 = dres2;
  a.dres3 = dres3;
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case IN_PLAIN: return bwd_dispatch<IN_PLAIN>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
    case IN_ADD: return bwd_dispatch<IN_ADD>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
    case IN_MERGE: return bwd_dispatch<IN_MERGE>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
    case IN_D2S2: return bwd_dispatch<IN_D2S2>(dtype, a, dgamma, dbeta, nparts, accumulate, st);
  }
  return -3;
}

int msu_tail_reduce_mode(int mode) {
  const int prev = g_msu_tail_on;
  g_msu_tail_on = mode ? 1 : 0;
  return prev;
}

int msu_colsum_batch(int nseg, const float* const* part, const long* stride, const int* nparts, const int* n,
                     float* const* out, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  for (int j0 = 0; j0 < nseg; j0 += CB_MAX) {
    ColBatch cb{};
    cb.nseg = nseg - j0 < CB_MAX ? nseg - j0 : CB_MAX;
    cb.accumulate = accumulate;
    int blocks = 0;
    for (int j = 0; j < cb.nseg; ++j) {
      const int k = j0 + j;
      if (n[k] % 4 || stride[k] % 4 || ((uintptr_t)part[k] & 15) || ((uintptr_t)out[k] & 15) || nparts[k] < 1) return -3;
      cb.part[j] = part[k];
      cb.out[j] = out[k];
      cb.stride[j] = stride[k];
      cb.n[j] = n[k];
      cb.nparts[j] = nparts[k];
      blocks += (n[k] / 4 + CB_NC - 1) / CB_NC;
      cb.bend[j] = blocks;
    }
    if (blocks == 0) continue;
    hipLaunchKernelGGL(colsum_batch_kernel, dim3(blocks), dim3(256), 0, st, cb);
    const int rc = MSU_CHECK_LAUNCH();
    if (rc) return rc;
  }
  return 0;
}

int msu_reduce_rows(const float* part, int nparts, int n, long stride, float* out,
                    int accumulate, void* stream) {
  colsum(part, nparts, n, stride, out, accumulate, (hipStream_t)stream);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
