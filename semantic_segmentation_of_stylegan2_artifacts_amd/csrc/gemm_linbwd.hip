// Stage-0 Linear backward in one pass over the tokens: the input gradient, the weight gradient
// and the bias gradient of y = x . W^T + b read dY once.
//
//   dX[M][K] = epi(dY[M][N] . W[N][K])           (epi: plain, or * GELU'(H) for mlp.3 -> mlp.0)
//   dW[N][K] += sum over tokens of dY^T X        (per-workgroup partial, reduced by colsum)
//   db[N]    += sum over tokens of dY
//
// Replaces, for the HBM-bound stage-0 shapes of the Swin block Linears (qkv, proj, mlp.0,
// mlp.3: K x N in {96 x 288, 96 x 96, 96 x 384, 384 x 96}; model_parts.py:143-151, torchvision
// block at :170 / :538), the token-GEMM input gradient on the main stream PLUS the weight
// gradient on the side stream: separately the two read every dY twice (the second read on the
// side stream, where it competed with the main stream's HBM-bound kernels: the side stream's
// weight gradients cost the main stream 5.9 ms/step).
//
// One 8-wave workgroup per CU, two waves per SIMD (the weight-gradient accumulators of a
// workgroup are the whole 32 x 32-tiled K x N product, at most 6 tiles = 96 registers per wave).
// W^T [K][N] (the trainer's transposed bf16 shadow) sits in LDS for the kernel's life; the token
// rows of dY and X come through a two-stage LDS image, register-staged D steps ahead.  Per
// 32-token step:
//   * input gradient: C^T[k][t] = W^T[k][:] . dY[t][:]^T, k-tiles dealt to the waves;
//   * weight gradient: C[k][n] += X[:, k]^T . dY[:, n] over the step's 32 tokens (two 16-deep
//     k steps, both operands read token-strided with ds_read_b64_tr_b16), the K/32 x N/32 tiles
//     dealt so that every wave issues about the same number of MFMAs;
//   * bias gradient: column sums of the dY image (VALU, rows dealt over all waves).
// W^T and dY rows are padded by 8 elements (row stride = 4 mod 8 dwords: the 16 rows of a
// ds_read_b128 lane group fall on 16 distinct bank groups); X rows, read only token-strided,
// use a stride of 16 or 48 mod 64 dwords (ldx_of).
#include <utility>

#include "common.h"
#include "reduce.h"

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
// (1 no dX stores, 2 no input-gradient MFMAs / reads, 4 no weight-gradient MFMAs / reads,
// 8 no staging loads, 16 no bias sums)
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace {

// Tokens per step: 64 for the K = 96 shapes whose W^T image leaves room for two 64-token
// stages (qkv, proj: half the barriers and LDS round trips per token), else 32.
// MSU_LB_TS64=0: every shape at 32 (A/B builds).
#ifndef MSU_LB_TS64
#define MSU_LB_TS64 1
#endif
constexpr int ts_of(int K, int N) { return (MSU_LB_TS64 && K == 96 && (N == 288 || N == 96)) ? 64 : 32; }
constexpr int NW = 8;                  // waves per workgroup
constexpr int NTHR = 64 * NW;

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

template <int I> using IC = std::integral_constant<int, I>;

template <typename F, int... I>
MSU_DEV __attribute__((always_inline)) void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(IC<I>{}), ...);
}
// f(IC<0>{}), ..., f(IC<N - 1>{})
template <int N, typename F>
MSU_DEV __attribute__((always_inline)) void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// LDS row stride of the X image (elements).  X is only read token-strided (ds_read_b64_tr_b16:
// 32 lanes = 4 rows x 16 dwords), which is conflict-free when the row stride is 16 or 48
// dwords mod 64 (K = 96: unpadded; K = 384: + 32 elements).  The dY image is also read
// row-wise with ds_read_b128 by the input gradient and keeps the 4-mod-8-dword pad.
template <int K>
constexpr int ldx_of() {
  int p = 0;
  while (((K + p) / 2) % 64 != 16 && ((K + p) / 2) % 64 != 48) p += 8;
  return K + p;
}

// register sets of staged token rows (steps of prefetch): as deep as the registers allow
// (MSU_LB_D96 / MSU_LB_DGG: A/B builds of the 96 x 96 and GELU' depths)
#ifndef MSU_LB_D96
#define MSU_LB_D96 4
#endif
#ifndef MSU_LB_DGG
#define MSU_LB_DGG 2
#endif
// MSU_LB_HALL: GELU' operands loaded by every wave for every slot (a wave without a second
// k-tile re-reads its first), so that the compiler's counts do not depend on the wave
#ifndef MSU_LB_HALL
#define MSU_LB_HALL 0
#endif
template <int K, int N, bool GG>
constexpr int ring_depth() {
  return GG ? MSU_LB_DGG : ts_of(K, N) == 64 ? 2 : (K == 96 && N == 96 ? MSU_LB_D96 : 3);
}

MSU_DEV v4s tr_read(const bf16_t* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p); }

// 16-B global loads of the staged token rows.  Plain (compiler-tracked) loads: the compiler
// places the vmcnt waits.  Loads it does not track (inline asm, waits counted by hand) kept
// more of the ring in flight, but the compiler then believes the destination registers are
// written at issue and may copy, spill or reuse them while the data is still on its way -- a
// build of that variant faulted on the GPU.
MSU_DEV u32x4 gload16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
// the same from a wave-uniform base and a per-lane byte offset (no 64-bit address VALU)
MSU_DEV u32x4 gload16_s(const void* base, unsigned off) {
  return *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(base) + off);
}

// row-major k-contiguous fragment: lane l -> row row0 + (l & 31), k = k0 + 8 (l >> 5) .. +7
MSU_DEV bf16x8 frag_rows(const bf16_t* base, int ld, int row0, int k0, int lane) {
  return *reinterpret_cast<const bf16x8*>(base + (row0 + (lane & 31)) * ld + k0 + 8 * (lane >> 5));
}

// k-strided fragment of a [k rows][cols] image: lane l -> col col0 + (l & 31), element e ->
// row r0 + 8 (l >> 5) + e (two ds_read_b64_tr_b16)
MSU_DEV bf16x8 frag_tr(const bf16_t* img, int ld, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  v4s both[2] = {tr_read(img + (r0 + 8 * h + q) * ld + col), tr_read(img + (r0 + 8 * h + 4 + q) * ld + col)};
  return *reinterpret_cast<bf16x8*>(both);
}

// Work of wave w: input-gradient k-tiles kt = w, w + 4, ...; weight-gradient tiles j (kt = j /
// NT, nt = j % NT) dealt greedily to the least-loaded wave (loads counted in MFMAs, the input
// gradient's NS16 per k-tile first).  Compile-time table: wg_tile(w, i) = j or -1.
template <int K, int N>
struct Plan {
  static constexpr int KT = K / 32, NT = N / 32, NS16 = N / 16, NWG = KT * NT;
  static constexpr int DMAX = (KT + NW - 1) / NW;
  static constexpr int CAP = 6;  // weight-gradient tiles per wave (96 accumulator registers)
  static_assert(NWG <= NW * CAP, "weight-gradient tiles exceed the register budget");
  struct Table {
    int tile[NW][NWG];
    int count[NW];
    int maxc;
  };
  static constexpr Table make() {
    Table t{};
    int load[NW] = {};
    for (int w = 0; w < NW; ++w) {
      t.count[w] = 0;
      load[w] = 0;
      for (int kt = w; kt < KT; kt += NW) load[w] += NS16;
      for (int i = 0; i < NWG; ++i) t.tile[w][i] = -1;
    }
    for (int j = 0; j < NWG; ++j) {
      // least-loaded wave with room: at most CAP tiles (16 registers each) per wave
      int best = -1;
      for (int w = 0; w < NW; ++w)
        if (t.count[w] < CAP && (best < 0 || load[w] < load[best])) best = w;
      t.tile[best][t.count[best]++] = j;
      load[best] += 2;
    }
    t.maxc = 0;
    for (int w = 0; w < NW; ++w)
      if (t.count[w] > t.maxc) t.maxc = t.count[w];
    return t;
  }
  static constexpr int WMAX = make().maxc;
};

// weight-gradient tile i of wave w (-1: none); i is a compile-time index after unrolling, w is
// wave-uniform: four selects of constants
template <int K, int N>
MSU_DEV int wg_tile(int w, int i) {
  using P = Plan<K, N>;
  constexpr auto t = P::make();
  int jt = -1;
#pragma unroll
  for (int ww = 0; ww < NW; ++ww)
    if (w == ww && i < t.count[ww]) jt = t.tile[ww][i];
  return jt;
}

// GX: X is GELU(H) re-derived from H while the rows are staged (X = H in the arguments): mlp.3
// after the fused MLP forward (csrc/mlp_fused.hip), which keeps H only
template <typename T, int K, int N, bool GG, bool GX = false>
__global__ void __launch_bounds__(NTHR, 1)
linbwd_kernel(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
              const bf16_t* __restrict__ H, bf16_t* __restrict__ dX, float* __restrict__ part, long M) {
  using P = Plan<K, N>;
  constexpr int TM = ts_of(K, N);
  static_assert(!GG || TM == 32, "the GELU' operands are staged for 32-token steps");
  constexpr int LDW = N + 8, LDY = N + 8, LDX = ldx_of<K>();
  constexpr int CY = N / 8, CX = K / 8;              // 16-B chunks per dY / X row
  constexpr int CHUNKS = TM * (CY + CX);
  constexpr int PER = (CHUNKS + NTHR - 1) / NTHR;    // staged chunks per thread and step
  constexpr int STAGE = TM * (LDY + LDX);            // elements per LDS stage
  constexpr int KT = P::KT, NS16 = P::NS16, DMAX = P::DMAX, WMAX = P::WMAX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16_t* sW = reinterpret_cast<bf16_t*>(smem_raw);  // [K][LDW]
  bf16_t* sS = sW + K * LDW;                         // 2 x ([TM][LDY] dY, [TM][LDX] X)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const long ntiles = (M + TM - 1) / TM;
  const int G = gridDim.x;
  const int b = blockIdx.x;
  const long nsteps = (ntiles - 1 - b) / G + 1;  // >= 1: the grid is at most ntiles (grid_of)

  // ---- W^T -> LDS (once)
  for (int i = tid; i < K * CY; i += NTHR) {
    const int r = i / CY, c = i - r * CY;
    *reinterpret_cast<u32x4*>(sW + r * LDW + 8 * c) = *reinterpret_cast<const u32x4*>(Wt + (long)r * N + 8 * c);
  }

  // ---- register-staged token rows, D steps ahead: set Q holds the rows of a step s with
  // s % D == Q (rows past M re-read row M - 1 and are zeroed when they go to LDS; chunks past
  // CHUNKS re-read dY row 0 and are dropped)
  constexpr int D = ring_depth<K, N, GG>();
  u32x4 st[D][PER];
  // chunk c = tid + NTHR j of a step: dY chunks first, then X chunks, then none.  The kind is
  // wave-uniform (the boundaries are multiples of 64); the offsets are step-invariant: element
  // offset from the step's first row in global memory and in the LDS stage
  int goff[PER], loff[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int c = tid + NTHR * j;
    goff[j] = 0;
    loff[j] = 0;
    if (c < TM * CY) {
      const int r = c / CY, cc = c - r * CY;
      goff[j] = r * N + 8 * cc;
      loff[j] = r * LDY + 8 * cc;
    } else if (c < CHUNKS) {
      const int c2 = c - TM * CY;
      const int r = c2 / CX, cc = c2 - r * CX;
      goff[j] = r * K + 8 * cc;
      loff[j] = TM * LDY + r * LDX + 8 * cc;
    }
  }
  auto kind = [&](int j) __attribute__((always_inline)) {  // 0 dY, 1 X, 2 none (wave-uniform)
    const int cw = wave * 64 + NTHR * j;
    return cw < TM * CY ? 0 : cw < CHUNKS ? 1 : 2;
  };
  // Issued on every path (past the last step: a dummy re-read of the last step's rows) so
  // that the compiler's wait before each LDS store leaves the younger sets in flight (with the
  // issue behind a branch it counts the path without it and waits for everything).
  auto load = [&](long step_, auto SET) __attribute__((always_inline)) {
    constexpr int set = decltype(SET)::value;
    const long step = step_ < nsteps ? step_ : nsteps - 1;
    const long m0 = (b + step * G) * TM;
    if (m0 + TM <= M) {  // whole step: uniform row base + per-lane 32-bit offset
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int kd = kind(j);
        const bf16_t* base = kd == 0 ? dY + m0 * N : kd == 1 ? X + m0 * K : dY;
        if constexpr ((MSU_EXP & 8) != 0) st[set][j] = u32x4{(unsigned)goff[j], 0u, 0u, 0u};
        else st[set][j] = gload16_s(base, 2u * (unsigned)goff[j]);
      }
    } else {  // the ragged last step: rows past M re-read row M - 1
      const int t0 = opaque(tid);
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int c = t0 + NTHR * j;
        const bf16_t* src = dY;
        if (c < TM * CY) {
          const int r = c / CY, cc = c - r * CY;
          const long m = m0 + r < M ? m0 + r : M - 1;
          src = dY + m * N + 8 * cc;
        } else if (c < CHUNKS) {
          const int c2 = c - TM * CY;
          const int r = c2 / CX, cc = c2 - r * CX;
          const long m = m0 + r < M ? m0 + r : M - 1;
          src = X + m * K + 8 * cc;
        }
        st[set][j] = gload16(src);
      }
    }
  };
  // set SET (rows of step `step`) -> LDS stage step & 1
  // after this one (they may stay in flight; other VMEM ops issued in between make the wait
  // retire more, never less)
  auto store = [&](long step, auto SET) __attribute__((always_inline)) {
    constexpr int set = decltype(SET)::value;
    if constexpr (GX) {
      // X chunks: GELU of the staged H (the forward's arithmetic: gelu_fast of the 16-bit H,
      // rounded to 16 bits), so the image holds exactly the activation the forward fed mlp.3
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (kind(j) == 1) {
          u32x4& q = st[set][j];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            q[i] = pack2<T>(gelu_fast(Fmt16<T>::lo(q[i])), gelu_fast(Fmt16<T>::hi(q[i])));
        }
      }
    }
    // every path passes one wait (the last D - 1 steps of a workgroup drain fully)
    bf16_t* y = sS + (int)(step & 1) * STAGE;
    const long m0 = (b + step * G) * TM;
    if (m0 + TM <= M) {
#pragma unroll
      for (int j = 0; j < PER; ++j)
        if (kind(j) != 2) *reinterpret_cast<u32x4*>(y + loff[j]) = st[set][j];
    } else {  // rows past M go to LDS as zeros
      const int t0 = opaque(tid);
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const int c = t0 + NTHR * j;
        const int r = c < TM * CY ? c / CY : (c - TM * CY) / CX;
        const u32x4 z = {0u, 0u, 0u, 0u};
        if (kind(j) != 2) *reinterpret_cast<u32x4*>(y + loff[j]) = m0 + r < M ? st[set][j] : z;
      }
    }
  };

  f32x16 accw[WMAX];  // weight-gradient tiles C[k][n] of this wave
#pragma unroll
  for (int i = 0; i < WMAX; ++i) accw[i] = f32x16{0};
  // bias gradient: thread tid sums column pair bp over the rows bg, bg + RG, ... of each step
  // (every wave takes a share instead of the N / 2 threads of the input-gradient waves)
  constexpr int NP = N / 2, RG = NTHR / NP < TM ? NTHR / NP : TM;
  const int bp = tid % NP, bg = tid / NP;
  float db0 = 0.f, db1 = 0.f;

  static_for<D>([&](auto I) __attribute__((always_inline)) {
    load(decltype(I)::value, I);
  });
  store(0, IC<0>{});
  __syncthreads();

  // one step (compile-time slot Q = s % D): compute from LDS stage s & 1; the rows of step s + D
  // are loaded into register set Q (its step-s rows went to LDS a step ago), the rows of step
  // s + 1 (set (Q + 1) % D) go to the other LDS stage at the end
  auto body = [&](long s, auto SLOT) __attribute__((always_inline)) {
    constexpr int slot = decltype(SLOT)::value;
    const bf16_t* y = sS + (int)(s & 1) * STAGE;
    const bf16_t* x = y + TM * LDY;
    const long m0 = (b + s * G) * TM;
    // GELU' operands of this wave's input-gradient tiles (lane: token m0 + (lane & 31)), issued
    // before the step s + D rows
    u32x4 hv[DMAX][2];
    if constexpr (GG) {
      const long m = m0 + (lane & 31);
      const long mh = m < M ? m : M - 1;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        const int kt0 = wave + NW * d;
        if (MSU_LB_HALL || kt0 < KT) {
          const int kt = kt0 < KT ? kt0 : wave;
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) hv[d][pp] = gload16(H + mh * K + 32 * kt + 16 * pp + 8 * h);
        }
      }
    }
    load(s + D, SLOT);

    // ---- weight gradient: this wave's tiles, two 16-token k steps
#pragma unroll
    for (int i = 0; i < WMAX; ++i) {
      const int jt = wg_tile<K, N>(wave, i);
      if (jt >= 0 && (MSU_EXP & 4) == 0) {
        const int jo = opaque(jt);
        const int kt = jo / P::NT, nt = jo - (jo / P::NT) * P::NT;
#pragma unroll
        for (int ks = 0; ks < TM / 16; ++ks)
          accw[i] = Fmt16<T>::mma32(frag_tr(x, LDX, 16 * ks, 32 * kt, lane), frag_tr(y, LDY, 16 * ks, 32 * nt, lane),
                                    accw[i]);
      }
      // fragment reads of later tiles are not hoisted above this tile's MFMAs (registers)
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- bias gradient: column sums of the dY image, rows dealt over RG thread groups
    if (bg < RG && (MSU_EXP & 16) == 0) {
      for (int r = bg; r < TM; r += RG) {
        const uint32_t w2 = *reinterpret_cast<const uint32_t*>(y + r * LDY + 2 * bp);
        db0 += Fmt16<T>::lo(w2);
        db1 += Fmt16<T>::hi(w2);
      }
    }

    // ---- input gradient: k-tiles kt = wave + NW d, C^T[k][token], 32-token tiles tt
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      const int kt = wave + NW * d;
#pragma unroll
      for (int tt = 0; tt < TM / 32; ++tt) if (kt < KT) {
        // lane: token m0 + 32 tt + (lane & 31); after the permlane32 swap, 8 consecutive k per pair
        const long m = m0 + 32 * tt + (lane & 31);
        f32x16 acc = f32x16{0};
#pragma unroll 3
        for (int ns = 0; ns < ((MSU_EXP & 2) ? 0 : NS16); ++ns)
          acc = Fmt16<T>::mma32(frag_rows(sW, LDW, 32 * kt, 16 * ns, lane), frag_rows(y, LDY, 32 * tt, 16 * ns, lane),
                                acc);
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int g0 = 2 * pp;
          float v[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[4 * g0 + e]),
                                                            __float_as_uint(acc[4 * g0 + 4 + e]), false, false);
            v[e] = __uint_as_float(r[0]);
            v[4 + e] = __uint_as_float(r[1]);
          }
          if constexpr (GG) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              v[2 * e] *= gelu_grad_fast(Fmt16<T>::lo(hv[d][pp][e]));
              v[2 * e + 1] *= gelu_grad_fast(Fmt16<T>::hi(hv[d][pp][e]));
            }
          }
          const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
          if (m < M && (MSU_EXP & 1) == 0) *reinterpret_cast<u32x4*>(dX + m * K + 32 * kt + 16 * pp + 8 * h) = pk;
        }
      }
    }
    // next step's rows -> the other stage (its previous readers finished before the last barrier)
    // (counted wait: the rows of steps s + 2 .. s + D may stay in flight; this step's dX stores
    // and GELU' loads are not counted, so the wait errs towards retiring more)
    if (s + 1 < nsteps) {
      store(s + 1, IC<(slot + 1) % D>{});
    }
    __syncthreads();
  };
  for (long s = 0; s < nsteps; s += D) {
    static_for<D>([&](auto I) __attribute__((always_inline)) {
      if (s + decltype(I)::value < nsteps) body(s + decltype(I)::value, I);
    });
  }

  // ---- partials: dW [N][K] (lane n, registers: 4 consecutive k per group) and db [N]
  float* pw = part + (long)b * (N * K + N);
#pragma unroll
  for (int i = 0; i < WMAX; ++i) {
    const int jt = wg_tile<K, N>(wave, i);
    if (jt >= 0) {
      const int kt = jt / P::NT, nt = jt - (jt / P::NT) * P::NT;
      const int n = 32 * nt + (lane & 31);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int k = 32 * kt + 8 * g + 4 * h;
        *reinterpret_cast<float4*>(pw + (long)n * K + k) =
            make_float4(accw[i][4 * g], accw[i][4 * g + 1], accw[i][4 * g + 2], accw[i][4 * g + 3]);
      }
    }
  }
  // row groups -> one sum per column pair, through the (now idle) LDS stages
  float2* red = reinterpret_cast<float2*>(sS);
  if (bg < RG) red[bg * NP + bp] = make_float2(db0, db1);
  __syncthreads();
  if (tid < NP) {
    float s0 = 0.f, s1 = 0.f;
    for (int g = 0; g < RG; ++g) {
      const float2 v = red[g * NP + tid];
      s0 += v.x;
      s1 += v.y;
    }
    pw[N * K + 2 * tid] = s0;
    pw[N * K + 2 * tid + 1] = s1;
  }
}

template <int K, int N>
constexpr size_t linbwd_lds() {
  return sizeof(bf16_t) * ((size_t)K * (N + 8) + 2 * (size_t)ts_of(K, N) * ((N + 8) + ldx_of<K>()));
}

int num_cus_lb() {
  static const int cus = [] {
    int n = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}

long grid_of(long M, int K, int N) {
  const int ts = ts_of(K, N);
  const long ntiles = (M + ts - 1) / ts;
  const long g = num_cus_lb();
  return ntiles < g ? ntiles : g;
}

template <typename T, int K, int N, bool GG, bool GX = false>
int launch_lb(const void* dY, const void* X, const void* Wt, const void* H, void* dX, float* part, long M,
              hipStream_t st) {
  constexpr size_t lds = linbwd_lds<K, N>();
  static_assert(lds <= 160 * 1024, "LDS");
  auto kern = linbwd_kernel<T, K, N, GG, GX>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -4;
    attr = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)grid_of(M, K, N)), dim3(NTHR), lds, st, (const bf16_t*)dY, (const bf16_t*)X,
                     (const bf16_t*)Wt, (const bf16_t*)H, (bf16_t*)dX, part, M);
  return 0;
}

bool lb_shape(int K, int N) {
  return (K == 96 && (N == 288 || N == 96 || N == 384)) || (K == 384 && N == 96);
}

}  // namespace

extern "C" {

// Whether msu_linear_bwd covers (K, N) = (in, out) features of the Linear.
int msu_linear_bwd_supported(long M, int K, int N) { return M > 0 && lb_shape(K, N) ? 1 : 0; }

// f32 workspace floats msu_linear_bwd needs (per-workgroup dW / db partials).
long msu_linear_bwd_workspace(long M, int K, int N) { return grid_of(M, K, N) * ((long)N * K + N); }

// One pass over the tokens of y = x . W^T + b (x [M][K], W [N][K], 16-bit dtype 1 bf16 / 2 f16):
//   dX = dY . W (times GELU'(H) when H != null: mlp.3's input gradient into mlp.0's output),
//   dW (+)= dY^T X and db (+)= column sums of dY (f32, accumulate != 0 adds to dW / db; db may
//   be null).  Wt is W^T [K][N] (16-bit).  X null with H given (mlp.3 only): X = GELU(H),
//   derived from H in the kernel.  Stream: `stream`.
int msu_linear_bwd(int dtype, const void* dY, const void* X, const void* Wt, const void* H, void* dX, float* dW,
                   float* db, float* workspace, long M, int K, int N, int accumulate, void* stream) {
  if (!msu_is16(dtype)) return -3;
  if (M <= 0 || !lb_shape(K, N)) return -2;
  if (H != nullptr && !(K == 384 && N == 96)) return -3;  // the GELU' epilogue: mlp.3 only
  if (X == nullptr && H == nullptr) return -2;
  hipStream_t st = (hipStream_t)stream;
  int rc = -3;
  if (X == nullptr) {
    MSU_DISPATCH16(dtype, T, rc = (launch_lb<T, 384, 96, true, true>(dY, H, Wt, H, dX, workspace, M, st)));
  } else {
#define MSU_LB(KK, NN, GG)                                                                   \
  if (K == KK && N == NN && (H != nullptr) == GG) {                                          \
    MSU_DISPATCH16(dtype, T, rc = launch_lb<T, KK, NN, GG>(dY, X, Wt, H, dX, workspace, M, st)); \
  }
  MSU_LB(96, 288, false)
  MSU_LB(96, 96, false)
  MSU_LB(96, 384, false)
  MSU_LB(384, 96, false)
  MSU_LB(384, 96, true)
  }
#undef MSU_LB
  if (rc) return rc;
  const int parts = (int)grid_of(M, K, N);
  const long stride = (long)N * K + N;
  const ColSeg segs[2] = {{workspace, (long)N * K, stride, dW}, {workspace + (long)N * K, N, stride, db}};
  colsum_multi(segs, db ? 2 : 1, parts, accumulate, st);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
