// Linear-layer weight (and bias) gradient: dW[N][K] = sum_m dY[m][n] X[m][k], db[n] = sum_m dY[m][n].
//
// Every nn.Linear on the MS-UNet path (torchvision block qkv / proj / mlp.0 / mlp.3,
// PatchMerging.reduction, PatchExpand.expand, concat_back_dim, FinalPatchExpand_X4_V2.expand,
// PatchEmbed.proj as im2col GEMM) has M = tokens (up to 8 x 65536 at 1024^2) and N, K = a
// small multiple of the embed width (96 / 128): a tall-skinny "TN" product whose reduction
// runs over M.  Library kernels tile it with far too few workgroups (hipBLASLt picked
// MT64x64x256 at ~0.76 ms/call).  Here:
//   * output tile BT x BT with BT = 96 (Swin-T/S widths) or 128 (Swin-B), 4 waves in 2x2,
//     each wave (BT/2)^2 = 3x3 or 4x4 v_mfma_f32_16x16x32_bf16 tiles;
//   * the M range is split across S workgroups per output tile (S fills the 256 CUs);
//   * operands are staged row-major ([m][n], [m][k]) in LDS, 64 rows per stage, double
//     buffered, and read k-strided with ds_read_b64_tr_b16;
//   * S partial tiles are reduced deterministically (colsum); the bias gradient rides along
//     on the k-tile-0 workgroups.
#include <stdlib.h>

#include "common.h"
#include "mfma_frag.h"
#include "reduce.h"

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace {

constexpr int BM = 64;

MSU_DEV void unpack8(const u32x4& q, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(q[i] << 16);
    v[2 * i + 1] = __uint_as_float(q[i] & 0xffff0000u);
  }
}  // rows of M per LDS stage (two MFMA k-steps)

template <typename T, int NTW>
__global__ void __launch_bounds__(256) wgrad_kernel(const T* __restrict__ dY, const T* __restrict__ X,
                                                    float* __restrict__ part, float* __restrict__ dbpart,
                                                    long M, int N, int K, long mchunk) {
  constexpr int WT = 16 * NTW;    // wave tile
  constexpr int BT = 2 * WT;      // block tile
  constexpr int LDT = BT + 8;     // LDS row stride (elements): rows stay 16-B aligned
  constexpr int EPC = 16 / (int)sizeof(T);  // elements per 16-B staging chunk
  constexpr int CPR = BT / EPC;   // chunks per row
  constexpr int CH = BM * CPR / 256;  // chunks per thread per operand
  __shared__ __attribute__((aligned(16))) T sA[2][BM * LDT];  // dY rows  [m][n]
  __shared__ __attribute__((aligned(16))) T sB[2][BM * LDT];  // X rows   [m][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntk = (K + BT - 1) / BT;
  const int tn = blockIdx.x / ntk, tk = blockIdx.x - (blockIdx.x / ntk) * ntk;
  const int n0 = tn * BT, k0 = tk * BT;
  const long m_begin = (long)blockIdx.y * mchunk;
  long m_end = m_begin + mchunk;
  if (m_end > M) m_end = M;
  const int wn = (wave >> 1) * WT, wk = (wave & 1) * WT;

  f32x4 acc[NTW][NTW];
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  const bool do_bias = dbpart != nullptr && tk == 0;

  // register-staged pipeline: issue the next stage's 16-B loads, compute the current
  // stage from LDS, then write the registers to the other LDS buffer (T14 split)
  uint4 ra[CH], rb[CH];
  auto load_regs = [&](long m0) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + 256 * c;
      const int r = idx / CPR, col = (idx - r * CPR) * EPC;
      const long m = m0 + r;
      const bool ok = m < m_end;
      ra[c] = (ok && n0 + col < N) ? *reinterpret_cast<const uint4*>(dY + m * (long)N + n0 + col) : make_uint4(0, 0, 0, 0);
      rb[c] = (ok && k0 + col < K) ? *reinterpret_cast<const uint4*>(X + m * (long)K + k0 + col) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_regs = [&](int buf) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = tid + 256 * c;
      const int r = idx / CPR, col = (idx - r * CPR) * EPC;
      *reinterpret_cast<uint4*>(&sA[buf][r * LDT + col]) = ra[c];
      *reinterpret_cast<uint4*>(&sB[buf][r * LDT + col]) = rb[c];
    }
  };

  int buf = 0;
  if (m_begin < m_end) {
    load_regs(m_begin);
    store_regs(0);
  }
  __syncthreads();
  for (long m0 = m_begin; m0 < m_end; m0 += BM) {
    const bool more = m0 + BM < m_end;
    if (more) load_regs(m0 + BM);
    const T* A = sA[buf];
    const T* B = sB[buf];
    auto rowA = [&](int k) { return A + k * LDT; };
    auto rowB = [&](int k) { return B + k * LDT; };
#pragma unroll
    for (int ks = 0; ks < BM; ks += 32)
#pragma unroll
      for (int i = 0; i < NTW; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) TR<T>::mma(acc[i][j], rowA, wn + 16 * i, rowB, wk + 16 * j, ks, lane);
    if (do_bias && tid < BT) {
#pragma unroll 8
      for (int r = 0; r < BM; ++r) dbacc += to_f32(A[r * LDT + tid]);
    }
    if (more) store_regs(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  float* out = part + (long)blockIdx.y * N * K;
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn + 16 * i + (lane >> 4) * 4 + r;
        const int k = k0 + wk + 16 * j + (lane & 15);
        if (n < N && k < K) out[(long)n * K + k] = acc[i][j][r];
      }
  if (do_bias && tid < BT && n0 + tid < N) dbpart[(long)blockIdx.y * N + n0 + tid] = dbacc;
}

// bf16: wave-sized output tiles.  Each wave owns a full WT x WT output tile (WT = 96 or
// 128, 36 / 64 accumulators of 16x16) so every fragment read from LDS feeds NTW MFMAs;
// the NW = 4 (or 3) waves split N (WN waves along N, sharing the X rows of the stage), K
// (WK waves along K, sharing the dY rows) and the rows of the stage (WM = NW / (WN WK)
// waves, each its own partial slab).  A workgroup covering more of the N x K output reads
// dY and X fewer times over all workgroups: dY is read K / (WK WT) times, X N / (WN WT)
// times.  Staging is LDS-DMA:
// a stage is RS = 32 * WM rows of dY [RS][BN+8] and X [RS][BK+8] written lane-linearly by
// global_load_lds_dwordx4 (pad slots re-read chunk 0 of their row; rows past the block's
// range read the spread zero region); a ring of NST stages keeps NST-1 in flight; raw
// s_barrier + counted vmcnt keep the prefetch alive across barriers.
// (An eight-wave form, two row groups at two waves per SIMD, was 10-13 % faster alone but slower
// in the step, where its LDS and waves crowd the input-gradient kernels it overlaps: r04m, gone.)
template <int WN, int WK> constexpr int wgrad_nw() { return WN * WK == 3 ? 3 : 4; }

template <typename T, int NTW, int WN, int WK, int NST>
__global__ void __launch_bounds__(256) wgrad_wave_kernel(const bf16_t* __restrict__ dY, const bf16_t* __restrict__ X,
                                                         float* __restrict__ part, float* __restrict__ dbpart,
                                                         long M, int N, int K, long mchunk, int ntiles) {
  constexpr int NW = wgrad_nw<WN, WK>();
  constexpr int WM = NW / (WN * WK), WT = 16 * NTW, BN = WN * WT, BK = WK * WT, RS = 32 * WM;
  static_assert(WM * WN * WK == NW, "wave split");
  constexpr int SA = (BN + 8) / 8, SB = (BK + 8) / 8;  // 16-B slots per row
  constexpr int LA = 8 * SA, LB = 8 * SB;              // row strides (elements)
  constexpr int SLOTS = RS * (SA + SB);
  constexpr int INS = ((SLOTS + 63) / 64 + NW - 1) / NW * NW;
  constexpr int PER_WAVE = INS / NW;
  constexpr int STG = INS * 64 * 8;
  static_assert(NST >= 2 && PER_WAVE * (NST - 2) < 64, "vmcnt");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  bf16_t* lds = reinterpret_cast<bf16_t*>(smem_raw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wni = wave % WN, wki = (wave / WN) % WK, wmi = wave / (WN * WK);
  const int ntk = K / BK;
  // 1-D grid of ntiles x splits work items: consecutive items (the output tiles of one row
  // split, which stream the same dY / X rows) go to one XCD (dispatch is round-robin over the 8
  // XCDs by block id), so the rows a split's tiles share are fetched from HBM once and re-read
  // from that XCD's L2 (r04c: 252 -> 109 MB read per 32768 x 1152 x 384 launch)
  const int item = xcd_remap(blockIdx.x, gridDim.x);
  const int split = item / ntiles, tile = item - split * ntiles;
  const int tn = tile / ntk, tk = tile - (tile / ntk) * ntk;
  const int n0 = tn * BN, k0 = tk * BK;
  const long m_begin = (long)split * mchunk;
  long m_end = m_begin + mchunk;
  if (m_end > M) m_end = M;
  const int nstage = m_end > m_begin ? (int)((m_end - m_begin + RS - 1) / RS) : 0;

  // per-lane DMA slot geometry, fixed across stages: row within the stage, element offset
  // from the stage's first row of dY (A slots) or X (B slots); pad slots re-read chunk 0
  int srow[PER_WAVE], soff[PER_WAVE];
  bool sisA[PER_WAVE];
#pragma unroll
  for (int r = 0; r < PER_WAVE; ++r) {
    const int s = 64 * (wave + NW * r) + lane;
    if (s < RS * SA) {
      const int row = s / SA, c = s - (s / SA) * SA;
      srow[r] = row;
      soff[r] = row * N + n0 + (c < SA - 1 ? 8 * c : 0);
      sisA[r] = true;
    } else {
      const int t = s < SLOTS ? s - RS * SA : 0;
      const int row = t / SB, c = t - (t / SB) * SB;
      srow[r] = s < SLOTS ? row : RS;  // slots past the image: always the zero region
      soff[r] = row * K + k0 + (c < SB - 1 ? 8 * c : 0);
      sisA[r] = false;
    }
  }
  auto issue = [&](int st) __attribute__((always_inline)) {
    bf16_t* buf = lds + (st % NST) * STG;
    const long m0 = m_begin + (long)st * RS;
    const long rem = m_end - m0;
    const int valid = rem > RS ? RS : (rem < 0 ? 0 : (int)rem);
    const bf16_t* baseA = dY + m0 * N;
    const bf16_t* baseB = X + m0 * K;
#pragma unroll
    for (int r = 0; r < PER_WAVE; ++r) {
      const bf16_t* src = (sisA[r] ? baseA : baseB) + soff[r];
      glds16(srow[r] < valid ? (const void*)src : zero_src(64 * r + lane), buf + 64 * 8 * (wave + NW * r));
    }
  };

  f32x4 acc[NTW][NTW];
  f32x4 accb[NTW];  // bias: dY rows times a ones operand
#pragma unroll
  for (int i = 0; i < NTW; ++i) {
    accb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bool do_bias = dbpart != nullptr && tk == 0 && wki == 0;
  const bf16x8 ones = splat8<T>(1.0f, 1.0f, 1.0f);
  // lane part of a k-strided fragment read (ds_read_b64_tr_b16), columns 4p.  The k order
  // is free (both operands use the same one): each 32-lane half reads 8 rows of one parity,
  // 2(4g + q) + half (g = lane group within the half), and the second half of the fragment
  // 16 rows further.  Rows 2j apart sit 2j * stride dwords apart, distinct multiples of 8
  // mod 64 for both row strides (52 and 196 dwords): the 32 lanes cover all 64 banks
  // exactly once (rows 8(lane>>4) + q put two rows on each bank span: 2-way conflicts).
  const int q = (lane & 15) >> 2, p4 = 4 * (lane & 3), r0 = wmi * 32 + 2 * (4 * ((lane >> 4) & 1) + q) + (lane >> 5);
  const int laneA = r0 * LA + wni * WT + p4, laneB = RS * LA + r0 * LB + wki * WT + p4;
  auto tr8 = [](const bf16_t* p, int second) {
    typedef __attribute__((address_space(3))) msu_v4s lds_v4s;
    const msu_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
    const msu_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p + second));
    msu_v4s both[2] = {lo, hi};
    return *reinterpret_cast<bf16x8*>(both);
  };

#pragma unroll
  for (int st = 0; st < NST - 1; ++st) issue(st);
  for (int st = 0; st < nstage; ++st) {
    wait_vmcnt<PER_WAVE * (NST - 2)>();
    __builtin_amdgcn_s_barrier();
    issue(st + NST - 1);  // into the buffer computed in the previous iteration
    // fragments by untracked reads (a visible ds_read would wait for the whole ring);
    // A fragment i+1 is read while the MFMAs of fragment i run
    if constexpr (MSU_EXP & 2) continue;
    const bf16_t* buf = lds + (st % NST) * STG;
    const uint32_t pa = lds_u32(buf + laneA), pb = lds_u32(buf + laneB);
    bf16x8 bf[NTW], af[2];
    unroll_for<NTW>([&](auto J) {
      constexpr int j = decltype(J)::value;
      bf[j] = tr8_untracked<32 * j, 32 * j + 32 * LB>(pb);
    });
    af[0] = tr8_untracked<0, 32 * LA>(pa);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < NTW; ++j) asm volatile("" : "+v"(bf[j]));
    asm volatile("" : "+v"(af[0]));
    unroll_for<NTW>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i + 1 < NTW) af[(i + 1) & 1] = tr8_untracked<32 * (i + 1), 32 * (i + 1) + 32 * LA>(pa);
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        if constexpr (MSU_EXP & 1)
          acc[i][j][0] += (float)af[i & 1][j] * (float)bf[j][i];
        else
          acc[i][j] = Fmt16<T>::mma16(af[i & 1], bf[j], acc[i][j]);
      }
      if constexpr (!(MSU_EXP & 1))
        accb[i] = Fmt16<T>::mma16(af[i & 1], ones, accb[i]);  // unconditional
      // the group's MFMAs stay above the wait: left to the scheduler they sank below it, so each
      // group waited on the read issued just before it (the LDS latency exposed 6x per stage)
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (i + 1 < NTW) lds_wait_tie<0>(af[(i + 1) & 1]);
    });
  }
  wait_vmcnt<0>();  // every DMA has landed: the ring may be reused
  // row-waves of the same output tile are summed in LDS first: one slab per split
  if constexpr (WM > 1) {
    // in HALVES passes over the accumulator rows i when one pass would not fit the LDS
    float* red = reinterpret_cast<float*>(smem_raw);  // [(N, K)-wave][WM - 1][rows of the pass][64]
    constexpr int PWF = (NTW * NTW * 4 + NTW * 4) * 64;  // floats per wave, all rows
    constexpr int HALVES = (size_t)WN * WK * (WM - 1) * PWF * 4 <= 160 * 1024 ? 1 : 2;
    constexpr int IH = NTW / HALVES;
    static_assert(IH * HALVES == NTW, "pass rows");
    constexpr int PW = (IH * NTW * 4 + IH * 4) * 64;  // floats per wave and pass
    static_assert((size_t)WN * WK * (WM - 1) * PW * 4 <= 160 * 1024, "LDS reduction");
    const int wnk = wni + WN * wki;
    float* mine = red + ((long)wnk * (WM - 1) + (wmi > 0 ? wmi - 1 : 0)) * PW;
    unroll_for<HALVES>([&](auto HI) {
      constexpr int h0 = decltype(HI)::value * IH;
      __syncthreads();  // the ring (first pass) / the previous pass's slots are free
      if (wmi > 0) {
#pragma unroll
        for (int i = h0; i < h0 + IH; ++i) {
#pragma unroll
          for (int j = 0; j < NTW; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) mine[(((i - h0) * NTW + j) * 4 + r) * 64 + lane] = acc[i][j][r];
#pragma unroll
          for (int r = 0; r < 4; ++r) mine[(IH * NTW * 4 + (i - h0) * 4 + r) * 64 + lane] = accb[i][r];
        }
      }
      __syncthreads();
      if (wmi == 0) {
#pragma unroll
        for (int w = 1; w < WM; ++w) {
          const float* other = red + ((long)wnk * (WM - 1) + w - 1) * PW;
#pragma unroll
          for (int i = h0; i < h0 + IH; ++i) {
#pragma unroll
            for (int j = 0; j < NTW; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[i][j][r] += other[(((i - h0) * NTW + j) * 4 + r) * 64 + lane];
#pragma unroll
            for (int r = 0; r < 4; ++r) accb[i][r] += other[(IH * NTW * 4 + (i - h0) * 4 + r) * 64 + lane];
          }
        }
      }
    });
  }
  if (wmi != 0) return;
  float* out = part + (long)split * N * K;
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < NTW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wni * WT + 16 * i + (lane >> 4) * 4 + r;
        const int k = k0 + wki * WT + 16 * j + (lane & 15);
        out[(long)n * K + k] = acc[i][j][r];
      }
  if (do_bias && (lane & 15) == 0) {
    // every column of accb holds the row sums
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dbpart[(long)split * N + n0 + wni * WT + 16 * i + (lane >> 4) * 4 + r] = accb[i][r];
  }
}

// bf16 plan: wave tile, waves along N and K, ring depth, splits
struct WavePlan {
  int ntw = 0, wn = 1, wk = 1, nst = 3, S = 1;
  int slabs() const { return S; }
};

// the (WN, WK) split of a workgroup's waves over the N x K tiles: least operand traffic
// M (N kt / WK + K nt / WN) (dY re-read per K group, X per N group), more waves on ties
// (round 3: +1.5 % over the round-2 plan of waves along N only)
inline void pick_wave_split(int nt, int kt, int& wn, int& wk) {
  static const int cand[8][2] = {{4, 1}, {2, 2}, {1, 4}, {3, 1}, {1, 3}, {2, 1}, {1, 2}, {1, 1}};
  long best = -1;
  for (const auto& c : cand) {
    if (nt % c[0] || kt % c[1]) continue;
    const long cost = (long)nt * kt / c[1] + (long)kt * nt / c[0];  // in units of M * WT
    if (best < 0 || cost < best) {
      best = cost;
      wn = c[0];
      wk = c[1];
    }
  }
}

inline WavePlan wave_plan(long M, int N, int K) {
  WavePlan p;
  if (N % 96 == 0 && K % 96 == 0) p.ntw = 6;
  else if (N % 128 == 0 && K % 128 == 0) p.ntw = 8;
  else return p;  // not supported: generic kernel
  const int wt = 16 * p.ntw, nt = N / wt, kt = K / wt;
  pick_wave_split(nt, kt, p.wn, p.wk);
  // ring depth that fits 160 KB, capped at 3 stages: the depth does not change the stage-0
  // streaming rate (measured 3-6 flat, r04d), and the smaller LDS footprint (<= 96 KB) lets the
  // kernel share CUs with the input-gradient kernels it overlaps on the side stream (+0.8 %)
  const int nw = p.wn * p.wk == 3 ? 3 : 4;
  const int rs = 32 * (nw / (p.wn * p.wk));
  {
    const int sa = (p.wn * wt + 8) / 8, sb = (p.wk * wt + 8) / 8;
    const int ins = ((rs * (sa + sb) + 63) / 64 + nw - 1) / nw * nw;
    const int nst = (int)((160L * 1024) / ((long)ins * 64 * 16));
    if (nst < 3) {  // ring too shallow: generic kernel
      p.ntw = 0;
      return p;
    }
    p.nst = 3;
  }
  const long tiles = (long)(nt / p.wn) * (kt / p.wk);
  // workgroup target: one per CU (no tail wave), long row ranges (128 / 512 measured no better
  // for the stage 2-3 shapes, r03x)
  long s = ((MSU_EXP & 512) ? 128 : 256) / tiles;  // (ablation 512: half the splits)
  const long max_s = (M + 8 * rs - 1) / (8 * rs);  // at least 8 stages per split
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  p.S = (int)s;
  return p;
}

template <typename T, int NTW, int WN, int WK, int NST>
void launch_wave(dim3 grid, const bf16_t* dY, const bf16_t* X, float* part, float* dbpart, long M, int N, int K,
                 long mchunk, int ntiles, hipStream_t st) {
  constexpr int NW = wgrad_nw<WN, WK>();
  constexpr int WM = NW / (WN * WK), WT = 16 * NTW, RS = 32 * WM;
  constexpr int SLOTS = RS * ((WN * WT + 8) / 8 + (WK * WT + 8) / 8);
  constexpr int INS = ((SLOTS + 63) / 64 + NW - 1) / NW * NW;
  constexpr size_t lds = (size_t)NST * INS * 64 * 16;
  if constexpr (lds <= 160 * 1024) {  // ring depths the plan never picks are not instantiated
    auto kern = wgrad_wave_kernel<T, NTW, WN, WK, NST>;
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    hipLaunchKernelGGL(kern, grid, dim3(64 * NW), lds, st, dY, X, part, dbpart, M, N, K, mchunk, ntiles);
  }
}

template <typename T>
int run_wave(const WavePlan& p, const bf16_t* dY, const bf16_t* X, float* part, float* dbpart, long M, int N, int K,
             hipStream_t st) {
  const int wt = 16 * p.ntw, nw = p.wn * p.wk == 3 ? 3 : 4, wm = nw / (p.wn * p.wk), rs = 32 * wm;
  long mchunk = (M + p.S - 1) / p.S;
  mchunk = (mchunk + rs - 1) / rs * rs;
  const int ntiles = (N / (p.wn * wt)) * (K / (p.wk * wt));
  const dim3 grid((unsigned)(ntiles * p.S));
#define MSU_WAVE(NTW, WN, WK)                                                                                        \
  if (p.ntw == NTW && p.wn == WN && p.wk == WK) {                                                                   \
    launch_wave<T, NTW, WN, WK, 3>(grid, dY, X, part, dbpart, M, N, K, mchunk, ntiles, st);                         \
    return 0;                                                                                                       \
  }
  MSU_WAVE(6, 1, 1) MSU_WAVE(6, 2, 1) MSU_WAVE(6, 4, 1) MSU_WAVE(6, 1, 2) MSU_WAVE(6, 2, 2) MSU_WAVE(6, 1, 4)
  MSU_WAVE(6, 3, 1) MSU_WAVE(6, 1, 3)
  MSU_WAVE(8, 1, 1) MSU_WAVE(8, 2, 1) MSU_WAVE(8, 4, 1) MSU_WAVE(8, 1, 2) MSU_WAVE(8, 2, 2) MSU_WAVE(8, 1, 4)
  MSU_WAVE(8, 3, 1) MSU_WAVE(8, 1, 3)
#undef MSU_WAVE
  return -3;
}

inline int tile_of(int N, int K) { return (N % 128 == 0 && K % 128 == 0) ? 128 : 96; }

inline int pick_splits(long M, int N, int K) {
  const int bt = tile_of(N, K);
  const long tiles = (long)((N + bt - 1) / bt) * ((K + bt - 1) / bt);
  long s = (1024 + tiles - 1) / tiles;
  const long max_s = (M + 511) / 512;  // keep >= 512 rows per split
  if (s > max_s) s = max_s;
  if (s < 1) s = 1;
  return (int)s;
}

}  // namespace

extern "C" {

int msu_wgrad_splits(long M, int N, int K) { return pick_splits(M, N, K); }

long msu_wgrad_workspace(long M, int N, int K) {
  const int S = pick_splits(M, N, K);
  long ws = (long)S * N * K + (long)S * N;
  const WavePlan p = wave_plan(M, N, K);
  if (p.ntw) {
    const long w2 = (long)p.slabs() * N * K + (long)p.slabs() * N;
    if (w2 > ws) ws = w2;
  }
  return ws;
}

// dW [N][K] f32 with row stride ldw >= K (overwritten, or accumulated when accumulate != 0;
// ldw > K: a column slice of a wider weight gradient, e.g. one input half of a skip-fusion
// Linear), db [N] f32 (may be null).
int msu_linear_wgrad_ld(int dtype, const void* dY, const void* X, float* dW, long ldw, float* db,
                        float* workspace, long M, int N, int K, int accumulate, void* stream) {
  if (N % 8 || K % 8 || M < 0 || ldw < K) return -2;  // 16-B staging chunks
  hipStream_t st = (hipStream_t)stream;
  // ablation build only (tools/build_exp.sh gemm_wgrad 256): no weight-gradient work at all, to
  // time what the side stream's weight gradients cost the step (results WRONG by design)
  if constexpr ((MSU_EXP & 256) != 0) return 0;
  if (M == 0) {
    if (!accumulate) hipMemset2DAsync(dW, sizeof(float) * ldw, 0, sizeof(float) * K, N, st);
    if (db && !accumulate) hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return MSU_CHECK_LAUNCH();
  }
  if (msu_is16(dtype)) {
    const WavePlan p = wave_plan(M, N, K);
    if (p.ntw) {
      float* part = workspace;
      float* dbpart = db ? workspace + (long)p.slabs() * N * K : nullptr;
      int rc = -3;
      MSU_DISPATCH16(dtype, T, rc = run_wave<T>(p, (const bf16_t*)dY, (const bf16_t*)X, part, dbpart, M, N, K, st));
      if (rc) return rc;
      const ColSeg segs[2] = {{part, (long)N * K, (long)N * K, dW, K, ldw}, {dbpart, N, N, db}};
      colsum_multi(segs, db ? 2 : 1, p.slabs(), accumulate, st);
      return MSU_CHECK_LAUNCH();
    }
  }
  const int S = pick_splits(M, N, K);
  long mchunk = (M + S - 1) / S;
  mchunk = (mchunk + BM - 1) / BM * BM;
  float* part = workspace;
  float* dbpart = db ? workspace + (long)S * N * K : nullptr;
  const int bt = tile_of(N, K);
  const dim3 grid((unsigned)(((N + bt - 1) / bt) * ((K + bt - 1) / bt)), (unsigned)S);
  MSU_DISPATCH(dtype, T,
    if (bt == 96)
      hipLaunchKernelGGL((wgrad_kernel<T, 3>), grid, dim3(256), 0, st, (const T*)dY, (const T*)X, part, dbpart, M,
                         N, K, mchunk);
    else
      hipLaunchKernelGGL((wgrad_kernel<T, 4>), grid, dim3(256), 0, st, (const T*)dY, (const T*)X, part, dbpart, M,
                         N, K, mchunk));
  const ColSeg segs[2] = {{part, (long)N * K, (long)N * K, dW, K, ldw}, {dbpart, N, N, db}};
  colsum_multi(segs, db ? 2 : 1, S, accumulate, st);
  return MSU_CHECK_LAUNCH();
}

int msu_linear_wgrad(int dtype, const void* dY, const void* X, float* dW, float* db, float* workspace,
                     long M, int N, int K, int accumulate, void* stream) {
  return msu_linear_wgrad_ld(dtype, dY, X, dW, K, db, workspace, M, N, K, accumulate, stream);
}

}  // extern "C"
