// Token GEMM: Y[M][N] = epi(A[M][K] . W[N][K]^T (+ bias)) for the Linear layers of the Swin
// blocks and MS-UNet glue (bf16 or f16 in / out, f32 accumulate).
//
// Replaces the forward and input-gradient GEMMs of torchvision's block Linears (qkv / proj /
// mlp.0 / mlp.3, called from model_parts.py:170 / :538), PatchMerging.reduction
// (model_parts.py:72, :96), PatchExpand.expand (:379, :399), concat_back_dim (:639-641,
// :793, :805, :824), FinalPatchExpand_X4_V2.expand (:443, :459) and PatchEmbed.proj as an
// im2col GEMM (:211, :222).  Input gradients run the same kernel with the transposed weight
// (dX = dY . W  =  dY . (W^T)^T).
//
// Shape class: M = tokens (up to 8 x 65536), N, K = small multiples of the embed width, so
// W is tens of KB while A / Y are hundreds of MB -- at stages 0-1 the product is HBM-bound
// by 4-5x over MFMA.  Hence a weight-stationary streaming design:
//   * a workgroup (4 waves) keeps an NC-column chunk of W ([NC][K+8] bf16) and its bias in
//     LDS for its whole life (persistent grid, one or two workgroups per CU);
//   * every wave streams its own 32-row tiles of A through a private NST-deep LDS ring fed by
//     global_load_lds_dwordx4 (LDS-DMA; rows padded by one 16-B slot whose lane re-reads the
//     row's first chunk) -- no workgroup barriers after the W load, only hand-counted vmcnt
//     waits (the only other loads in the loop, GELU_GRAD's H, are inline asm, counted too);
//   * v_mfma_f32_32x32x16_bf16 with W as the A operand and the token rows as the B operand,
//     so each lane ends up owning one token row (output "row per lane"); pairs of 8-column
//     groups are exchanged with v_permlane32_swap so every store is a 16-B dwordx4;
//   * epilogues: + bias; GELU_DUAL writes both the pre-activation H and GELU(H) (mlp.0: H
//     is what mlp.1's backward needs, GELU(H) what mlp.3 reads -- the standalone GELU
//     kernels disappear); GELU_GRAD multiplies by GELU'(H) (mlp.3's input gradient becomes
//     mlp.0's output gradient in the same pass);
//   * CONCAT: columns [0, K1) of A come from A and [K1, K) from A2 -- torch.cat([x, skip])
//     of the skip fusion (model_parts.py:792-794) is never materialised;
//   * blocks that own different column chunks of the same rows sit on the same XCD and walk
//     the rows in the same order, so the chunk re-reads of A hit that XCD's L2.
//
// The kernel template lives here; gemm_tok_k{48,96,128}.hip instantiate it per stage depth
// (parallel compilation) and gemm_tok.hip holds the planner and the C-ABI entry points.
#pragma once
#include "common.h"

namespace msu_tok {

constexpr int RT = 32;  // token rows per tile (one 32x32 MFMA B operand)
// waves per workgroup: a template parameter NW (4, or 8 when the W image leaves room for
// eight 2-deep rings: two waves per SIMD overlap one's epilogue with the other's MFMAs)

enum { EPI_PLAIN = 0, EPI_GELU_DUAL = 1, EPI_GELU_GRAD = 2 };

struct TokArgs {
  const bf16_t* A;   // [M][K1] (or [M][K] when A2 == nullptr)
  const bf16_t* A2;  // [M][K - K1] or nullptr
  const bf16_t* W;   // [N][K]
  const float* bias; // [N] or nullptr
  bf16_t* Y;         // [M][N]
  bf16_t* Y2;        // [M][N] GELU(Y) (GELU_DUAL)
  const bf16_t* H;   // [M][N] pre-activation (GELU_GRAD)
  long M;
  int N, K, K1;
  int nchunk;        // N / NC
  int rgroups;       // row groups (gridDim.x / nchunk)
};

// Storage pointers are raw 16-bit words (bf16_t); the kernel's T (bf16_t / f16_t) says how
// they are interpreted (conversions, MFMA opcode).

template <int KC>
struct StageGeom {
  static constexpr int SR = KC / 8 + 1;               // 16-B slots per row (incl. one pad slot)
  static constexpr int LD = SR * 8;                   // LDS row stride (elements)
  static constexpr int SLOTS = RT * SR;
  static constexpr int INS = (SLOTS + 63) / 64;       // DMA instructions per stage per wave
  static constexpr int BYTES = INS * 64 * 16;         // LDS bytes per stage
};

// 16-B global load the compiler does not track (counted by hand against the DMA ring)
MSU_DEV u32x4 load16_untracked(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// LDS accesses the compiler does not see: the epilogue stages through a ring slot while LDS
// DMAs are pending on other slots, and a visible ds_read there would be preceded by a
// conservative vmcnt(0) (pending LDS-DMA alias) that drains the ring.
MSU_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)(p);
}
MSU_DEV void ds_write16_untracked(uint32_t addr, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1" : : "v"(addr), "v"(v) : "memory");
}
MSU_DEV u32x4 ds_read16_untracked(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

// output column block staged per round: the widest of 128/96/64/32 dividing NC whose
// 32-row image (row stride CW*2 + 16 B) fits in one ring stage
template <int KC, int NC>
constexpr int stage_cols() {
  constexpr int bytes = StageGeom<KC>::BYTES;
  return (NC % 128 == 0 && 32 * (128 * 2 + 16) <= bytes) ? 128
       : (NC % 96 == 0 && 32 * (96 * 2 + 16) <= bytes)   ? 96
       : (NC % 64 == 0 && 32 * (64 * 2 + 16) <= bytes)   ? 64 : 32;
}

template <typename T, int KC, int NC, int NST, int NW, int EPI, bool BIAS, bool CONCAT>
__global__ void __launch_bounds__(64 * NW) tokgemm_kernel(TokArgs a) {
  constexpr int WPB = NW;
  using G = StageGeom<KC>;
  constexpr int NT = NC / 32;                 // 32-column MFMA tiles per chunk
  constexpr int NPAIR = NC / 16;              // 16-column store pairs
  constexpr bool GGRAD = EPI == EPI_GELU_GRAD;
  constexpr int E = NPAIR * (EPI == EPI_GELU_DUAL ? 2 : 1);  // stores per tile
  constexpr int HL = GGRAD ? NPAIR : 0;                       // H loads per tile
  static_assert(NC % 32 == 0 && KC % 16 == 0 && (NST == 2 || NST == 3), "tile shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int K = a.K;
  const int LDW = K + (BIAS ? 16 : 0) + 8;  // [w(n, 0..K-1) | bias_hi, bias_lo, 0 x 14 | pad]
  bf16_t* sW = reinterpret_cast<bf16_t*>(smem_raw);
  unsigned char* ring_base = smem_raw + (size_t)NC * LDW * 2;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // block -> (chunk, row group); blocks of one row group share an XCD (round-robin dispatch)
  const int b = blockIdx.x, xcd = b & 7, local = b >> 3;
  const int chunk = local % a.nchunk;
  const int rg = (local / a.nchunk) * 8 + xcd;
  const int n0 = chunk * NC;

  // ---- W chunk + bias -> LDS (once)
  {
    const int cpr = K / 8;  // 16-B chunks per weight row
    for (int i = tid; i < NC * cpr; i += 64 * WPB) {
      const int r = i / cpr, c = i - r * cpr;
      *reinterpret_cast<uint4*>(sW + r * LDW + 8 * c) =
          *reinterpret_cast<const uint4*>(a.W + (long)(n0 + r) * K + 8 * c);
    }
    if (BIAS) {
      // bias as an extra k-block: 16-bit hi + lo parts (~16 / 22 significant bits for bf16 /
      // f16) times a ones column
      for (int i = tid; i < NC * 2; i += 64 * WPB) {
        const int r = i >> 1, half = i & 1;
        uint4 q = make_uint4(0, 0, 0, 0);
        if (half == 0) {
          const float bv = a.bias[n0 + r];
          const float hi = round16<T>(bv);
          q.x = pack2<T>(hi, bv - hi);
        }
        *reinterpret_cast<uint4*>(sW + r * LDW + K + 8 * half) = q;
      }
    }
  }
  __syncthreads();

  // ---- this wave's tiles: t = ws, ws + S, ...; stage st = (tile st / nkc, k chunk st % nkc)
  const long ntiles = (a.M + RT - 1) / RT;
  const int S = a.rgroups * WPB;
  const int ws = rg * WPB + wave;
  const int nkc = K / KC;
  const long my_tiles = ws < ntiles ? (ntiles - ws + S - 1) / S : 0;
  const long total = my_tiles * nkc;
  if (total == 0) return;
  unsigned char* ring = ring_base + (size_t)wave * NST * G::BYTES;

  // per-lane DMA slot geometry (fixed): row within the tile and 16-B chunk within the stage
  int srow[G::INS], scol[G::INS];
#pragma unroll
  for (int i = 0; i < G::INS; ++i) {
    const int s = i * 64 + lane;
    const int row = s / G::SR, c = s - row * G::SR;
    srow[i] = s < G::SLOTS ? row : RT;            // RT = "no row": read the zero region
    scol[i] = c < G::SR - 1 ? 8 * c : 0;          // pad slot re-reads the row's first chunk
  }
  const int lda = CONCAT ? a.K1 : K, K2 = K - a.K1;
  // DMA of the next stage into its ring slot; stages are issued in order, so the (tile, k
  // chunk, slot) of the next one advance incrementally (stages past the end load zeros:
  // the counts stay uniform)
  long i_ti = 0;
  int i_kc = 0, i_slot = 0;
  auto issue = [&]() __attribute__((always_inline)) {
    unsigned char* dst = ring + i_slot * G::BYTES;
    const long m0 = (ws + i_ti * (long)S) * RT;
    const int kc0 = i_kc * KC;
    const bool live = i_ti < my_tiles;
    if (++i_kc == nkc) { i_kc = 0; ++i_ti; }
    if (++i_slot == NST) i_slot = 0;
#pragma unroll
    for (int i = 0; i < G::INS; ++i) {
      const long m = m0 + srow[i];
      const void* src;
      if (live && srow[i] < RT && m < a.M) {
        const int k = kc0 + scol[i];
        src = (CONCAT && k >= a.K1) ? (const void*)(a.A2 + m * K2 + (k - a.K1)) : (const void*)(a.A + m * lda + k);
      } else {
        src = zero_src(i * 64 + lane);
      }
      glds16(src, dst + (size_t)i * 1024);
    }
  };

  f32x16 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[n][r] = 0.f;

  // fragment addressing: lane l reads row (l & 31), k offset 8 * (l >> 5)
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  const bf16_t* wfrag = sW + fr * LDW + fk;
  u32x4 hv[GGRAD ? NPAIR : 1];

#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue();
  long st = 0;
  int c_slot = 0, last_slot = 0;
  bool ragged = false;  // a tile that ended within the last two stages stored fewer than E rows
  for (long ti = 0; ti < my_tiles; ++ti) {
    const long mrow = (ws + ti * (long)S) * RT + fr;
    for (int kc = 0; kc < nkc; ++kc, ++st) {
      // ---- wait for stage st: VM ops retire in issue order; the ops younger than DMA(st)
      // are the later DMAs plus the stores / H loads of tiles that ended in between.  A tile
      // cut by M skips whole store instructions, so after one the counts drop to zero (a count
      // above the ops really issued would let the wave read a stage whose DMA is in flight)
      const bool p1 = st >= 1 && kc == 0;                  // stage st-1 ended a tile
      const bool p2 = st >= 2 && (nkc == 1 || kc == 1);    // stage st-2 ended a tile
      if (ragged) {
        wait_vmcnt<0>();
      } else if constexpr (NST == 2) {
        if (p1) wait_vmcnt<(E > 63 ? 63 : E)>();
        else wait_vmcnt<0>();
      } else {
        constexpr int C00 = G::INS, C10 = G::INS + HL + E, C01 = G::INS + E, C11 = G::INS + HL + 2 * E;
        if (p1 && p2) wait_vmcnt<(C11 > 63 ? 63 : C11)>();
        else if (p1) wait_vmcnt<(C10 > 63 ? 63 : C10)>();
        else if (p2) wait_vmcnt<(C01 > 63 ? 63 : C01)>();
        else wait_vmcnt<C00>();
      }
      asm volatile("" ::: "memory");
      const bool last = kc == nkc - 1;
      if constexpr (GGRAD) {
        // H for this tile's epilogue, issued before the next DMA (waited for below)
        if (last) {
          const long mh = mrow < a.M ? mrow : a.M - 1;
#pragma unroll
          for (int p = 0; p < NPAIR; ++p)
            hv[p] = load16_untracked(a.H + mh * a.N + n0 + 16 * p + (lane >= 32 ? 8 : 0));
        }
      }
      issue();
      last_slot = c_slot;
      const bf16_t* afrag = reinterpret_cast<const bf16_t*>(ring + c_slot * G::BYTES) + fr * G::LD + fk;
      if (++c_slot == NST) c_slot = 0;
      const bf16_t* wk = wfrag + kc * KC;
#ifdef MSU_TOK_NOPIPE
#pragma unroll
      for (int kk = 0; kk < KC / 16; ++kk) {
        const bf16x8 bx = *reinterpret_cast<const bf16x8*>(afrag + 16 * kk);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const bf16x8 wx = *reinterpret_cast<const bf16x8*>(wk + n * 32 * LDW + 16 * kk);
          acc[n] = Fmt16<T>::mma32(wx, bx, acc[n]);
        }
      }
#else
      // MFMA j = (k slice kk, column tile n) in sequence, the W fragment of MFMA j + 2 and the
      // token fragment of slice kk + 1 read before MFMA j, the order pinned: the compiler's own
      // schedule read each W fragment right before its MFMA and waited lgkmcnt(0) on it, i.e.
      // every 32-cycle MFMA paid an LDS round trip
      {
        constexpr int NKK = KC / 16, NJ = NKK * NT;
        auto rdw = [&](int j) __attribute__((always_inline)) {
          return *reinterpret_cast<const bf16x8*>(wk + (j % NT) * 32 * LDW + 16 * (j / NT));
        };
        bf16x8 wr[3], bxr[2];
        bxr[0] = *reinterpret_cast<const bf16x8*>(afrag);
        wr[0] = rdw(0);
        if (NJ > 1) wr[1] = rdw(1);
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int kk = j / NT, n = j % NT;
          if (j + 2 < NJ) wr[(j + 2) % 3] = rdw(j + 2);
          if (n == 0 && kk + 1 < NKK) bxr[(kk + 1) & 1] = *reinterpret_cast<const bf16x8*>(afrag + 16 * (kk + 1));
          acc[n] = Fmt16<T>::mma32(wr[j % 3], bxr[kk & 1], acc[n]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#endif
      if (BIAS && last) {
        // + bias: the W image's bias k-block times a ones column (k = 0, 1 of lanes 0-31)
        const bf16x8 ones = lane < 32 ? splat8<T>(1.0f, 1.0f, 0.0f) : splat8<T>(0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const bf16x8 wx = *reinterpret_cast<const bf16x8*>(wfrag + K + n * 32 * LDW);
          acc[n] = Fmt16<T>::mma32(wx, ones, acc[n]);
        }
      }
    }

    ragged = mrow - fr + RT > a.M;  // (wave-uniform) this tile's stores are cut by M
    // ---- epilogue: lane owns token row mrow; pair p covers columns 16p .. 16p+15
    if constexpr (GGRAD) {
      // the H loads are older than the one DMA issued after them
      wait_vmcnt<G::INS>();
#pragma unroll
      for (int p = 0; p < NPAIR; ++p) asm volatile("" : "+v"(hv[p]));
    }
    // The results go out through the ring slot of the stage just consumed (free until the next
    // stage's DMA): round q writes columns [q*CW, (q+1)*CW) of the 32-row tile there as a
    // row-major image, reads it back linearly and stores whole CW*2-byte row segments (the
    // row-per-lane layout would store 32 rows x 32 B per instruction: 32-B L2 write requests).
    constexpr int CW = stage_cols<KC, NC>();
    constexpr int PPR = CW / 16;                  // pairs per round
    constexpr int RSTR = CW * 2 + 16;             // staged row stride (bytes)
    constexpr int CPR = CW / 8;                   // 16-B chunks per staged row
    constexpr int RD = RT * CPR / 64;             // linear 16-B reads per lane per round
    static_assert(RT * CPR % 64 == 0, "round image");
    const uint32_t sbase = lds_addr(ring + last_slot * G::BYTES);
    const long m0 = mrow - fr;
#pragma unroll
    for (int out = 0; out < (EPI == EPI_GELU_DUAL ? 2 : 1); ++out) {
      bf16_t* Yo = out == 0 ? a.Y : a.Y2;
#pragma unroll
      for (int q = 0; q < NC / CW; ++q) {
#pragma unroll
        for (int pp = 0; pp < PPR; ++pp) {
          const int p = q * PPR + pp;
          const int n = p >> 1, g0 = 2 * (p & 1);  // groups g0, g0+1 of MFMA tile n (r / 4)
          float v[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[n][4 * g0 + i]),
                                                            __float_as_uint(acc[n][4 * g0 + 4 + i]), false, false);
            v[i] = __uint_as_float(r[0]);
            v[4 + i] = __uint_as_float(r[1]);
          }
          if constexpr (GGRAD) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(hv[p][i]));
              v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(hv[p][i]));
            }
          }
          if (EPI == EPI_GELU_DUAL && out == 1) {
            // GELU of the rounded pre-activation, as the unfused GELU kernel would see it
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = gelu_fast(round16<T>(v[i]));
          }
          const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]),
                            pack2<T>(v[6], v[7])};
          ds_write16_untracked(sbase + fr * RSTR + (16 * pp + (lane >= 32 ? 8 : 0)) * 2, pk);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        u32x4 rv[RD];
#pragma unroll
        for (int i = 0; i < RD; ++i) {
          const int L = i * 64 + lane, row = L / CPR, c = L - row * CPR;
          rv[i] = ds_read16_untracked(sbase + row * RSTR + c * 16);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < RD; ++i) asm volatile("" : "+v"(rv[i]));
#pragma unroll
        for (int i = 0; i < RD; ++i) {
          const int L = i * 64 + lane, row = L / CPR, c = L - row * CPR;
          if (m0 + row < a.M)
            *reinterpret_cast<u32x4*>(Yo + (m0 + row) * a.N + n0 + q * CW + 8 * c) = rv[i];
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[n][r] = 0.f;
  }
  wait_vmcnt<0>();  // no DMA may still target LDS when the workgroup retires
}

// ------------------------------------------------------------------ host side
struct TokPlan {
  int kc = 0, nc = 0, nst = 0, nw = 4;
  size_t lds = 0;
  int nchunk = 0, grid = 0;
};

constexpr size_t LDS_MAX = 160 * 1024;



inline size_t plan_lds(int kc, int nc, int nst, int K, int nw = 4) {
  const size_t stage = (size_t)((RT * (kc / 8 + 1) + 63) / 64) * 1024;
  return (size_t)nc * (K + 16 + 8) * 2 + (size_t)nw * nst * stage;  // W image incl. bias block
}

template <typename T, int KC, int NC, int NST, int NW, int EPI, bool BIAS, bool CONCAT>
int launch_tok(const TokPlan& p, TokArgs a, hipStream_t st) {
  auto kern = tokgemm_kernel<T, KC, NC, NST, NW, EPI, BIAS, CONCAT>;
  static size_t attr = 0;
  if (attr < p.lds) {
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p.lds) != hipSuccess)
      return -4;
    attr = p.lds;
  }
  a.nchunk = p.nchunk;
  a.rgroups = p.grid / p.nchunk;
  hipLaunchKernelGGL(kern, dim3(p.grid), dim3(64 * NW), p.lds, st, a);
  return 0;
}

// epilogue variants instantiated per (KC, NC, NST); FULL = all five, else plain (+bias) only
template <typename T, int KC, int NC, int NST, int NW, bool FULL>
int dispatch_epi(const TokPlan& p, const TokArgs& a, int epi, bool bias, bool concat, hipStream_t st) {
#define MSU_TOK(E, B, C) \
  if (epi == E && bias == B && concat == C) return launch_tok<T, KC, NC, NST, NW, E, B, C>(p, a, st);
  MSU_TOK(EPI_PLAIN, true, false)
  MSU_TOK(EPI_PLAIN, false, false)
  if constexpr (FULL) {
    MSU_TOK(EPI_PLAIN, true, true)
    MSU_TOK(EPI_GELU_DUAL, true, false)
    MSU_TOK(EPI_GELU_GRAD, false, false)
  }
#undef MSU_TOK
  return -3;
}

template <typename T, int KC, bool FULL>
int dispatch_nc(const TokPlan& p, const TokArgs& a, int epi, bool bias, bool concat, hipStream_t st) {
#define MSU_NC(NC)                                                                                      \
  if (p.nc == NC) {                                                                                     \
    if (p.nst == 3) return dispatch_epi<T, KC, NC, 3, 4, FULL>(p, a, epi, bias, concat, st);           \
    if (p.nst == 2 && p.nw == 8) return dispatch_epi<T, KC, NC, 2, 8, FULL>(p, a, epi, bias, concat, st); \
    if (p.nst == 2) return dispatch_epi<T, KC, NC, 2, 4, FULL>(p, a, epi, bias, concat, st);           \
  }
  MSU_NC(384) MSU_NC(288) MSU_NC(256) MSU_NC(192) MSU_NC(128) MSU_NC(96) MSU_NC(64)
#undef MSU_NC
  return -3;
}

int dispatch_k96(int dtype, const TokPlan& p, const TokArgs& a, int epi, bool bias, bool concat, hipStream_t st);
int dispatch_k128(int dtype, const TokPlan& p, const TokArgs& a, int epi, bool bias, bool concat, hipStream_t st);
int dispatch_k48(int dtype, const TokPlan& p, const TokArgs& a, int epi, bool bias, bool concat, hipStream_t st);

}  // namespace msu_tok
