// 2-D tiled 16-bit GEMM on 32x32x16 MFMA for the Linear layers of stages 1-3 (and their input
// gradients): Y[M][N] = epi(A[M][K] . W[N][K]^T + bias), A and W both K-contiguous ("NT"), f32
// accumulation.  The token GEMM (gemm_tok.h) keeps the whole weight in LDS and streams the
// tokens, which is what the HBM-bound stage-0 shapes want; at stages 1-3 the weights are wide
// (up to 3072 x 768) and the token counts small (8k-131k), so the work is MFMA-heavier and
// tiled both ways here:
//   * 128 x 128 output tile per 4-wave workgroup (waves 2 x 2, 64 x 64 each, four 32 x 32
//     accumulators), K steps of 64 (or 32);
//   * A and W tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4), double-buffered: the
//     next K step's tiles are in flight while this one's MFMAs run (counted vmcnt + raw
//     s_barrier, so the barrier does not drain the prefetch);
//   * the LDS image is lane-linear (the DMA's constraint) with the 16-B k-chunks of each row
//     permuted by the row's position in its 256-B bank row: the fragment reads (16 rows x 16 B
//     per quarter-wave) then hit every bank group once -- the permutation is applied to the
//     per-lane GLOBAL address;
//   * accumulators hold C^T tiles (W rows on the accumulator rows, tokens on the lanes), so a
//     permlane32 swap gives each lane 8 consecutive output columns of its token row: 16-B
//     stores, bias / GELU / GELU' epilogues fused (the token GEMM's EPI_* semantics);
//   * blocks are mapped XCD-contiguously with the N tiles of one M tile adjacent: the A rows of
//     a tile are fetched from HBM once per XCD and re-read from its L2 by the other N tiles.
// Model call sites: network/model_parts.py Mlp / WindowAttention qkv / proj, PatchMerging
// reduction, PatchExpand expand, concat_back_dim (via ops.linear / ops.mlp) when routed in
// (ops.gemm_route, MSU_GEMM_ROUTE=nt): alone it beats hipBLASLt on most stage 1-3 shapes, inside
// the overlapped training step it has not (GEMM routing).
#include <cstring>

#include "common.h"

namespace {

constexpr int BM = 128, BN = 128;
enum { EPI_PLAIN = 0, EPI_GELU_DUAL = 1, EPI_GELU_GRAD = 2 };

struct NtArgs {
  const bf16_t* A;     // [M][K]
  const bf16_t* W;     // [N][K]
  const float* bias;   // [N] or null
  bf16_t* Y;           // [M][N]
  bf16_t* Y2;          // [M][N] (GELU_DUAL: GELU(Y))
  const bf16_t* H;     // [M][N] (GELU_GRAD: pre-activation)
  int M, N, K;
  int tiles_n;
};

// Tile geometry for a K step of BK: CH = BK / 8 16-B chunks per row; a 256-B LDS bank row
// holds 128 / BK rows, and chunk c of row r is stored at chunk c ^ ((r >> SH) & (CH - 1)), so a
// half-wave's 16 fragment rows (16 B each) land on 16 distinct bank groups.
template <int BK>
struct NtTile {
  static constexpr int CH = BK / 8, SH = BK == 64 ? 1 : 2;
  // LDS element offset of k-chunk `chunk` (8 elements) of tile row `row`
  static MSU_DEV int off(int row, int chunk) { return row * BK + ((chunk ^ ((row >> SH) & (CH - 1))) << 3); }
  // One 128 x BK operand tile -> LDS: 128 * CH 16-B slots, CH / 2 per thread.  Slot p = c*256 +
  // tid is row p / CH, LDS chunk p % CH, which holds the global chunk that off() puts there; rows
  // past the tensor re-read its last row (their results are never stored).
  static MSU_DEV void stage(const bf16_t* __restrict__ src, int row0, int rows, int K, int k0, bf16_t* tile,
                            int tid) {
    const int wave = tid >> 6;
#pragma unroll
    for (int c = 0; c < CH / 2; ++c) {
      const int p = c * 256 + tid;
      const int row = p / CH, g = (p % CH) ^ ((row >> SH) & (CH - 1));
      int r = row0 + row;
      if (r >= rows) r = rows - 1;
      glds16(src + (size_t)r * K + k0 + 8 * g, tile + (c * 256 + wave * 64) * 8);
    }
  }
  // 32-row fragment: lane l -> row row0 + (l & 31), k = 16 ks + 8 (l >> 5) .. +7
  static MSU_DEV bf16x8 frag(const bf16_t* tile, int row0, int ks, int lane) {
    const int row = row0 + (lane & 31);
    return *reinterpret_cast<const bf16x8*>(tile + off(row, 2 * ks + (lane >> 5)));
  }
};

// W given as [K][N] (N-contiguous: the forward weight [N_fwd][K_fwd] of an input-gradient GEMM,
// dX = dY . W, read without a transposed copy).  Its BK x 128 tile is staged as a [k][n] image
// (256-B rows); 16-B chunk c of row r sits at chunk c ^ 4(r & 3), so the four rows a half-wave's
// transposed read covers fall on four different 64-B bank groups.
struct KnTile {
  static MSU_DEV int off(int row, int col) { return row * BN + ((((col >> 3) ^ (4 * (row & 3)))) << 3) + (col & 7); }
  // 64 x 128 tile: 1024 16-B slots, 4 per thread; columns past N re-read column n0
  static MSU_DEV void stage(const bf16_t* __restrict__ W, int n0, int N, int k0, bf16_t* tile, int tid) {
    const int wave = tid >> 6;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int p = c * 256 + tid;
      const int row = p >> 4, lc = (p & 15) ^ (4 * (row & 3));
      int n = n0 + 8 * lc;
      if (n >= N) n = n0;
      glds16(W + (size_t)(k0 + row) * N + n, tile + (c * 256 + wave * 64) * 8);
    }
  }
  // 32-column fragment (the MFMA A operand): lane l -> column col0 + (l & 31), element e -> k =
  // 16 ks + 8 (l >> 5) + e, as two ds_read_b64_tr_b16 (4 k rows x 4 columns per lane group)
  static MSU_DEV bf16x8 frag(const bf16_t* tile, int col0, int ks, int lane) {
    typedef short v4s __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
    const int col = col0 + 16 * (g & 1) + 4 * p;
    const int row = 16 * ks + 8 * h + q;
    v4s both[2] = {__builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + off(row, col))),
                   __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(tile + off(row + 4, col)))};
    return *reinterpret_cast<bf16x8*>(both);
  }
};

// Runtime-selected s_waitcnt vmcnt(n * PER), n in [0, 2] (DMA steps allowed to stay in flight)
template <int PER>
MSU_DEV void wait_steps(int n) {
  if (n >= 2) wait_vmcnt<2 * PER>();
  else if (n == 1) wait_vmcnt<PER>();
  else wait_vmcnt<0>();
}

// NST-stage LDS ring of K steps (prefetch distance NST - 1, one barrier per K step): the
// short-K stage 1-3 shapes (K = 192..768: 3-24 steps) otherwise wait out a DMA round trip per
// step.  Fragments of k-slice ks + 1 are read before the MFMAs of ks.
template <typename T, int EPI, int BK, int NST, bool WKN>
__global__ void __launch_bounds__(256, 2) gemm_nt_kernel(NtArgs a) {
  typedef NtTile<BK> Tl;
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  static_assert(!WKN || BK == 64, "[K][N] weights: 64-deep K steps");
  constexpr int KSL = BK / 16;  // 16-wide k slices per step
  __shared__ __attribute__((aligned(16))) bf16_t lds[NST][2][BM * BK];  // [stage][A | W]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;  // this wave's 64 x 64 quarter (tokens, columns)
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = t / a.tiles_n, nt = t - mt * a.tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int nk = a.K / BK;  // K % 64 == 0 (nt_shape_ok)

  f32x16 acc[2][2];  // [column tile ni][token tile mi]: C^T, W rows on the accumulator rows
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0};

#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) {
      Tl::stage(a.A, m0, a.M, a.K, s * BK, lds[s][0], tid);
      if constexpr (WKN) KnTile::stage(a.W, n0, a.N, s * BK, lds[s][1], tid);
      else Tl::stage(a.W, n0, a.N, a.K, s * BK, lds[s][1], tid);
    }
  for (int kt = 0; kt < nk; ++kt) {
    // this step's DMAs done; those of steps kt+1 .. kt+NST-2 may stay in flight
    wait_steps<Tl::CH>(min(NST - 2, nk - 1 - kt));
    __builtin_amdgcn_s_barrier();  // every wave's DMA of step kt has landed, and every wave is
    asm volatile("" ::: "memory");  // done reading step kt-1's stage (refilled below)
    if (kt + NST - 1 < nk) {
      const int sn = (kt + NST - 1) % NST;
      Tl::stage(a.A, m0, a.M, a.K, (kt + NST - 1) * BK, lds[sn][0], tid);
      if constexpr (WKN) KnTile::stage(a.W, n0, a.N, (kt + NST - 1) * BK, lds[sn][1], tid);
      else Tl::stage(a.W, n0, a.N, a.K, (kt + NST - 1) * BK, lds[sn][1], tid);
    }
    const bf16_t* ta = lds[kt % NST][0];
    const bf16_t* tw = lds[kt % NST][1];
    bf16x8 fw[2][2], fx[2][2];
    auto rd = [&](int ks, int set) {
      if constexpr (WKN) {
        fw[set][0] = KnTile::frag(tw, 64 * wn, ks, lane);
        fw[set][1] = KnTile::frag(tw, 64 * wn + 32, ks, lane);
      } else {
        fw[set][0] = Tl::frag(tw, 64 * wn, ks, lane);
        fw[set][1] = Tl::frag(tw, 64 * wn + 32, ks, lane);
      }
      fx[set][0] = Tl::frag(ta, 64 * wm, ks, lane);
      fx[set][1] = Tl::frag(ta, 64 * wm + 32, ks, lane);
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < KSL; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < KSL) rd(ks + 1, cur ^ 1);
      acc[0][0] = Fmt16<T>::mma32(fw[cur][0], fx[cur][0], acc[0][0]);
      acc[0][1] = Fmt16<T>::mma32(fw[cur][0], fx[cur][1], acc[0][1]);
      acc[1][0] = Fmt16<T>::mma32(fw[cur][1], fx[cur][0], acc[1][0]);
      acc[1][1] = Fmt16<T>::mma32(fw[cur][1], fx[cur][1], acc[1][1]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // epilogue: lane (l & 31) is token m; after the swap, 8 consecutive columns per store
  const int hh = lane >> 5;
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int m = m0 + 64 * wm + 32 * mi + (lane & 31);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
#pragma unroll
      for (int g0 = 0; g0 < 4; g0 += 2) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(acc[ni][mi][4 * g0 + i]),
                                                          __float_as_uint(acc[ni][mi][4 * g0 + 4 + i]), false, false);
          v[i] = __uint_as_float(r[0]);
          v[4 + i] = __uint_as_float(r[1]);
        }
        const int n = n0 + 64 * wn + 32 * ni + 8 * g0 + 8 * hh;
        if (m >= a.M || n >= a.N) continue;
        if (a.bias) {
          const float4 b0 = *reinterpret_cast<const float4*>(a.bias + n);
          const float4 b1 = *reinterpret_cast<const float4*>(a.bias + n + 4);
          v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
          v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        const size_t off = (size_t)m * a.N + n;
        if constexpr (EPI == EPI_GELU_GRAD) {
          const u32x4 hv = *reinterpret_cast<const u32x4*>(a.H + off);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(hv[i]));
            v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(hv[i]));
          }
        }
        const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
        *reinterpret_cast<u32x4*>(a.Y + off) = pk;
        if constexpr (EPI == EPI_GELU_DUAL) {
          // GELU of the rounded pre-activation, as the unfused GELU kernel would see it
          float gv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) gv[i] = gelu_fast(round16<T>(v[i]));
          const u32x4 pg = {pack2<T>(gv[0], gv[1]), pack2<T>(gv[2], gv[3]), pack2<T>(gv[4], gv[5]),
                            pack2<T>(gv[6], gv[7])};
          *reinterpret_cast<u32x4*>(a.Y2 + off) = pg;
        }
      }
    }
  }
}

bool nt_shape_ok(long M, int N, int K) {
  return M > 0 && M < (1L << 31) && N > 0 && N % 32 == 0 && K > 0 && K % 64 == 0 && (long)M * N < (1L << 40);
}

// Ring configuration (A/B switch MSU_NT_CFG = BKxNST): 64x2 (default: 64 KB of LDS, one K step
// in flight), 32x4 (64 KB, three steps in flight), 32x3 (48 KB: three workgroups per CU).  The
// deeper rings measured 2-15 % slower alone (tools/nt_cfg_ab.sh): the per-step DMA latency is
// not what bounds these tiles.
int nt_cfg() {
  static const int cfg = [] {
    const char* e = getenv("MSU_NT_CFG");
    if (e && !strcmp(e, "32x4")) return 324;
    if (e && !strcmp(e, "32x3")) return 323;
    return 642;
  }();
  return cfg;
}

template <typename T, int BK, int NST, bool WKN>
void launch_nt(int epi, long tiles, const NtArgs& a, hipStream_t st) {
  switch (epi) {
    case EPI_PLAIN: hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_PLAIN, BK, NST, WKN>), dim3((unsigned)tiles), dim3(256), 0, st, a); break;
    case EPI_GELU_DUAL: hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_GELU_DUAL, BK, NST, WKN>), dim3((unsigned)tiles), dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_GELU_GRAD, BK, NST, WKN>), dim3((unsigned)tiles), dim3(256), 0, st, a); break;
  }
}

int nt_launch(int dtype, const void* A, const void* W, const float* bias, void* Y, void* Y2, const void* H, long M,
              int N, int K, int epi, void* stream, bool wkn) {
  if (!msu_is16(dtype)) return -3;
  if (!nt_shape_ok(M, N, K)) return -2;
  if (epi == EPI_GELU_DUAL && (Y2 == nullptr || bias == nullptr)) return -3;
  if (epi == EPI_GELU_GRAD && (H == nullptr || bias != nullptr)) return -3;
  if (epi < 0 || epi > 2) return -3;
  NtArgs a;
  a.A = (const bf16_t*)A;
  a.W = (const bf16_t*)W;
  a.bias = bias;
  a.Y = (bf16_t*)Y;
  a.Y2 = (bf16_t*)Y2;
  a.H = (const bf16_t*)H;
  a.M = (int)M;
  a.N = N;
  a.K = K;
  a.tiles_n = (N + BN - 1) / BN;
  const long tiles = (long)((M + BM - 1) / BM) * a.tiles_n;
  hipStream_t st = (hipStream_t)stream;
  MSU_DISPATCH16(dtype, T,
    if (wkn) launch_nt<T, 64, 2, true>(epi, tiles, a, st);
    else if (nt_cfg() == 642) launch_nt<T, 64, 2, false>(epi, tiles, a, st);
    else if (nt_cfg() == 323) launch_nt<T, 32, 3, false>(epi, tiles, a, st);
    else launch_nt<T, 32, 4, false>(epi, tiles, a, st));
  return MSU_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

// Whether msu_nt_gemm covers this shape (K % 64, N % 32).
int msu_nt_gemm_supported(long M, int N, int K) { return nt_shape_ok(M, N, K) ? 1 : 0; }

// Y[M][N] = epi(A . W^T + bias), 16-bit in / out (dtype 1 bf16, 2 f16), f32 accumulation.
// epi 0: plain (+ bias when given); 1: Y = H and Y2 = GELU(H) (needs bias); 2: Y = (A . W^T) *
// GELU'(H) (no bias).  Same semantics as msu_tok_gemm without the split-A input.
int msu_nt_gemm(int dtype, const void* A, const void* W, const float* bias, void* Y, void* Y2, const void* H,
                long M, int N, int K, int epi, void* stream) {
  return nt_launch(dtype, A, W, bias, Y, Y2, H, M, N, K, epi, stream, false);
}

// Same with the weight given as Wk[K][N] (Y = epi(A . Wk + bias)): the input gradient of a Linear,
// dX[M][K_fwd] = dY[M][N_fwd] . W[N_fwd][K_fwd], straight from the forward weight (no W^T copy).
int msu_nt_gemm_kn(int dtype, const void* A, const void* Wk, const float* bias, void* Y, void* Y2, const void* H,
                   long M, int N, int K, int epi, void* stream) {
  return nt_launch(dtype, A, Wk, bias, Y, Y2, H, M, N, K, epi, stream, true);
}

}  // extern "C"
