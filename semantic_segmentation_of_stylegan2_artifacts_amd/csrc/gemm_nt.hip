// 2-D tiled 16-bit GEMM on 32x32x16 MFMA for the Linear layers of stages 1-3 (and their input
// gradients): Y[M][N] = epi(A[M][K] . W[N][K]^T + bias), A and W both K-contiguous ("NT"), f32
// accumulation.  The token GEMM (gemm_tok.h) keeps the whole weight in LDS and streams the
// tokens, which is what the HBM-bound stage-0 shapes want; at stages 1-3 the weights are wide
// (up to 3072 x 768) and the token counts small (8k-131k), so the work is MFMA-heavier and
// tiled both ways here:
//   * 128 x 128 output tile per 4-wave workgroup (waves 2 x 2, 64 x 64 each, four 32 x 32
//     accumulators), K steps of 64 (or 32);
//   * A and W tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4), double-buffered: the
//     next K step's tiles are in flight while this one's MFMAs run (raw s_barrier);
//   * persistent: the workgroups walk their tiles as one flat sequence of K steps (the ring
//     runs across tile boundaries; see gemm_nt_kernel);
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
// reduction, PatchExpand expand, concat_back_dim (via ops.linear / ops.mlp), routed by
// ops.gemm_route for the stage 1-3 shapes the token GEMM does not take.
#include <cstdlib>
#include <cstring>
#include <utility>

#include "common.h"
#include "mfma_frag.h"

// MSU_EXP: ablation bits for timing experiments only (tools/build_exp.sh); 0 in every real build
#ifndef MSU_EXP
#define MSU_EXP 0
#endif

namespace {

constexpr int BN = 128, BK = 64;  // N tile and K step of the KN form
enum { EPI_PLAIN = 0, EPI_GELU_DUAL = 1, EPI_GELU_GRAD = 2 };

struct NtArgs {
  const bf16_t* A;     // [M][K] (or [M][K1] when A2 is set)
  const bf16_t* A2;    // null, or A's columns [K1, K): [M][K - K1] (the skip concatenation)
  const bf16_t* W;     // [N][K]
  const float* bias;   // [N] or null
  bf16_t* Y;           // [M][N]
  bf16_t* Y2;          // [M][N] (GELU_DUAL: GELU(Y))
  const bf16_t* H;     // [M][N] (GELU_GRAD: pre-activation)
  int M, N, K, K1;
  int tiles_m, tiles_n;
  int* tq;             // tile-queue slot (common.h; the two-stage kernel only) or null: static
};

// A ROWS x KB operand tile (K-contiguous rows, KB = 64 or 32) staged by NTHR threads.  A 256-B
// LDS bank row holds RPL = 128 / KB tile rows; chunk c of row r is stored at chunk c ^ ((r / RPL)
// % CH), so a half-wave's 16 fragment rows (16 B each) land on 16 distinct bank groups.  When the
// tile's 16-B slots are not a whole number of rounds of NTHR (192 rows x 4 chunks over 512
// threads), the last round is issued by the first FULLW waves only (wave-uniform).
template <int ROWS, int NTHR, int KB = 64>
struct RowTile {
  static constexpr int CH = KB / 8, RPL = 128 / KB;
  static constexpr int PER = (ROWS * CH + NTHR - 1) / NTHR;  // DMA instructions per thread (max)
  static constexpr int FULLW = (ROWS * CH - (PER - 1) * NTHR) / 64;  // waves issuing all PER
  static_assert((ROWS * CH) % 64 == 0 && KB % 32 == 0, "whole-wave DMA instructions");
  // DMA instructions of wave w
  static MSU_DEV constexpr int per_wave(int w) { return w < FULLW ? PER : PER - 1; }
  // LDS element offset of k-chunk `chunk` (8 elements) of tile row `row`
  static MSU_DEV int off(int row, int chunk) { return row * KB + ((chunk ^ ((row / RPL) % CH)) << 3); }
  // slot p = c * NTHR + tid is row p / CH, LDS chunk p % CH, which holds the global chunk that
  // off() puts there; rows past the tensor re-read its last row (their results are never stored)
  static MSU_DEV void stage(const bf16_t* __restrict__ src, int row0, int rows, int K, int k0, bf16_t* tile,
                            int tid) {
    const int wave = tid >> 6;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      if (c == PER - 1 && __builtin_amdgcn_readfirstlane(wave) >= FULLW) break;
      const int p = c * NTHR + tid;
      const int row = p / CH, g = (p % CH) ^ ((row / RPL) % CH);
      int r = row0 + row;
      if (r >= rows) r = rows - 1;
      glds16(src + (size_t)r * K + k0 + 8 * g, tile + (c * NTHR + wave * 64) * 8);
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
template <int NTHR>
struct KnTile {
  static constexpr int PER = BK * BN / 8 / NTHR;
  static MSU_DEV int off(int row, int col) { return row * BN + ((((col >> 3) ^ (4 * (row & 3)))) << 3) + (col & 7); }
  // 64 x 128 tile: 1024 16-B slots; columns past N re-read column n0
  static MSU_DEV void stage(const bf16_t* __restrict__ W, int n0, int N, int k0, bf16_t* tile, int tid) {
    const int wave = tid >> 6;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const int p = c * NTHR + tid;
      const int row = p >> 4, lc = (p & 15) ^ (4 * (row & 3));
      int n = n0 + 8 * lc;
      if (n >= N) n = n0;
      glds16(W + (size_t)(k0 + row) * N + n, tile + (c * NTHR + wave * 64) * 8);
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

// Persistent: a grid of at most one (WM = 4) or two (WM = 2) workgroups per CU walks the output
// tiles t = L, L + G, L + 2G, ... (L = the XCD-remapped block index, G = grid size) as ONE flat
// sequence of K steps, so the LDS ring never drains at a tile boundary: the first K steps of
// the next tile are staged while the last ones of the current tile are multiplied, and the
// epilogue's stores leave while those DMAs are in flight.  The stage-1..3 shapes have only
// 3-24 K steps per tile (K = 192..1536), so a per-tile prologue / epilogue was a large share of
// a non-persistent tile's time.  In one round of tiles an XCD takes a contiguous range of tile
// indices, i.e. the N tiles of a few M tiles: their A rows come from HBM once and from that
// XCD's L2 after.
// Tiles: (64 WM) x 128 outputs, WM x 2 waves of 64 x 64 (four 32 x 32 accumulators each).
//   WM = 2, NST = 2: 128 x 128, 64 KB ring, two workgroups per CU, vmcnt(0) before each step;
//   WM = 4, NST = 3: 256 x 128, 144 KB ring, one 8-wave workgroup per CU, two K steps in flight
//   across the raw barrier (counted vmcnt: the DMAs of the younger step and the epilogue stores
//   issued after the awaited step's DMA may stay outstanding).
// BNT: the tile's column width, 128 or 192 (waves 64 x 64 or 64 x 96: NI = 2 or 3 column
// accumulators).  192 makes the N = 384 / 768 / 1152 / 2304 shapes of Swin-T's stages 2-3 whole
// rounds of tiles on 256 CUs (N = 384 at M = 32768: 256 tiles of 256 x 192 instead of 384 of
// 256 x 128, i.e. 1.5 rounds); KN (input-gradient) form: 128 only.
// KB: K step (64).  A 32-deep step with a four-stage ring (three steps in flight in the same LDS)
// was 25-50 % slower on every stage 1-3 shape (r04u) and is gone.
// NST = 4 (A3W2): the 256 x 192 tile with the A operand two K steps ahead -- a ring of THREE A
// stages (32 KB each) beside TWO W stages (24 KB): 144 KB, where three whole stages (168 KB) do not
// fit.  A streams from HBM (or a sibling N tile's L2 lines), W is a small L2-resident weight: the
// operand with the long latency gets the deeper prefetch.  Per step s the waves issue W(s + 1), then
// A(s + 2); the wait for step s lets A(s + 1) (and a preceding epilogue's stores) stay in flight.
template <typename T, int EPI, int WM, int NST, bool WKN, int BNT, int KB>
__global__ void __launch_bounds__(128 * WM) gemm_nt_kernel(NtArgs a) {
  constexpr int NTHR = 128 * WM, BM = 64 * WM, NI = BNT / 64;
  constexpr bool A3 = NST == 4;
  static_assert(!WKN || (BNT == BN && KB == BK), "KN tiles are 128 wide, 64 deep");
  static_assert(!A3 || (!WKN && WM == 4 && BNT == 192), "A3W2: the 256 x 192 NT tile");
  typedef RowTile<BM, NTHR, KB> TA;
  typedef RowTile<BNT, NTHR, KB> TW;
  typedef KnTile<NTHR> TK;
  constexpr int KSL = KB / 16;  // 16-wide k slices per step
  constexpr int STG = (BM + BNT) * KB;  // elements per ring stage
  // per thread and step: DMA instructions (waves below DW0 issue D, the others D - 1), and
  // epilogue stores of a tile
  constexpr int D = TA::PER + (WKN ? TK::PER : TW::PER);
  static_assert(TA::FULLW * 64 == NTHR, "A rows: whole rounds");
  constexpr int DW0 = WKN ? 64 : TW::FULLW;
  constexpr int E = (EPI == EPI_GELU_DUAL ? 8 : 4) * NI;
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  static_assert(NST == 2 || ((A3 ? TA::PER + TW::PER : (NST - 2) * D) + E < 64), "vmcnt range");
  static_assert(!A3 || TW::FULLW * 64 == NTHR, "A3W2: every wave issues all its W DMA");
  constexpr int LDS_ELEMS = A3 ? 3 * BM * KB + 2 * BNT * KB : NST * STG;
  __shared__ __attribute__((aligned(16))) bf16_t lds[LDS_ELEMS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;  // this wave's 64 x 64 piece (tokens, columns)
  const int G = gridDim.x;
  const int L = xcd_remap(blockIdx.x, G);
  const int ntiles = a.tiles_m * a.tiles_n;
  const int nk = a.K / KB;  // K % 64 == 0 (nt_shape_ok)
  const int mine = L < ntiles ? (ntiles - 1 - L) / G + 1 : 0;
  const int nsteps = mine * nk;
  // NST = 2 walks tiles (tcur, then tnext): statically L, L + G, ..., or with the tile queue
  // claims of this XCD's counter -- the same tiles xcd_remap gives the XCD (first tile x0 +
  // local, then rounds of qx tiles G apart), in round order, so a row block of A still stays on
  // one XCD's L2.  The next tile is claimed by thread 0 at a tile's first K step (after its
  // barrier), published at the second (after that step's vmcnt(0)) through sq[ti & 1] and read
  // after its barrier -- before the last step issues the next tile's first DMA (nk >= 2: the
  // launch passes no queue for single-step tiles).
  int* const tq = NST == 2 ? a.tq : nullptr;
  const int xcd = blockIdx.x & 7;
  const int qx = (G >> 3) + (xcd < (G & 7) ? 1 : 0);
  const int x0 = L - (int)(blockIdx.x >> 3);
  __shared__ int sq[2];

  // K step kk of tile t: its A / W tiles -> LDS at dst
  auto issue_a_t = [&](int t, int kk, bf16_t* dst) __attribute__((always_inline)) {
    const int mt = t / a.tiles_n;
    if (a.A2 == nullptr) TA::stage(a.A, mt * BM, a.M, a.K, kk * KB, dst, tid);
    else if (kk * KB < a.K1) TA::stage(a.A, mt * BM, a.M, a.K1, kk * KB, dst, tid);  // K1 % 64 == 0
    else TA::stage(a.A2, mt * BM, a.M, a.K - a.K1, kk * KB - a.K1, dst, tid);
  };
  auto issue_w_t = [&](int t, int kk, bf16_t* dst) __attribute__((always_inline)) {
    const int mt = t / a.tiles_n, nt = t - mt * a.tiles_n;
    if constexpr (WKN) TK::stage(a.W, nt * BNT, a.N, kk * KB, dst, tid);
    else TW::stage(a.W, nt * BNT, a.N, a.K, kk * KB, dst, tid);
  };
  // K step s of this workgroup's static sequence
  auto issue_a = [&](int s, bf16_t* dst) __attribute__((always_inline)) {
    const int ti = s / nk;
    issue_a_t(L + ti * G, s - ti * nk, dst);
  };
  auto issue_w = [&](int s, bf16_t* dst) __attribute__((always_inline)) {
    const int ti = s / nk;
    issue_w_t(L + ti * G, s - ti * nk, dst);
  };
  // K step kk of tile t -> ring stage `st` (NST = 2 / 3: A and W in one stage)
  auto issue_tk = [&](int t, int kk, int st) __attribute__((always_inline)) {
    bf16_t* dst = lds + st * STG;
    issue_a_t(t, kk, dst);
    issue_w_t(t, kk, dst + BM * KB);
  };
  auto issue = [&](int s, int st) __attribute__((always_inline)) {
    const int ti = s / nk;
    issue_tk(L + ti * G, s - ti * nk, st);
  };
  bf16_t* const ldsW = lds + 3 * BM * KB;  // A3W2: the W stages after the three A stages

  f32x16 acc[NI][2];  // [column tile ni][token tile mi]: C^T, W rows on the accumulator rows
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0};

  if constexpr (A3) {
    // A(0), W(0), A(1): step 0 waits for W(0) with A(1) in flight
    if (nsteps > 0) {
      issue_a(0, lds);
      issue_w(0, ldsW);
    }
    if (nsteps > 1) issue_a(1, lds + BM * KB);
  } else {
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
      if (s < nsteps) issue(s, s);
  }
  int kk = 0, ti = 0;  // K step within the tile, tile ordinal (within this workgroup)
  int tcur = L, tnext = L + G;  // NST = 2: this tile, the next (tq: known from the tile's 2nd step)
  int nn = 0;                   // thread 0 (tq): the claim in flight
  int cst = 0;         // LDS stage of step s
  int epi_age = 99;    // steps since the last epilogue (its stores follow that step's DMA issue)
  bool a3_more_a = false;  // A3W2: this step also issued A(s + 2)
  bool epi_full = true;  // that epilogue issued all E stores of this wave (no ragged M / N edge)
  for (int s = 0; NST == 2 ? tcur < ntiles : s < nsteps; ++s) {
    // step s's DMA landed; younger DMAs (step s + 1) and epilogue stores issued after step s's
    // DMA may stay in flight (NST = 3, tiles of >= 3 K steps); else everything retires.
    // The counts must never exceed the ops really issued after step s's DMA: a wave whose last
    // epilogue sat on a ragged edge skipped some stores (all of them when its 64 columns lie
    // past N), so it does not count them -- counting them let that wave pass the barrier with
    // its share of step s's DMA still in flight, and the other waves read stale LDS (found as
    // run-to-run differences of the eager step with the side stream on, round 3)
    if constexpr (A3) {
      // W(s) landed (and A(s), issued a step earlier); A(s + 1), issued after W(s), and the
      // stores of an epilogue that followed them may stay in flight
      const bool younger = s + 1 < nsteps;
      const bool stores = epi_age == 0 && epi_full;
      if (younger && stores) wait_vmcnt<TA::PER + E>();
      else if (younger) wait_vmcnt<TA::PER>();
      else if (stores) wait_vmcnt<E>();
      else wait_vmcnt<0>();
    } else if constexpr (NST == 2) {
      wait_vmcnt<0>();
      if (tq != nullptr && kk == 1 && tid == 0) {
        sq[ti & 1] = nn;  // (nothing in flight here)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // landed before the raw barrier
      }
    } else if constexpr (NST == 3) {
      const bool younger = s + 1 < nsteps;
      const bool stores = epi_age <= 1 && nk >= 3 && epi_full;
      if (nk < 3) wait_vmcnt<0>();
      else if (younger && stores) wait_vmcnt<D + E>();
      else if (younger) wait_vmcnt<D>();
      else if (stores) wait_vmcnt<E>();
      else wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();   // every wave's DMA of step s has landed, and every wave is
    asm volatile("" ::: "memory");  // done reading step s-1's stage (refilled below)
    ++epi_age;
    const bool last = kk + 1 == nk;
    if (NST == 2 && tq != nullptr) {
      if (kk == 0) {
        if (tid == 0) nn = tq_claim(tq, xcd);
      } else if (kk == 1) {
        // read before this step's DMA issue: no LDS-DMA in flight
        const int c = __builtin_amdgcn_readfirstlane(sq[ti & 1]);
        tnext = x0 + G * (1 + c / qx) + c % qx;
      }
    }
    const int t = NST == 2 ? tcur : L + ti * G;
    const int mt = t / a.tiles_n, nt = t - mt * a.tiles_n;
    const int m0 = mt * BM, n0 = nt * BNT;
    const int hh = lane >> 5;
    constexpr int WNC = BNT / 2;  // columns per wave
    // the epilogue's operands (bias columns, GELU' pre-activations), loaded before the tile's
    // last MFMAs and before the next stage's DMA: one counted wait in the epilogue
    float4 eb[NI][2][2];
    u32x4 eh[2][NI][2];
    if (last) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          const int n = min(n0 + WNC * wn + 32 * ni + 16 * g + 8 * hh, a.N - 8);
          if constexpr (EPI == EPI_GELU_GRAD) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
              const int m = min(m0 + 64 * wm + 32 * mi + (lane & 31), a.M - 1);
              eh[mi][ni][g] = *reinterpret_cast<const u32x4*>(a.H + (size_t)m * a.N + n);
            }
          } else if (a.bias) {
            eb[ni][g][0] = *reinterpret_cast<const float4*>(a.bias + n);
            eb[ni][g][1] = *reinterpret_cast<const float4*>(a.bias + n + 4);
          }
        }
    }
    const bf16_t* ta;
    const bf16_t* tw;
    bool more;  // DMA issued in this step (the epilogue's wait lets it stay in flight)
    if constexpr (A3) {
      // W(s + 1) into the W stage step s - 1 used, A(s + 2) into the A stage of step s - 1
      const int wst = s & 1, ast = cst;  // cst: A stage of step s (s % 3)
      const bool mw = s + 1 < nsteps, ma = s + 2 < nsteps;
      if (mw) issue_w(s + 1, ldsW + (wst ^ 1) * BNT * KB);
      if (ma) issue_a(s + 2, lds + (ast == 0 ? 2 : ast - 1) * BM * KB);
      more = mw;
      a3_more_a = ma;
      ta = lds + ast * BM * KB;
      tw = ldsW + wst * BNT * KB;
      cst = cst + 1 == 3 ? 0 : cst + 1;
    } else if constexpr (NST == 2) {
      more = !last || tnext < ntiles;
      if (more) issue_tk(last ? tnext : tcur, last ? 0 : kk + 1, cst ^ 1);
      ta = lds + cst * STG;
      tw = ta + BM * KB;
      cst ^= 1;
    } else {
      more = s + NST - 1 < nsteps;
      if (more) issue(s + NST - 1, cst == 0 ? NST - 1 : cst - 1);
      ta = lds + cst * STG;
      tw = ta + BM * KB;
      cst = cst + 1 == NST ? 0 : cst + 1;
    }
    bf16x8 fw[2][NI], fx[2][2];
    auto rd = [&](int ks, int set) {
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        if constexpr (WKN) fw[set][ni] = TK::frag(tw, WNC * wn + 32 * ni, ks, lane);
        else fw[set][ni] = TW::frag(tw, WNC * wn + 32 * ni, ks, lane);
      }
      fx[set][0] = TA::frag(ta, 64 * wm, ks, lane);
      fx[set][1] = TA::frag(ta, 64 * wm + 32, ks, lane);
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < KSL; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < KSL) rd(ks + 1, cur ^ 1);
      // all of slice ks + 1's fragment reads go out before slice ks's MFMAs (the wait before
      // those is then lgkmcnt(reads of ks + 1)); left alone, the scheduler sank some reads
      // between the MFMAs into registers freed by them and waited lgkmcnt(0) two MFMAs later
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        acc[ni][0] = Fmt16<T>::mma32(fw[cur][ni], fx[cur][0], acc[ni][0]);
        acc[ni][1] = Fmt16<T>::mma32(fw[cur][ni], fx[cur][1], acc[ni][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (!last) {
      ++kk;
      continue;
    }
    kk = 0;
    ++ti;
    if constexpr (NST == 2) {
      tcur = tnext;
      tnext = tcur + G;  // (static; tq: replaced at the next tile's first step)
    }
    epi_age = 0;
    epi_full = m0 + 64 * wm + 64 <= a.M && n0 + WNC * wn + WNC <= a.N;
    // the epilogue operands (and every older DMA) have landed; the DMA just issued may stay
    // in flight (NST = 3).  One wait, not one per exec-masked store branch.
    if constexpr (A3) {
      // the epilogue operands were loaded before this step's W(s + 1) / A(s + 2) DMAs
      if (more && a3_more_a) wait_vmcnt<TW::PER + TA::PER>();
      else if (more) wait_vmcnt<TW::PER>();
      else wait_vmcnt<0>();
    } else if (NST >= 3 && more) {
      if (wave < DW0) wait_vmcnt<D>();
      else wait_vmcnt<D - 1>();
    } else {
      wait_vmcnt<0>();
    }
    // ---- epilogue of tile t: lane (l & 31) is token m; after the swap, 8 consecutive columns
    // per store
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int m = m0 + 64 * wm + 32 * mi + (lane & 31);
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
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
          const int n = n0 + WNC * wn + 32 * ni + 8 * g0 + 8 * hh;
          if (m >= a.M || n >= a.N) continue;
          if (EPI != EPI_GELU_GRAD && a.bias) {
            const float4 b0 = eb[ni][g0 >> 1][0], b1 = eb[ni][g0 >> 1][1];
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
          }
          const size_t off = (size_t)m * a.N + n;
          if constexpr (EPI == EPI_GELU_GRAD) {
            const u32x4 hv = eh[mi][ni][g0 >> 1];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              v[2 * i] *= gelu_grad_fast(Fmt16<T>::lo(hv[i]));
              v[2 * i + 1] *= gelu_grad_fast(Fmt16<T>::hi(hv[i]));
            }
          }
          const u32x4 pk = {pack2<T>(v[0], v[1]), pack2<T>(v[2], v[3]), pack2<T>(v[4], v[5]), pack2<T>(v[6], v[7])};
          // ablation 16: no output stores (results wrong; the never-true test keeps the MFMAs).
          // These 16-B stores cover 32 tokens x 32 B per instruction; an epilogue staged through
          // the consumed ring stage and stored as 192-B row pieces was neutral (r05z).
          if constexpr ((MSU_EXP & 16) != 0) if (v[0] != 1.2345e-30f) continue;
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
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0};
  }
  tq_finish(tq);
}

}  // namespace

#include "gemm_pp.h"

namespace {

// msu_nt_gemm_mode(1): the ping-pong kernel (gemm_pp.h) where the shape tiles exactly; 0 (the
// default): the persistent 2-barrier kernel everywhere.  A/B switch MSU_NT_PP, set by the Python
// side at import: the ping-pong kernel measured 0.72-0.98x of the persistent one (r05g)
int g_nt_pp = 0;
// tile-form override for kernel-timing tools (msu_nt_gemm_mode bits 1-2): 0 = the cost model,
// 1 = 128 x 192 (two workgroups per CU), 2 = 256 x 128 (three-stage ring), 3 = 128 x 128
int g_nt_force = 0;
// msu_nt_gemm_mode bit 3: the 256 x 192 tile on the A3W2 ring (gemm_nt_kernel NST = 4)
int g_nt_a3 = 0;
// msu_nt_gemm_mode bit 4: the two-stage kernel's tile queue (opt-in MSU_NT_DYN=1: the claim's
// round trip costs 2-3 us on the short stage-2/3 launches and the step did not gain, r06q/r06r)
int g_nt_dyn = 0;

int num_cus_nt();

// BN of the ping-pong kernel for this shape, or 0 (gemm_nt_kernel takes it): exact tiling, and
// rounds of tiles at least 3/4 full (the stage-3 shapes, 96-288 tiles of 256 rows on 256 CUs,
// keep the persistent kernel's 128-row tiles)
int pp_bn(long M, int N, int K, int epi, bool wkn) {
  // (the GELU' epilogue's operands, 16-bit pre-activations of the whole tile, would be global
  // loads the compiler drains the DMA ring for: that form stays on gemm_nt_kernel)
  // (K >= 192: a tile's output stores are spread over the next tile's first four load slots)
  if (!g_nt_pp || wkn || epi == EPI_GELU_GRAD || M % pp::BM != 0 || K % 64 != 0 || K < 192) return 0;
  int bn = 0;
  if (N % 192 == 0) bn = 192;
  if (!bn) return 0;
  const long tiles = (M / pp::BM) * (N / bn), cus = num_cus_nt();
  const long rounds = (tiles + cus - 1) / cus;
  return 4 * tiles >= 3 * rounds * cus ? bn : 0;
}

bool nt_shape_ok(long M, int N, int K) {
  return M > 0 && M < (1L << 31) && N > 0 && N % 32 == 0 && K > 0 && K % 64 == 0 && (long)M * N < (1L << 40);
}

int num_cus_nt() {
  static const int cus = [] {
    int n = 0, dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
  }();
  return cus;
}

// Tile configuration of a shape, by a rounds-of-tiles cost model: the output is covered in
// rounds of (CUs x workgroups per CU) tiles, each round costing a workgroup's tile area times the
// workgroups sharing a CU, times the measured cost per output of the tile form (x 0.78 for the
// 192-wide tiles: 64 x 96 wave tiles read 5 fragments per 6 MFMAs instead of 4 per 4; r04b
// same-box kbench at whole-round shapes: 32768 x 384 x 1152 39-42 vs 57-58 us, 131072 x 192 x 768
// 59-61 vs 84-88 us):
//   wm 4, bn 128: 256 x 128, three-stage ring, one workgroup per CU;
//   wm 2, bn 128: 128 x 128, two-stage ring, two workgroups per CU;
//   wm 4, bn 192: 256 x 192, two-stage ring (3 x 56 KB does not fit), one workgroup per CU;
//   wm 2, bn 192: 128 x 192, two-stage ring, two workgroups per CU (2 x 80 KB of LDS).
// KN (input-gradient with the forward weight in place) keeps bn 128.  (A 192 x 192 tile with a
// three-stage ring, 6 waves, was slower on every shape, r04j: gone.)
struct NtCfg {
  int wm, bn;
};

NtCfg nt_cfg(long M, int N, bool wkn) {
  if (g_nt_force == 1 && !wkn && N % 192 == 0) return NtCfg{2, 192};
  if (g_nt_force == 2) return NtCfg{4, 128};
  if (g_nt_force == 3) return NtCfg{2, 128};
  const long cus = num_cus_nt();
  const NtCfg cands[4] = {{4, 128}, {2, 128}, {4, 192}, {2, 192}};
  NtCfg best = cands[0];
  double best_cost = -1.0;
  for (const NtCfg& c : cands) {
    if (c.bn == 192 && (wkn || N % 192 != 0)) continue;
    // rounds of resident tiles x the output area a CU computes per round (x 0.78 for the
    // 192-wide form).  A 128-row (two-per-CU) form with no more tiles than CUs has ONE tile per
    // CU, at a per-area cost of 1.57 (it shares the CU with nobody): r04h sweep, 8192 x 768 x
    // 3072: 128 x 192 on all 256 CUs 59 us vs 256 x 128 (the previous pick) 65 us and 256 x 192
    // on 128 CUs 75 us
    const long bm = 64L * c.wm, slots = c.wm == 2 ? 2 : 1;
    const long tiles = ((M + bm - 1) / bm) * ((N + c.bn - 1) / c.bn);
    const long rounds = (tiles + cus * slots - 1) / (cus * slots);
    const long occ = c.wm == 2 ? std::min(2L, (tiles + cus - 1) / cus) : 1;
    const double cost = (double)rounds * bm * c.bn * occ * (c.bn == 192 ? 0.78 : 1.0) * (c.wm == 2 && occ == 1 ? 1.57 : 1.0);
    if (best_cost < 0 || cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

template <typename T, int WM, int NST, bool WKN, int BNT, int KB = 64>
void launch_nt(int epi, const NtArgs& a, hipStream_t st) {
  const long tiles = (long)a.tiles_m * a.tiles_n;
  const long cap = (long)num_cus_nt() * (WM == 2 ? 2 : 1);
  const unsigned grid = (unsigned)(tiles < cap ? tiles : cap);
  const dim3 blk(128 * WM);
  NtArgs q = a;
  q.tq = NST == 2 && g_nt_dyn && a.K >= 2 * KB ? tile_queue(st) : nullptr;
  switch (epi) {
    case EPI_PLAIN: hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_PLAIN, WM, NST, WKN, BNT, KB>), dim3(grid), blk, 0, st, q); break;
    case EPI_GELU_DUAL: hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_GELU_DUAL, WM, NST, WKN, BNT, KB>), dim3(grid), blk, 0, st, q); break;
    default: hipLaunchKernelGGL((gemm_nt_kernel<T, EPI_GELU_GRAD, WM, NST, WKN, BNT, KB>), dim3(grid), blk, 0, st, q); break;
  }
}

int nt_launch(int dtype, const void* A, const void* W, const float* bias, void* Y, void* Y2, const void* H, long M,
              int N, int K, int epi, void* stream, bool wkn, const void* A2 = nullptr, int K1 = 0) {
  if (!msu_is16(dtype)) return -3;
  if (!nt_shape_ok(M, N, K)) return -2;
  if (epi == EPI_GELU_DUAL && (Y2 == nullptr || bias == nullptr)) return -3;
  if (epi == EPI_GELU_GRAD && (H == nullptr || bias != nullptr)) return -3;
  if (epi < 0 || epi > 2) return -3;
  NtArgs a;
  a.tq = nullptr;
  if (A2 != nullptr && (wkn || epi != EPI_PLAIN || K1 <= 0 || K1 >= K || K1 % 64)) return -3;
  a.A = (const bf16_t*)A;
  a.A2 = (const bf16_t*)A2;
  a.K1 = A2 != nullptr ? K1 : K;
  a.W = (const bf16_t*)W;
  a.bias = bias;
  a.Y = (bf16_t*)Y;
  a.Y2 = (bf16_t*)Y2;
  a.H = (const bf16_t*)H;
  a.M = (int)M;
  a.N = N;
  a.K = K;
  const NtCfg cfg = nt_cfg(M, N, wkn);
  a.tiles_n = (N + cfg.bn - 1) / cfg.bn;
  a.tiles_m = (int)((M + 64 * cfg.wm - 1) / (64 * cfg.wm));
  if ((long)a.tiles_m * a.tiles_n >= (1L << 31)) return -2;
  hipStream_t st = (hipStream_t)stream;
  const int pbn = pp_bn(M, N, K, epi, wkn);
  if (pbn) {
    a.tiles_n = N / pbn;
    a.tiles_m = (int)(M / pp::BM);
    const long tiles = (long)a.tiles_m * a.tiles_n;
    const unsigned grid = (unsigned)(tiles < num_cus_nt() ? tiles : num_cus_nt());
    MSU_DISPATCH16(dtype, T,
      if (epi == EPI_PLAIN) hipLaunchKernelGGL((pp::gemm_pp_kernel<T, EPI_PLAIN, 192>), dim3(grid), dim3(512), 0, st, a);
      else hipLaunchKernelGGL((pp::gemm_pp_kernel<T, EPI_GELU_DUAL, 192>), dim3(grid), dim3(512), 0, st, a));
    return MSU_CHECK_LAUNCH();
  }
  MSU_DISPATCH16(dtype, T,
    if (cfg.bn == 192) {
      if (cfg.wm == 4 && g_nt_a3) launch_nt<T, 4, 4, false, 192>(epi, a, st);
      else if (cfg.wm == 4) launch_nt<T, 4, 2, false, 192>(epi, a, st);
      else launch_nt<T, 2, 2, false, 192>(epi, a, st);
    } else if (cfg.wm == 4) {
      if (wkn) launch_nt<T, 4, 3, true, 128>(epi, a, st);
      else launch_nt<T, 4, 3, false, 128>(epi, a, st);
    } else {
      if (wkn) launch_nt<T, 2, 2, true, 128>(epi, a, st);
      else launch_nt<T, 2, 2, false, 128>(epi, a, st);
    });
  return MSU_CHECK_LAUNCH();
}

}  // namespace

extern "C" {

// Whether msu_nt_gemm covers this shape (K % 64, N % 32).
int msu_nt_gemm_supported(long M, int N, int K) { return nt_shape_ok(M, N, K) ? 1 : 0; }

// The tile msu_nt_gemm picks for M x N (the [N, K] weight form, plain epilogue, K = 384):
// rows * 1000 + columns, + 1000000 for the ping-pong kernel.
int msu_nt_gemm_plan(long M, int N) {
  const int pbn = pp_bn(M, N, 384, EPI_PLAIN, false);
  if (pbn) return 1000000 + pp::BM * 1000 + pbn;
  const NtCfg c = nt_cfg(M, N, false);
  return 64 * c.wm * 1000 + c.bn;
}

// bit 0 -- 1: the ping-pong kernel where the shape tiles exactly, 0 (the default, MSU_NT_PP=0): the
// persistent 2-barrier kernel everywhere; bits 1-2: a forced tile form for kernel-timing tools
// (0: the cost model; 1: 128 x 192, 2: 256 x 128, 3: 128 x 128); bit 3: the 256 x 192 tile on the
// A3W2 ring (A two K steps ahead).  Returns the previous mode.
int msu_nt_gemm_mode(int mode) {
  const int prev = g_nt_pp | (g_nt_force << 1) | (g_nt_a3 << 3) | (g_nt_dyn << 4);
  g_nt_pp = mode & 1;
  g_nt_force = (mode >> 1) & 3;
  g_nt_a3 = (mode >> 3) & 1;
  g_nt_dyn = (mode >> 4) & 1;
  return prev;
}

// Y[M][N] = epi(A . W^T + bias), 16-bit in / out (dtype 1 bf16, 2 f16), f32 accumulation.
// epi 0: plain (+ bias when given); 1: Y = H and Y2 = GELU(H) (needs bias); 2: Y = (A . W^T) *
// GELU'(H) (no bias).  Same semantics as msu_tok_gemm without the split-A input.
int msu_nt_gemm(int dtype, const void* A, const void* W, const float* bias, void* Y, void* Y2, const void* H,
                long M, int N, int K, int epi, void* stream) {
  return nt_launch(dtype, A, W, bias, Y, Y2, H, M, N, K, epi, stream, false);
}

// Y[M][N] = [A | A2] . W^T + bias (plain epilogue): A [M][K1], A2 [M][K - K1], K1 % 64 == 0 -- the
// skip fusion torch.cat([x, skip], -1) -> concat_back_dim Linear without the concatenated copy.
int msu_nt_gemm_cat(int dtype, const void* A, const void* A2, int K1, const void* W, const float* bias, void* Y,
                    long M, int N, int K, void* stream) {
  if (A2 == nullptr) return -3;
  return nt_launch(dtype, A, W, bias, Y, nullptr, nullptr, M, N, K, EPI_PLAIN, stream, false, A2, K1);
}

// Same with the weight given as Wk[K][N] (Y = epi(A . Wk + bias)): the input gradient of a Linear,
// dX[M][K_fwd] = dY[M][N_fwd] . W[N_fwd][K_fwd], straight from the forward weight (no W^T copy).
int msu_nt_gemm_kn(int dtype, const void* A, const void* Wk, const float* bias, void* Y, void* Y2, const void* H,
                   long M, int N, int K, int epi, void* stream) {
  return nt_launch(dtype, A, Wk, bias, Y, Y2, H, M, N, K, epi, stream, true);
}

}  // extern "C"
