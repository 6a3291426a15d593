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
#include "common.h"
#include "mfma_frag.h"
#include "reduce.h"

namespace {

constexpr int BM = 64;  // rows of M per LDS stage (two MFMA k-steps)

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
  return (long)S * N * K + (long)S * N;
}

// dW [N][K] f32 (overwritten, or accumulated when accumulate != 0), db [N] f32 (may be null).
int msu_linear_wgrad(int dtype, const void* dY, const void* X, float* dW, float* db, float* workspace,
                     long M, int N, int K, int accumulate, void* stream) {
  if (N % 8 || K % 8 || M < 0) return -2;  // 16-B staging chunks
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {
    if (!accumulate) hipMemsetAsync(dW, 0, sizeof(float) * (long)N * K, st);
    if (db && !accumulate) hipMemsetAsync(db, 0, sizeof(float) * N, st);
    return MSU_CHECK_LAUNCH();
  }
  const int S = pick_splits(M, N, K);
  long mchunk = (M + S - 1) / S;
  mchunk = (mchunk + BM - 1) / BM * BM;
  float* part = workspace;
  float* dbpart = db ? workspace + (long)S * N * K : nullptr;
  const int bt = tile_of(N, K);
  const dim3 grid((unsigned)(((N + bt - 1) / bt) * ((K + bt - 1) / bt)), (unsigned)S);
  if (dtype == MSU_BF16) {
    if (bt == 96)
      hipLaunchKernelGGL((wgrad_kernel<bf16_t, 3>), grid, dim3(256), 0, st, (const bf16_t*)dY,
                         (const bf16_t*)X, part, dbpart, M, N, K, mchunk);
    else
      hipLaunchKernelGGL((wgrad_kernel<bf16_t, 4>), grid, dim3(256), 0, st, (const bf16_t*)dY,
                         (const bf16_t*)X, part, dbpart, M, N, K, mchunk);
  } else {
    if (bt == 96)
      hipLaunchKernelGGL((wgrad_kernel<float, 3>), grid, dim3(256), 0, st, (const float*)dY,
                         (const float*)X, part, dbpart, M, N, K, mchunk);
    else
      hipLaunchKernelGGL((wgrad_kernel<float, 4>), grid, dim3(256), 0, st, (const float*)dY,
                         (const float*)X, part, dbpart, M, N, K, mchunk);
  }
  colsum(part, S, (long)N * K, (long)N * K, dW, accumulate, st);
  if (db) colsum(dbpart, S, N, N, db, accumulate, st);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
