// Linear-layer weight (and bias) gradient: dW[N][K] = sum_m dY[m][n] X[m][k], db[n] = sum_m dY[m][n].
//
// Every nn.Linear on the MS-UNet path (torchvision block qkv / proj / mlp.0 / mlp.3,
// PatchMerging.reduction, PatchExpand.expand, concat_back_dim, FinalPatchExpand_X4_V2.expand,
// PatchEmbed.proj as im2col GEMM) has M = tokens (up to 8 x 65536 at 1024^2) and N, K <= a
// few thousand: a tall-skinny "TN" product whose reduction runs over M.  Library kernels
// tile it with far too few workgroups (hipBLASLt picked MT64x64x256 at ~0.76 ms/call).
// Here the M range is split across S workgroups per 64x64 output tile (S chosen to fill
// the 256 CUs), operands are staged row-major in LDS and read k-strided with
// ds_read_b64_tr_b16 into v_mfma_f32_16x16x32_bf16, and the S partial tiles are reduced
// deterministically (colsum).  The bias gradient rides along on the k-tile-0 workgroups.
#include "common.h"
#include "mfma_frag.h"
#include "reduce.h"

namespace {

constexpr int BM = 32;       // rows of M per step (one MFMA K)
constexpr int BT = 64;       // output tile: 64 (n) x 64 (k)
constexpr int LDT = BT + 8;  // LDS row stride (elements), 16-B aligned rows

template <typename T>
__global__ void __launch_bounds__(256) wgrad_kernel(const T* __restrict__ dY, const T* __restrict__ X,
                                                    float* __restrict__ part, float* __restrict__ dbpart,
                                                    long M, int N, int K, int S, long mchunk) {
  __shared__ __attribute__((aligned(16))) T sA[2][BM * LDT];  // dY rows  [m][n]
  __shared__ __attribute__((aligned(16))) T sB[2][BM * LDT];  // X rows   [m][k]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntk = (K + BT - 1) / BT;
  const int tile = blockIdx.x, split = blockIdx.y;
  const int tn = tile / ntk, tk = tile - (tile / ntk) * ntk;
  const int n0 = tn * BT, k0 = tk * BT;
  const long m_begin = (long)split * mchunk;
  long m_end = m_begin + mchunk;
  if (m_end > M) m_end = M;
  const int wn = (wave >> 1) * 32, wk = (wave & 1) * 32;  // wave sub-tile 32 x 32

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  const bool do_bias = dbpart != nullptr && tk == 0;

  // staging: 32 rows x 64 cols = 512 4-element chunks per operand, 2 per thread
  auto stage = [&](int buf, long m0) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int idx = tid + c * 256;
      const int r = idx >> 4, col = (idx & 15) * 4;
      const long m = m0 + r;
      float va[4] = {0.f, 0.f, 0.f, 0.f}, vb[4] = {0.f, 0.f, 0.f, 0.f};
      if (m < m_end) {
        if (n0 + col < N) Vec4<T>::load(dY + m * (long)N + n0 + col, va);
        if (k0 + col < K) Vec4<T>::load(X + m * (long)K + k0 + col, vb);
      }
      Vec4<T>::store(&sA[buf][r * LDT + col], va);
      Vec4<T>::store(&sB[buf][r * LDT + col], vb);
    }
  };

  int buf = 0;
  if (m_begin < m_end) stage(0, m_begin);
  __syncthreads();
  for (long m0 = m_begin; m0 < m_end; m0 += BM) {
    if (m0 + BM < m_end) stage(buf ^ 1, m0 + BM);
    const T* A = sA[buf];
    const T* B = sB[buf];
    auto ra = [&](int k) { return A + k * LDT; };
    auto rb = [&](int k) { return B + k * LDT; };
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) TR<T>::mma(acc[i][j], ra, wn + 16 * i, rb, wk + 16 * j, 0, lane);
    if (do_bias && tid < BT) {
#pragma unroll 8
      for (int r = 0; r < BM; ++r) dbacc += to_f32(A[r * LDT + tid]);
    }
    __syncthreads();
    buf ^= 1;
  }
  // partial tile -> part[split][n][k]
  float* out = part + (long)split * N * K;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn + 16 * i + (lane >> 4) * 4 + r;
        const int k = k0 + wk + 16 * j + (lane & 15);
        if (n < N && k < K) out[(long)n * K + k] = acc[i][j][r];
      }
  if (do_bias && tid < BT && n0 + tid < N) dbpart[(long)split * N + n0 + tid] = dbacc;
}

inline int pick_splits(long M, int N, int K) {
  const long tiles = (long)((N + BT - 1) / BT) * ((K + BT - 1) / BT);
  long s = (2048 + tiles - 1) / tiles;
  const long max_s = (M + 255) / 256;  // keep >= 256 rows per split
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
  if (N % 4 || K % 4 || M < 0) return -2;
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
  const dim3 grid((unsigned)(((N + BT - 1) / BT) * ((K + BT - 1) / BT)), (unsigned)S);
  if (dtype == MSU_BF16)
    hipLaunchKernelGGL(wgrad_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)dY, (const bf16_t*)X,
                       part, dbpart, M, N, K, S, mchunk);
  else
    hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, st, (const float*)dY, (const float*)X,
                       part, dbpart, M, N, K, S, mchunk);
  colsum(part, S, (long)N * K, (long)N * K, dW, accumulate, st);
  if (db) colsum(dbpart, S, N, N, db, accumulate, st);
  return MSU_CHECK_LAUNCH();
}

}  // extern "C"
