// MFMA 16x16 operand fragments read from natural [k rows][n cols] LDS images.
//
// For a product that sums over the ROW index of a row-major LDS image (weight gradients:
// sum over pixels / tokens), each lane needs 8 (bf16) k-consecutive elements of one column:
// ds_read_b64_tr_b16 delivers a 4-row x 16-col block column-major to 16 lanes, so two of
// them form one v_mfma_f32_16x16x32_bf16 operand (lane l: k = 8(l>>4) + j, column l&15).
// Every lane supplies its own row address, so row maps may be arbitrary (tap shifts,
// gathered rows); addresses must be 8-byte aligned and EXEC all ones.
#pragma once
#include "common.h"

namespace {

typedef short msu_v4s __attribute__((ext_vector_type(4)));

template <typename T> struct TR;
template <> struct TR<bf16_t> {
  template <typename RowFn>
  static MSU_DEV bf16x8 frag(RowFn row_ptr, int kbase, int col0, int lane) {
    const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const bf16_t* a0 = row_ptr(kbase + 8 * gq + q) + col0 + 4 * p;
    const bf16_t* a1 = row_ptr(kbase + 8 * gq + 4 + q) + col0 + 4 * p;
    typedef __attribute__((address_space(3))) msu_v4s lds_v4s;
    const msu_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
    const msu_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a1));
    msu_v4s both[2] = {lo, hi};
    return *reinterpret_cast<bf16x8*>(both);
  }
  // acc(16x16) += A(16 x 32) B(32 x 16): A(m,k) = ra(k)[colA + m], B(k,n) = rb(k)[colB + n]
  template <typename RA, typename RB>
  static MSU_DEV void mma(f32x4& acc, RA ra, int colA, RB rb, int colB, int kbase, int lane) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag(ra, kbase, colA, lane), frag(rb, kbase, colB, lane),
                                                  acc, 0, 0, 0);
  }
};
template <> struct TR<float> {
  template <typename RA, typename RB>
  static MSU_DEV void mma(f32x4& acc, RA ra, int colA, RB rb, int colB, int kbase, int lane) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int k = kbase + 4 * s + (lane >> 4);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra(k)[colA + (lane & 15)], rb(k)[colB + (lane & 15)], acc, 0, 0, 0);
    }
  }
};

}  // namespace
