// MFMA 16x16 operand fragments read from natural [k rows][n cols] LDS images.
//
// For a product that sums over the ROW index of a row-major LDS image (weight gradients:
// sum over pixels / tokens), each lane needs 8 (bf16) k-consecutive elements of one column:
// ds_read_b64_tr_b16 delivers a 4-row x 16-col block column-major to 16 lanes, so two of
// them form one v_mfma_f32_16x16x32_{bf16,f16} operand (lane l: k = 8(l>>4) + j, column l&15).
// Every lane supplies its own row address, so row maps may be arbitrary (tap shifts,
// gathered rows); addresses must be 8-byte aligned and EXEC all ones.
#pragma once
#include <utility>

#include "common.h"

namespace {

typedef short msu_v4s __attribute__((ext_vector_type(4)));

template <typename T> struct TR;
template <typename T> struct TR16 {
  template <typename RowFn>
  static MSU_DEV bf16x8 frag(RowFn row_ptr, int kbase, int col0, int lane) {
    const int gq = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const auto* a0 = row_ptr(kbase + 8 * gq + q) + col0 + 4 * p;
    const auto* a1 = row_ptr(kbase + 8 * gq + 4 + q) + col0 + 4 * p;
    typedef __attribute__((address_space(3))) msu_v4s lds_v4s;
    const msu_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
    const msu_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a1));
    msu_v4s both[2] = {lo, hi};
    return *reinterpret_cast<bf16x8*>(both);
  }
  // acc(16x16) += A(16 x 32) B(32 x 16): A(m,k) = ra(k)[colA + m], B(k,n) = rb(k)[colB + n]
  template <typename RA, typename RB>
  static MSU_DEV void mma(f32x4& acc, RA ra, int colA, RB rb, int colB, int kbase, int lane) {
    acc = Fmt16<T>::mma16(frag(ra, kbase, colA, lane), frag(rb, kbase, colB, lane), acc);
  }
};
template <> struct TR<bf16_t> : TR16<bf16_t> {};
template <> struct TR<f16_t> : TR16<f16_t> {};
// Untracked fragment reads for LDS images filled by LDS-DMA (global_load_lds): the compiler
// treats every pending LDS-DMA as a possible alias of a visible ds_read and puts an
// s_waitcnt vmcnt(0) in front of it, draining the whole prefetch ring every stage.  These
// reads are inline asm (byte offsets folded into the instruction); the caller makes the
// data visible with lds_wait_tie() before the MFMAs that consume it.
template <int OFF>
MSU_DEV msu_v4s ds_tr_b64_untracked(uint32_t addr) {
  msu_v4s v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF>
MSU_DEV uint32_t ds_b32_untracked(uint32_t addr) {
  uint32_t v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int OFF0, int OFF1>
MSU_DEV bf16x8 tr8_untracked(uint32_t addr) {
  const msu_v4s lo = ds_tr_b64_untracked<OFF0>(addr);
  const msu_v4s hi = ds_tr_b64_untracked<OFF1>(addr);
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
// s_waitcnt lgkmcnt(N), then pin the fragments after it (an empty asm rewriting each one, so
// no consumer can be scheduled above the wait)
template <typename T>
MSU_DEV void vreg_pin(T& v) {
  asm volatile("" : "+v"(v));
}
template <int N, typename... Fr>
MSU_DEV void lds_wait_tie(Fr&... fr) {
  static_assert(N >= 0 && N < 16, "lgkmcnt range");
  asm volatile("s_waitcnt lgkmcnt(%0)" : : "i"(N) : "memory");
  (vreg_pin(fr), ...);
}
template <typename F, int... Is>
MSU_DEV void unroll_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(std::integral_constant<int, Is>{}), ...);
}
// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): indices usable as template
// arguments (instruction offsets) and as constant register-array indices
template <int N, typename F>
MSU_DEV void unroll_for(F&& f) {
  unroll_for_impl(f, std::make_integer_sequence<int, N>{});
}
MSU_DEV uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)(p);
}

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
