// conv_mfma32.h — the 32x32x16 MFMA operand traits and half-wave reductions used by conv5.hip.
#pragma once
#include "conv_src16.h"

namespace unet {

typedef __attribute__((ext_vector_type(16))) float f32x16;

template <typename T> struct Mma32;
template <> struct Mma32<bf16> {
  typedef bf16x8 frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mma32<f16> {
  typedef f16x8 frag;
  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

// sum over the 32 lanes l with equal l >> 5 (one pixel row of the 32x32 accumulator): DPP row sums, then the
// partner row through v_permlane16_swap; every lane receives its half's total
__device__ __forceinline__ float half32_sum(float v) {
  v = row16_sum(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

}  // namespace unet
