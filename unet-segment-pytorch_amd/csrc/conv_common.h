// conv_common.h — MFMA operand traits shared by the conv / wgrad kernels (gfx950).
#pragma once
#include "src_gather.h"

namespace unet {

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KC = 32;     // channels per staged chunk (64 bytes)
  static constexpr int KSTEP = 32;  // K of one MFMA
  static constexpr int E = 8;       // operand elements per lane
  typedef bf16x8 frag;
  __device__ static __forceinline__ frag load(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
  __device__ static __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KC = 16;
  static constexpr int KSTEP = 4;
  static constexpr int E = 1;
  typedef float frag;
  __device__ static __forceinline__ frag load(const float* p) { return *p; }
  __device__ static __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

template <typename T> __host__ __device__ constexpr int kc_of() { return sizeof(T) == 2 ? 32 : 16; }
static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }
__device__ __forceinline__ int round_up_d(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace unet
