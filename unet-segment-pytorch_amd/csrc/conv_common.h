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
template <> struct Mma<f16> {
  static constexpr int KC = 32;
  static constexpr int KSTEP = 32;
  static constexpr int E = 8;
  typedef f16x8 frag;
  __device__ static __forceinline__ frag load(const f16* p) { return *reinterpret_cast<const f16x8*>(p); }
  __device__ static __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
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

// UNET_OUT_SHUFFLE2 epilogue store: the 1x1 conv's channel co = (2a+b)*Ct + c at input pixel (oh, ow)
// is the ConvTranspose2d(k=2, s=2) output at (2*oh + a, 2*ow + b), channel c (+ bias)
template <typename T>
__device__ __forceinline__ void store_shuffle2(const unet_conv_desc& d, long long n, int oh, int ow, int co, float v) {
  const int ct = d.Cout >> 2;
  const int q = co / ct, c = co - q * ct;
  const long long o = ((n * (2 * d.H) + 2 * oh + (q >> 1)) * (long long)(2 * d.W) + 2 * ow + (q & 1)) * ct + c;
  reinterpret_cast<T*>(d.out)[o] = from_f<T>(v + (d.bias ? d.bias[c] : 0.f));
}

template <typename T> __host__ __device__ constexpr int kc_of() { return sizeof(T) == 2 ? 32 : 16; }
static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }
__device__ __forceinline__ int round_up_d(int a, int b) { return (a + b - 1) / b * b; }

}  // namespace unet
