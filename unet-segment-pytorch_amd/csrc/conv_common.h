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

// packed weight rows (Cout, or Cin for the transposed dgrad weights) are padded to this: the largest
// output-channel block of any conv kernel (unet_packed_weight_elems, pack.hip, conv5.hip)
constexpr int PACK_NPAD = 128;

template <typename T> __host__ __device__ constexpr int kc_of() { return sizeof(T) == 2 ? 32 : 16; }
static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }
__device__ __forceinline__ int round_up_d(int a, int b) { return (a + b - 1) / b * b; }


// internal output mode of the conv kernels: the y epilogue of a dgrad that also reduces the BatchNorm
// backward sums of the activation it is the gradient of (unet_conv_desc.bnb_*)
constexpr int OM_Y_BNB = 8;

// 4 x 16-bit values (8 bytes) -> 4 floats
template <typename T>
__device__ __forceinline__ void unpack4_16(const uint2& q, float* v) {
  if constexpr (__is_same(T, bf16)) {
    v[0] = __uint_as_float(q.x << 16);
    v[1] = __uint_as_float(q.x & 0xffff0000u);
    v[2] = __uint_as_float(q.y << 16);
    v[3] = __uint_as_float(q.y & 0xffff0000u);
  } else {
    typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
    const f16x4 h = __builtin_bit_cast(f16x4, q);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (float)h[i];
  }
}

}  // namespace unet
