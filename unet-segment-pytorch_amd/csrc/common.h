// common.h — shared device helpers for the gfx950 (CDNA4) Attention-U-Net kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "unet_hip.h"

namespace unet {

typedef __bf16 bf16;
typedef _Float16 f16;   // fp16 operand mode (BASELINE C5): same 16-bit storage and MFMA rate as bf16
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) short i16x4;

constexpr int WAVE = 64;

// ------------------------------------------------------------------------------------------------
// element traits: a 16-byte vector of T, conversions to/from float
// ------------------------------------------------------------------------------------------------
template <typename T> struct Vec;
template <> struct Vec<float> {
  static constexpr int N = 4;
  typedef float4 type;
};
template <> struct Vec<bf16> {
  static constexpr int N = 8;
  typedef uint4 type;
};
template <> struct Vec<f16> {
  static constexpr int N = 8;
  typedef uint4 type;
};

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(f16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ f16 from_f<f16>(float x) { return (f16)x; }

// an fp32 result the compiler may not fold into the 16-bit conversion that follows: fptrunc(fma) contracts to
// v_fma_mix{lo,hi}_f16 (the exact fma rounded once, straight to 16 bits) wherever the instruction selector finds the
// pattern, so two instantiations of one expression could round an element differently (round 6: the pooled and
// plain BN-backward applies); behind this, every path rounds to fp32 first, then to the storage type
__device__ __forceinline__ float f32_rounded(float x) {
  __asm__("" : "+v"(x));
  return x;
}

// load VEC elements (16 B aligned) into floats
template <typename T> __device__ __forceinline__ void load_vec(const T* p, float* v);
template <> __device__ __forceinline__ void load_vec<float>(const float* p, float* v) {
  float4 q = *reinterpret_cast<const float4*>(p);
  v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
}
template <> __device__ __forceinline__ void load_vec<bf16>(const bf16* p, float* v) {
  uint4 q = *reinterpret_cast<const uint4*>(p);
  unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(u[i] << 16);
    v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
  }
}
template <> __device__ __forceinline__ void load_vec<f16>(const f16* p, float* v) {
  const f16x8 q = *reinterpret_cast<const f16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)q[i];
}
template <typename T> __device__ __forceinline__ void store_vec(T* p, const float* v);
template <> __device__ __forceinline__ void store_vec<float>(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
template <> __device__ __forceinline__ void store_vec<f16>(f16* p, const float* v) {
  f16x8 q;
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = (f16)v[i];
  *reinterpret_cast<f16x8*>(p) = q;
}
template <> __device__ __forceinline__ void store_vec<bf16>(bf16* p, const float* v) {
  bf16 b[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) b[i] = (bf16)v[i];
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(b);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// ------------------------------------------------------------------------------------------------
// wave reductions (wave64)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// XCD-aware block order (cdna_hip_programming.md T1): the hardware deals blocks b, b + 8, ... to one XCD; this
// bijection on [0, nb) gives each XCD a contiguous range of logical blocks, so neighbouring logical blocks (which
// share input rows) share one L2.  Speed only: correctness never depends on the placement.
__device__ __forceinline__ unsigned xcd_block(unsigned b, unsigned nb) {
  const unsigned q = nb >> 3, r = nb & 7u, x = b & 7u, k = b >> 3;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + k;
}

// ------------------------------------------------------------------------------------------------
// error plumbing
// ------------------------------------------------------------------------------------------------
void set_error(const char* msg);
int check_launch(const char* what);

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// 16-byte vector of 8 x 16-bit values <-> 8 floats, for either 16-bit operand type
template <typename T>
__device__ __forceinline__ void unpack8_16(const uint4& q, float* v) {
  if constexpr (__is_same(T, bf16)) {
    const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  } else {
    const f16x8 h = __builtin_bit_cast(f16x8, q);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)h[i];
  }
}
// two floats -> one dword of two 16-bit values, round to nearest even: __builtin_convertvector on a float2 is
// one v_cvt_pk_{bf16,f16}_f32 (two scalar conversions compiled to two converts and a v_perm)
template <typename T>
__device__ __forceinline__ unsigned pack2_16(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  if constexpr (__is_same(T, bf16)) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{a, b}), bf16x2));
  } else {
    typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2{a, b}), f16x2));
  }
}
template <typename T>
__device__ __forceinline__ uint4 pack8_16(const float* v) {
  return make_uint4(pack2_16<T>(v[0], v[1]), pack2_16<T>(v[2], v[3]), pack2_16<T>(v[4], v[5]),
                    pack2_16<T>(v[6], v[7]));
}

// run `body` with T = float / bf16 / f16 for a UNET_F32 / UNET_BF16 / UNET_F16 code
#define UNET_DISPATCH_T(code, ...)                                  \
  ((code) == UNET_BF16 ? [&]() { using T = bf16; return __VA_ARGS__; }()  \
   : (code) == UNET_F16 ? [&]() { using T = f16; return __VA_ARGS__; }()  \
                        : [&]() { using T = float; return __VA_ARGS__; }())

}  // namespace unet
