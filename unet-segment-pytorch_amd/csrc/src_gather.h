// src_gather.h — the "virtual activation" reader shared by the conv / wgrad tile loaders.
//
// A conv input channel range is described by a unet_src: a stored NHWC tensor plus the transform
// that the reference applies between layers (BN-apply + ReLU, MaxPool2d(2), bilinear x2 with
// align_corners=True, F.pad, the attention multiply x*sigmoid(psi)).  The loaders call
// src_gather() once per staged 16-byte LDS vector, so none of these intermediates ever exist in
// HBM.  Reference: unet/models/layers.py:34-37 (ReLU after BN), :56 (MaxPool2d(2)),
// :78/:183/:212 (bilinear, align_corners=True), :101/:250 (pad), :192 (x * attention).
#pragma once
#include "common.h"

namespace unet {

// PyTorch's linear-interpolation index/lambda rule for align_corners=True
// (area_pixel_compute_source_index + guard_index_and_lambda, fp32 opmath).
__device__ __forceinline__ void lin_idx(float scale, int dst, int in_size, int& i0, int& i1, float& l1) {
  float r = scale * (float)dst;
  int i = (int)floorf(r);
  i = i < in_size - 1 ? i : in_size - 1;
  float l = r - (float)i;
  l = fminf(fmaxf(l, 0.f), 1.f);
  i0 = i;
  i1 = i + ((i < in_size - 1) ? 1 : 0);
  l1 = l;
}

template <typename T>
__device__ __forceinline__ void act_vec(const unet_src& s, int c, int cnt, float* v) {
#pragma unroll
  for (int j = 0; j < Vec<T>::N; ++j) {
    if (j < cnt) {
      float x = v[j] * s.scale[c + j] + s.shift[c + j];
      v[j] = s.relu ? fmaxf(x, 0.f) : x;
    }
  }
}

// load channels [c, c+cnt) of stored tensor s at stored pixel (n, y, x) as floats (raw, no act)
template <typename T>
__device__ __forceinline__ void raw_vec(const unet_src& s, long long n, int y, int x, int c, int cnt, float* v) {
  constexpr int VEC = Vec<T>::N;
  const T* base = (const T*)s.data + (((n * s.H + y) * (long long)s.W + x) * s.C + c);
  if (cnt == VEC && (s.C % VEC) == 0 && (c % VEC) == 0) {
    load_vec<T>(base, v);
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = (j < cnt) ? to_f(base[j]) : 0.f;
  }
}

template <typename T>
__device__ void src_gather_one(const unet_src& s, long long n, int y, int x, int cl, int cnt, float* v);

// Gather VEC channels [c, c+VEC) of the (virtual, concatenated) conv input at conv-input pixel (n, y, x).
// Channels >= Cin and pixels outside [0,H)x[0,W) read as zero (the conv's zero padding).
template <typename T>
__device__ __forceinline__ void src_gather(const unet_src* srcs, int nsrc, int Cin, int H, int W, long long n,
                                           int y, int x, int c, float* v) {
  constexpr int VEC = Vec<T>::N;
#pragma unroll
  for (int j = 0; j < VEC; ++j) v[j] = 0.f;
  if (y < 0 || y >= H || x < 0 || x >= W || c >= Cin) return;
  if (nsrc > 1 && c < srcs[0].C && c + VEC > srcs[0].C) {
    // the vector straddles the concat boundary (skip channels not a multiple of VEC): two halves
    float a[VEC], b[VEC];
    const int n0 = srcs[0].C - c;
    src_gather_one<T>(srcs[0], n, y, x, c, n0, a);
    src_gather_one<T>(srcs[1], n, y, x, 0, VEC - n0 < srcs[1].C ? VEC - n0 : srcs[1].C, b);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float r = a[j];
#pragma unroll
      for (int k = 0; k < VEC; ++k)
        if (j >= n0 && k == j - n0) r = b[k];
      v[j] = r;
    }
    return;
  }
  int si = 0;
  int cl = c;
  if (nsrc > 1 && c >= srcs[0].C) { si = 1; cl = c - srcs[0].C; }
  const unet_src& s = srcs[si];
  int cnt = s.C - cl;
  cnt = cnt < VEC ? cnt : VEC;
  src_gather_one<T>(s, n, y, x, cl, cnt, v);
}

// channels [cl, cl+cnt) of one source (cnt <= VEC), rest zero
template <typename T>
__device__ void src_gather_one(const unet_src& s, long long n, int y, int x, int cl, int cnt, float* v) {
  constexpr int VEC = Vec<T>::N;
#pragma unroll
  for (int j = 0; j < VEC; ++j) v[j] = 0.f;
  switch (s.kind) {
    case UNET_SRC_PLAIN:
      raw_vec<T>(s, n, y, x, cl, cnt, v);
      break;
    case UNET_SRC_ACT: {
      raw_vec<T>(s, n, y, x, cl, cnt, v);
      act_vec<T>(s, cl, cnt, v);
      if (s.gate_p) {
        float p = s.gate_p[(n * s.H + y) * (long long)s.W + x];
        float g = sigmoidf_(p * s.gate_ab[0] + s.gate_ab[1]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] *= g;
      }
    } break;
    case UNET_SRC_POOL_ACT: {
      float m[VEC];
      float t[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) m[j] = -INFINITY;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        raw_vec<T>(s, n, 2 * y + (q >> 1), 2 * x + (q & 1), cl, cnt, t);
        act_vec<T>(s, cl, cnt, t);
#pragma unroll
        for (int j = 0; j < VEC; ++j) m[j] = (t[j] > m[j] || t[j] != t[j]) ? t[j] : m[j];
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] = (j < cnt) ? m[j] : 0.f;
    } break;
    case UNET_SRC_UP_ACT: {
      int uy = y - s.pad_t, ux = x - s.pad_l;
      if (uy < 0 || uy >= s.up_h || ux < 0 || ux >= s.up_w) return;
      int y0, y1, x0, x1;
      float ly, lx;
      lin_idx(s.sh, uy, s.H, y0, y1, ly);
      lin_idx(s.sw, ux, s.W, x0, x1, lx);
      float a[VEC], b[VEC], cc[VEC], dd[VEC];
      raw_vec<T>(s, n, y0, x0, cl, cnt, a);
      raw_vec<T>(s, n, y0, x1, cl, cnt, b);
      raw_vec<T>(s, n, y1, x0, cl, cnt, cc);
      raw_vec<T>(s, n, y1, x1, cl, cnt, dd);
      act_vec<T>(s, cl, cnt, a);
      act_vec<T>(s, cl, cnt, b);
      act_vec<T>(s, cl, cnt, cc);
      act_vec<T>(s, cl, cnt, dd);
      const float hy0 = 1.f - ly, wx0 = 1.f - lx;
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        v[j] = (j < cnt) ? hy0 * (wx0 * a[j] + lx * b[j]) + ly * (wx0 * cc[j] + lx * dd[j]) : 0.f;
    } break;
    case UNET_SRC_NCHW_F32: {
      const float* base = (const float*)s.data;
      const long long plane = (long long)s.H * s.W;
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        v[j] = (j < cnt) ? base[(n * s.C + cl + j) * plane + (long long)y * s.W + x] : 0.f;
    } break;
    case UNET_SRC_UP_PLAIN: {
      int uy = y - s.pad_t, ux = x - s.pad_l;
      if (uy < 0 || uy >= s.up_h || ux < 0 || ux >= s.up_w) return;
      raw_vec<T>(s, n, uy, ux, cl, cnt, v);
    } break;
    default:
      break;
  }
}

}  // namespace unet
