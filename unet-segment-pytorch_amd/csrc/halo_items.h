// halo_items.h — software-pipelined tile gather shared by the conv and wgrad kernels.
//
// A thread owns a fixed 16-byte channel vector of a staged tile.  item_issue() issues the raw global
// loads of one staged vector (1 load, or the 4 corners of a max-pool window / bilinear tap), so they
// can be in flight under MFMAs; item_finish() later applies the virtual-activation transform
// (BN-apply + ReLU, max-pool, bilinear, attention gate; see src_gather.h) and returns the floats to
// store into LDS.  Only "fast" sources (C % VEC == 0, NHWC) use this path.
//
// VALU economy (the transform runs beside MFMAs, so every instruction counts): 32-bit byte offsets
// from a per-chunk base pointer; max-pool as relu(s * (s >= 0 ? max : min) + b) over the raw values
// (BN-apply is monotone per channel, so only one affine per channel instead of four; NaNs are not
// propagated); bilinear weights formed once per item.
#pragma once
#include "conv_common.h"

#ifndef UNET_PK_UP
#define UNET_PK_UP 1   // the bilinear source transform on packed fp32 (0: the per-element form, for A/B builds;
                       // round-4 A/B: materialise 169 -> 141 us/step)
#endif

namespace unet {

template <typename T>
__device__ __forceinline__ void unpack16(const uint4& q, float* v) {
  if constexpr (sizeof(T) == 2) {
    unpack8_16<T>(q, v);
  } else {
    v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
  }
}

// per-chunk view of the source that owns a thread's channel vector
struct SrcView {
  const char* base;      // data + cl * sizeof(T): the thread's 16-byte channel vector of pixel 0
  const float* gate_p;
  const float* gate_ab;
  unsigned pixb;         // bytes per pixel (C * sizeof(T))
  int kind, H, W, relu, up_h, up_w, pad_t, pad_l, fast;
  float sh, sw;
};

template <int RAW>
struct Item {
  uint4 q[RAW];
  float w0, w1, w2, w3;  // bilinear weights (UP) ; w0 = gate pre-activation (ACT with gate)
  int mode;              // 0 zero, 1 plain, 2 act, 3 pool, 4 up
};

__device__ __forceinline__ uint4 ld16b(const char* base, unsigned byte_off) {
  return *reinterpret_cast<const uint4*>(base + byte_off);
}

template <typename T, int RAW>
__device__ __forceinline__ void item_issue(const SrcView& s, int H, int W, int n, int y, int x, int valid,
                                           Item<RAW>& it) {
  it.mode = 0;
  if (!valid || y < 0 || y >= H || x < 0 || x >= W) return;
  if (!s.fast) return;  // channels beyond Cin (the host routes every other non-fast case to conv_generic)
  switch (s.kind) {
    case UNET_SRC_PLAIN: {
      const unsigned px = ((unsigned)n * s.H + y) * s.W + x;
      it.q[0] = ld16b(s.base, px * s.pixb);
      it.mode = 1;
    } break;
    case UNET_SRC_ACT: {
      const unsigned px = ((unsigned)n * s.H + y) * s.W + x;
      it.q[0] = ld16b(s.base, px * s.pixb);
      it.w0 = s.gate_p ? s.gate_p[px] : 0.f;
      it.mode = 2;
    } break;
    case UNET_SRC_POOL_ACT:
      if constexpr (RAW == 4) {
        const unsigned p0 = ((unsigned)n * s.H + 2 * y) * s.W + 2 * x;
        const unsigned rb = s.W * s.pixb;
        it.q[0] = ld16b(s.base, p0 * s.pixb);
        it.q[1] = ld16b(s.base, p0 * s.pixb + s.pixb);
        it.q[2] = ld16b(s.base, p0 * s.pixb + rb);
        it.q[3] = ld16b(s.base, p0 * s.pixb + rb + s.pixb);
        it.mode = 3;
      }
      break;
    case UNET_SRC_UP_ACT: {
      const int uy = y - s.pad_t, ux = x - s.pad_l;
      if (uy < 0 || uy >= s.up_h || ux < 0 || ux >= s.up_w) return;
      if constexpr (RAW == 4) {
        int y0, y1, x0, x1;
        float ly, lx;
        lin_idx(s.sh, uy, s.H, y0, y1, ly);
        lin_idx(s.sw, ux, s.W, x0, x1, lx);
        const unsigned r0 = ((unsigned)n * s.H + y0) * s.W, r1 = ((unsigned)n * s.H + y1) * s.W;
        it.q[0] = ld16b(s.base, (r0 + x0) * s.pixb);
        it.q[1] = ld16b(s.base, (r0 + x1) * s.pixb);
        it.q[2] = ld16b(s.base, (r1 + x0) * s.pixb);
        it.q[3] = ld16b(s.base, (r1 + x1) * s.pixb);
        const float hy0 = 1.f - ly, wx0 = 1.f - lx;
        it.w0 = hy0 * wx0;
        it.w1 = hy0 * lx;
        it.w2 = ly * wx0;
        it.w3 = ly * lx;
        it.mode = 4;
      }
    } break;
    case UNET_SRC_UP_PLAIN: {
      const int uy = y - s.pad_t, ux = x - s.pad_l;
      if (uy < 0 || uy >= s.up_h || ux < 0 || ux >= s.up_w) return;
      const unsigned px = ((unsigned)n * s.H + uy) * s.W + ux;
      it.q[0] = ld16b(s.base, px * s.pixb);
      it.mode = 1;
    } break;
    default:
      break;
  }
}

template <typename T, int RAW, typename D>
__device__ __forceinline__ void item_finish(const D& d, const SrcView& s, const float* sc, const float* sf,
                                            int n, int y, int x, int c, const Item<RAW>& it, float* v) {
  constexpr int VEC = Vec<T>::N;
  const int mode = it.mode;
  if (mode == 1) {
    unpack16<T>(it.q[0], v);
  } else if (mode == 2) {
    unpack16<T>(it.q[0], v);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float a = v[j] * sc[j] + sf[j];
      v[j] = s.relu ? fmaxf(a, 0.f) : a;
    }
    if (s.gate_p) {
      const float g = sigmoidf_(it.w0 * s.gate_ab[0] + s.gate_ab[1]);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] *= g;
    }
  } else if (mode == 3) {
    if constexpr (RAW == 4) {
      float t0[VEC], t1[VEC], t2[VEC], t3[VEC];
      unpack16<T>(it.q[0], t0);
      unpack16<T>(it.q[1], t1);
      unpack16<T>(it.q[2], t2);
      unpack16<T>(it.q[3], t3);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float mx = fmaxf(fmaxf(t0[j], t1[j]), fmaxf(t2[j], t3[j]));
        const float mn = fminf(fminf(t0[j], t1[j]), fminf(t2[j], t3[j]));
        const float a = (sc[j] >= 0.f ? mx : mn) * sc[j] + sf[j];
        v[j] = s.relu ? fmaxf(a, 0.f) : a;
      }
    }
  } else if (mode == 4) {
    if constexpr (RAW == 4) {
      float t0[VEC], t1[VEC], t2[VEC], t3[VEC];
      unpack16<T>(it.q[0], t0);
      unpack16<T>(it.q[1], t1);
      unpack16<T>(it.q[2], t2);
      unpack16<T>(it.q[3], t3);
#if UNET_PK_UP
      // channel pairs on packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: half the VALU of the BN apply and the blend;
      // ReLU stays per element, gfx950 has no packed fp32 max)
      typedef __attribute__((ext_vector_type(2))) float f2;
      const f2 w0 = {it.w0, it.w0}, w1 = {it.w1, it.w1}, w2 = {it.w2, it.w2}, w3 = {it.w3, it.w3};
#pragma unroll
      for (int j = 0; j < VEC; j += 2) {
        const f2 c = {sc[j], sc[j + 1]}, f = {sf[j], sf[j + 1]};
        f2 a0 = __builtin_elementwise_fma(f2{t0[j], t0[j + 1]}, c, f);
        f2 a1 = __builtin_elementwise_fma(f2{t1[j], t1[j + 1]}, c, f);
        f2 a2 = __builtin_elementwise_fma(f2{t2[j], t2[j + 1]}, c, f);
        f2 a3 = __builtin_elementwise_fma(f2{t3[j], t3[j + 1]}, c, f);
        if (s.relu) {
          a0 = f2{fmaxf(a0[0], 0.f), fmaxf(a0[1], 0.f)};
          a1 = f2{fmaxf(a1[0], 0.f), fmaxf(a1[1], 0.f)};
          a2 = f2{fmaxf(a2[0], 0.f), fmaxf(a2[1], 0.f)};
          a3 = f2{fmaxf(a3[0], 0.f), fmaxf(a3[1], 0.f)};
        }
        const f2 r = __builtin_elementwise_fma(w3, a3, __builtin_elementwise_fma(w2, a2, __builtin_elementwise_fma(w1, a1, w0 * a0)));
        v[j] = r[0];
        v[j + 1] = r[1];
      }
#else
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float a0 = t0[j] * sc[j] + sf[j], a1 = t1[j] * sc[j] + sf[j];
        float a2 = t2[j] * sc[j] + sf[j], a3 = t3[j] * sc[j] + sf[j];
        if (s.relu) { a0 = fmaxf(a0, 0.f); a1 = fmaxf(a1, 0.f); a2 = fmaxf(a2, 0.f); a3 = fmaxf(a3, 0.f); }
        v[j] = it.w0 * a0 + it.w1 * a1 + it.w2 * a2 + it.w3 * a3;
      }
#endif
    }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = 0.f;
  }
}

// D: unet_conv_desc or unet_wgrad_desc (both carry nsrc / src[2] / Cin)
template <typename T, typename D>
__device__ __forceinline__ void make_view(const D& d, int c, SrcView& s, float* sc, float* sf) {
  constexpr int VEC = Vec<T>::N;
  const int si = (d.nsrc > 1 && c >= d.src[0].C) ? 1 : 0;
  const unet_src& u = d.src[si];
  const int cl = c - (si ? d.src[0].C : 0);
  s.base = (const char*)u.data + (long long)cl * (long long)sizeof(T);
  s.pixb = (unsigned)u.C * (unsigned)sizeof(T);
  s.gate_p = u.gate_p;
  s.gate_ab = u.gate_ab;
  s.kind = u.kind;
  s.H = u.H; s.W = u.W; s.relu = u.relu;
  s.up_h = u.up_h; s.up_w = u.up_w; s.pad_t = u.pad_t; s.pad_l = u.pad_l;
  s.sh = u.sh; s.sw = u.sw;
  const bool straddle = d.nsrc > 1 && si == 0 && c + VEC > u.C;
  s.fast = (c < d.Cin) && !straddle && (cl + VEC <= u.C) && (u.C % VEC == 0) && (cl % VEC == 0) &&
           u.kind != UNET_SRC_NCHW_F32;
  const bool act = u.kind == UNET_SRC_ACT || u.kind == UNET_SRC_POOL_ACT || u.kind == UNET_SRC_UP_ACT;
  if (s.fast && act) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) { sc[j] = u.scale[cl + j]; sf[j] = u.shift[cl + j]; }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) { sc[j] = 1.f; sf[j] = 0.f; }
  }
}

}  // namespace unet
