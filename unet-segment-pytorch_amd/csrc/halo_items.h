// halo_items.h — software-pipelined tile gather shared by the conv and wgrad kernels.
//
// A thread owns a fixed 16-byte channel vector of a staged tile.  item_issue() issues the raw global
// loads of one staged vector (1 load, or the 4 corners of a max-pool window / bilinear tap), so they
// can be in flight under MFMAs; item_finish() later applies the virtual-activation transform
// (BN-apply + ReLU, max-pool, bilinear, attention gate; see src_gather.h) and returns the floats to
// store into LDS.  Only "fast" sources (C % VEC == 0, NHWC) use this path.
#pragma once
#include "conv_common.h"

namespace unet {

template <typename T>
__device__ __forceinline__ void unpack16(const uint4& q, float* v) {
  if constexpr (sizeof(T) == 2) {
    const unsigned u[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(u[i] << 16);
      v[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  } else {
    v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
  }
}

// per-chunk view of the source that owns a thread's channel vector
struct SrcView {
  const char* data;
  const float* gate_p;
  const float* gate_ab;
  int kind, C, H, W, relu, up_h, up_w, pad_t, pad_l, cl, fast;
  float sh, sw;
};

template <int RAW>
struct Item {
  uint4 q[RAW];
  float la, lb, pg;
  int mode;   // 0 zero, 1 plain, 2 act, 3 pool, 4 up, 5 slow (full gather at finish time)
};

template <typename T>
__device__ __forceinline__ uint4 ld16(const char* base, long long elem) {
  return *reinterpret_cast<const uint4*>(base + elem * (long long)sizeof(T));
}

template <typename T, int RAW>
__device__ __forceinline__ void item_issue(const SrcView& s, int H, int W, long long n, int y, int x, int valid,
                                           Item<RAW>& it) {
  it.mode = 0;
  if (!valid || y < 0 || y >= H || x < 0 || x >= W) return;
  if (!s.fast) return;  // channels beyond Cin (the host routes every other non-fast case to conv_generic)
  switch (s.kind) {
    case UNET_SRC_PLAIN:
      it.q[0] = ld16<T>(s.data, ((n * s.H + y) * (long long)s.W + x) * s.C + s.cl);
      it.mode = 1;
      break;
    case UNET_SRC_ACT: {
      const long long px = (n * s.H + y) * (long long)s.W + x;
      it.q[0] = ld16<T>(s.data, px * s.C + s.cl);
      it.pg = s.gate_p ? s.gate_p[px] : 0.f;
      it.mode = 2;
    } break;
    case UNET_SRC_POOL_ACT:
      if constexpr (RAW == 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          it.q[q] = ld16<T>(s.data, ((n * s.H + 2 * y + (q >> 1)) * (long long)s.W + 2 * x + (q & 1)) * s.C + s.cl);
        it.mode = 3;
      } else {
        it.mode = 5;
      }
      break;
    case UNET_SRC_UP_ACT: {
      const int uy = y - s.pad_t, ux = x - s.pad_l;
      if (uy < 0 || uy >= s.up_h || ux < 0 || ux >= s.up_w) return;
      if constexpr (RAW == 4) {
        int y0, y1, x0, x1;
        lin_idx(s.sh, uy, s.H, y0, y1, it.la);
        lin_idx(s.sw, ux, s.W, x0, x1, it.lb);
        const long long r0 = (n * s.H + y0) * (long long)s.W, r1 = (n * s.H + y1) * (long long)s.W;
        it.q[0] = ld16<T>(s.data, (r0 + x0) * s.C + s.cl);
        it.q[1] = ld16<T>(s.data, (r0 + x1) * s.C + s.cl);
        it.q[2] = ld16<T>(s.data, (r1 + x0) * s.C + s.cl);
        it.q[3] = ld16<T>(s.data, (r1 + x1) * s.C + s.cl);
        it.mode = 4;
      } else {
        it.mode = 5;
      }
    } break;
    case UNET_SRC_UP_PLAIN: {
      const int uy = y - s.pad_t, ux = x - s.pad_l;
      if (uy < 0 || uy >= s.up_h || ux < 0 || ux >= s.up_w) return;
      it.q[0] = ld16<T>(s.data, ((n * s.H + uy) * (long long)s.W + ux) * s.C + s.cl);
      it.mode = 1;
    } break;
    default:
      it.mode = 5;
      break;
  }
}

template <typename T, int RAW, typename D>
__device__ __forceinline__ void item_finish(const D& d, const SrcView& s, const float* sc,
                                            const float* sf, long long n, int y, int x, int c, const Item<RAW>& it,
                                            float* v) {
  constexpr int VEC = Vec<T>::N;
  const int mode = it.mode;
  if (mode == 0) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = 0.f;
  } else if (mode == 1) {
    unpack16<T>(it.q[0], v);
  } else if (mode == 2) {
    unpack16<T>(it.q[0], v);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float a = v[j] * sc[j] + sf[j];
      v[j] = s.relu ? fmaxf(a, 0.f) : a;
    }
    if (s.gate_p) {
      const float g = sigmoidf_(it.pg * s.gate_ab[0] + s.gate_ab[1]);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] *= g;
    }
  } else if (mode == 3 || mode == 4) {
    if constexpr (RAW == 4) {
      float t[4][VEC];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        unpack16<T>(it.q[q], t[q]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float a = t[q][j] * sc[j] + sf[j];
          t[q][j] = s.relu ? fmaxf(a, 0.f) : a;
        }
      }
      if (mode == 3) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float m = t[0][j];
#pragma unroll
          for (int q = 1; q < 4; ++q) m = (t[q][j] > m || t[q][j] != t[q][j]) ? t[q][j] : m;
          v[j] = m;
        }
      } else {
        const float ly = it.la, lx = it.lb, hy0 = 1.f - ly, wx0 = 1.f - lx;
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = hy0 * (wx0 * t[0][j] + lx * t[1][j]) + ly * (wx0 * t[2][j] + lx * t[3][j]);
      }
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
  s.data = (const char*)u.data;
  s.gate_p = u.gate_p;
  s.gate_ab = u.gate_ab;
  s.kind = u.kind;
  s.C = u.C; s.H = u.H; s.W = u.W; s.relu = u.relu;
  s.up_h = u.up_h; s.up_w = u.up_w; s.pad_t = u.pad_t; s.pad_l = u.pad_l;
  s.sh = u.sh; s.sw = u.sw;
  s.cl = c - (si ? d.src[0].C : 0);
  const bool straddle = d.nsrc > 1 && si == 0 && c + VEC > u.C;
  s.fast = (c < d.Cin) && !straddle && (s.cl + VEC <= u.C) && (u.C % VEC == 0) && (s.cl % VEC == 0) &&
           u.kind != UNET_SRC_NCHW_F32;
  const bool act = u.kind == UNET_SRC_ACT || u.kind == UNET_SRC_POOL_ACT || u.kind == UNET_SRC_UP_ACT;
  if (s.fast && act) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) { sc[j] = u.scale[s.cl + j]; sf[j] = u.shift[s.cl + j]; }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) { sc[j] = 1.f; sf[j] = 0.f; }
  }
}

}  // namespace unet
