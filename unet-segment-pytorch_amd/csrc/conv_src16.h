// conv_src16.h — the 16-bit conv kernels' halo staging: buffer-resource loads of virtual activations
// (conv3_body.inc).  One 16-byte channel vector of one halo pixel per staged item:
//  * every global read is a buffer load (SGPR descriptor + 32-bit offset).  Zero padding, pixels
//    outside the placed up-sampled map and channels past the source all read as 0 through the
//    descriptor's range check (offset >= OOB), so no load sits behind a per-lane branch;
//  * the source feeding a staged chunk is wave-uniform, so the virtual-activation transform is a
//    uniform switch, and each item's pixel geometry (corner offsets, bilinear weights, attention-gate
//    value x validity) is computed once per source (conv3_geo) instead of once per chunk.
#pragma once
#include "halo_items.h"

namespace unet {

constexpr unsigned OOB = 0x40000000u;  // >= every source byte size the host admits (< 1 GiB)

typedef __amdgpu_buffer_rsrc_t rsrc_t;
__device__ __forceinline__ rsrc_t mk_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bld(rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
// compile-time knowledge of the sources (the kernel's SK parameter): SK_ANY switches on each source's kind
// at run time; SK_PLAIN: every source is a stored map (dgrad inputs, materialised pool / upsample);
// SK_ACT: one BN(+ReLU)(+attention gate) source; SK_ACT_PLAIN: src0 BN(+ReLU)(+gate), src1 stored (the
// up-block conv0 [skip, up]).  Known kinds drop the other kinds' code and their live registers.
enum { SK_ANY = 0, SK_PLAIN = 1, SK_ACT = 2, SK_ACT_PLAIN = 3 };

// per halo item and source: corner byte offsets (>= OOB when outside) and weights
// (UP: bilinear weights, 0 outside; ACT / POOL: w[0] = validity x attention gate)
template <int RAW>
struct Geo {
  unsigned off[RAW];
  float w[RAW];
};

template <int RAW, int HWID, int HALO, int HP, int NT, int NV, int ITEMS, int SK = SK_ANY>
__device__ __forceinline__ void conv3_geo(const unet_conv_desc& d, const unet_src& s, int n, int h0, int w0, int tid,
                                          Geo<RAW> (&g)[ITEMS]) {
  const unsigned pixb = (unsigned)s.C * 2u;
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int hp = (tid + k * NT) / NV;
    const int y = h0 + hp / HWID - HALO, x = w0 + hp % HWID - HALO;
    const bool inb = hp < HP && y >= 0 && y < d.H && x >= 0 && x < d.W;
#pragma unroll
    for (int j = 0; j < RAW; ++j) { g[k].off[j] = OOB; g[k].w[j] = 0.f; }
    if (SK != SK_ANY || s.kind == UNET_SRC_PLAIN || s.kind == UNET_SRC_ACT) {
      if (inb) {
        const unsigned px = ((unsigned)n * s.H + y) * s.W + x;
        g[k].off[0] = px * pixb;
        if constexpr (SK != SK_PLAIN) g[k].w[0] = s.gate_p ? sigmoidf_(s.gate_p[px] * s.gate_ab[0] + s.gate_ab[1]) : 1.f;
      }
    } else if (s.kind == UNET_SRC_POOL_ACT) {
      if (inb) {
        g[k].off[0] = (((unsigned)n * s.H + 2 * y) * s.W + 2 * x) * pixb;
        g[k].w[0] = 1.f;
      }
    } else if (s.kind == UNET_SRC_UP_ACT) {
      if constexpr (RAW == 4) {
        const int uy = y - s.pad_t, ux = x - s.pad_l;
        if (inb && uy >= 0 && uy < s.up_h && ux >= 0 && ux < s.up_w) {
          int y0, y1, x0, x1;
          float ly, lx;
          lin_idx(s.sh, uy, s.H, y0, y1, ly);
          lin_idx(s.sw, ux, s.W, x0, x1, lx);
          const unsigned r0 = ((unsigned)n * s.H + y0) * s.W, r1 = ((unsigned)n * s.H + y1) * s.W;
          g[k].off[0] = (r0 + x0) * pixb;
          g[k].off[1] = (r0 + x1) * pixb;
          g[k].off[2] = (r1 + x0) * pixb;
          g[k].off[3] = (r1 + x1) * pixb;
          const float hy0 = 1.f - ly, wx0 = 1.f - lx;
          g[k].w[0] = hy0 * wx0;
          g[k].w[1] = hy0 * lx;
          g[k].w[2] = ly * wx0;
          g[k].w[3] = ly * lx;
        }
      }
    } else {  // UNET_SRC_UP_PLAIN
      const int uy = y - s.pad_t, ux = x - s.pad_l;
      if (inb && uy >= 0 && uy < s.up_h && ux >= 0 && ux < s.up_w)
        g[k].off[0] = (((unsigned)n * s.H + uy) * s.W + ux) * pixb;
    }
  }
}

// wave-uniform view of the source of one chunk plus this lane's channel vector
struct ChunkV {
  rsrc_t rs;
  unsigned cb;     // byte offset of the lane's 8 channels inside a pixel (>= OOB past the source)
  unsigned pixb, rowb;
  int kind;
  float lo;        // ReLU floor: 0 or -inf
  float sc[8], sf[8];
};

template <int RAW, int ABL = 0, int SK = SK_ANY>
__device__ __forceinline__ void conv3_view(const unet_conv_desc& d, int si, int cl0, int v, ChunkV& cv) {
  const unet_src& s = d.src[si];
  cv.kind = s.kind;
  cv.pixb = (unsigned)s.C * 2u;
  cv.rowb = cv.pixb * (unsigned)s.W;
  cv.rs = mk_rsrc(s.data, (unsigned)((long long)d.N * s.H * s.W) * cv.pixb);
  const int cl = cl0 + v * 8;
  const bool cok = cl < s.C;
  cv.cb = cok ? (unsigned)cl * 2u : OOB;
  cv.lo = s.relu ? 0.f : -INFINITY;
  if constexpr (SK == SK_PLAIN) return;
  const bool act = SK == SK_ACT || s.kind == UNET_SRC_ACT || s.kind == UNET_SRC_POOL_ACT || s.kind == UNET_SRC_UP_ACT;
  if (act && (ABL & 16)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { cv.sc[j] = 1.f; cv.sf[j] = 0.f; }
  } else if (act) {
    // channels past the source get scale = shift = 0, so their activation is exactly 0
    const rsrc_t rsc = mk_rsrc(s.scale, (unsigned)s.C * 4u), rsf = mk_rsrc(s.shift, (unsigned)s.C * 4u);
    const unsigned o = cok ? (unsigned)cl * 4u : OOB;
    const uint4 a0 = bld(rsc, o, 0), a1 = bld(rsc, o + 16u, 0), b0 = bld(rsf, o, 0), b1 = bld(rsf, o + 16u, 0);
    const unsigned ua[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const unsigned ub[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) { cv.sc[j] = __uint_as_float(ua[j]); cv.sf[j] = __uint_as_float(ub[j]); }
  }
}

template <int RAW, int SK = SK_ANY>
__device__ __forceinline__ void conv3_issue(const ChunkV& cv, const Geo<RAW>& g, uint4 (&q)[RAW]) {
  if constexpr (SK != SK_ANY) {
    q[0] = bld(cv.rs, g.off[0] + cv.cb, 0);
    return;
  }
  if (cv.kind == UNET_SRC_POOL_ACT) {
    if constexpr (RAW == 4) {
      const unsigned o = g.off[0] + cv.cb;
      q[0] = bld(cv.rs, o, 0);
      q[1] = bld(cv.rs, o + cv.pixb, 0);
      q[2] = bld(cv.rs, o, cv.rowb);
      q[3] = bld(cv.rs, o + cv.pixb, cv.rowb);
    }
  } else if (cv.kind == UNET_SRC_UP_ACT) {
    if constexpr (RAW == 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) q[j] = bld(cv.rs, g.off[j] + cv.cb, 0);
    }
  } else {
    q[0] = bld(cv.rs, g.off[0] + cv.cb, 0);
  }
}

template <typename T, int RAW, int ABL = 0, int SK = SK_ANY>
__device__ __forceinline__ uint4 conv3_finish(const ChunkV& cv, const Geo<RAW>& g, const uint4 (&q)[RAW]) {
  if constexpr ((ABL & 32) != 0 || SK == SK_PLAIN) return q[0];
  float v[8];
  if (SK == SK_ACT || cv.kind == UNET_SRC_ACT) {
    unpack16<T>(q[0], v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j] * cv.sc[j] + cv.sf[j], cv.lo) * g.w[0];
    return pack8_16<T>(v);
  }
  if constexpr (SK != SK_ANY) return q[0];  // SK_ACT_PLAIN: the stored source
  if constexpr (RAW == 4) {
    if (cv.kind == UNET_SRC_POOL_ACT) {
      float t0[8], t1[8], t2[8], t3[8];
      unpack16<T>(q[0], t0);
      unpack16<T>(q[1], t1);
      unpack16<T>(q[2], t2);
      unpack16<T>(q[3], t3);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float mx = fmaxf(fmaxf(t0[j], t1[j]), fmaxf(t2[j], t3[j]));
        const float mn = fminf(fminf(t0[j], t1[j]), fminf(t2[j], t3[j]));
        v[j] = fmaxf((cv.sc[j] >= 0.f ? mx : mn) * cv.sc[j] + cv.sf[j], cv.lo) * g.w[0];
      }
      return pack8_16<T>(v);
    }
    if (cv.kind == UNET_SRC_UP_ACT) {
      float t0[8], t1[8], t2[8], t3[8];
      unpack16<T>(q[0], t0);
      unpack16<T>(q[1], t1);
      unpack16<T>(q[2], t2);
      unpack16<T>(q[3], t3);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a0 = fmaxf(t0[j] * cv.sc[j] + cv.sf[j], cv.lo), a1 = fmaxf(t1[j] * cv.sc[j] + cv.sf[j], cv.lo);
        const float a2 = fmaxf(t2[j] * cv.sc[j] + cv.sf[j], cv.lo), a3 = fmaxf(t3[j] * cv.sc[j] + cv.sf[j], cv.lo);
        v[j] = g.w[0] * a0 + g.w[1] * a1 + g.w[2] * a2 + g.w[3] * a3;
      }
      return pack8_16<T>(v);
    }
  }
  return q[0];  // PLAIN / UP_PLAIN: stored bf16 as is (range-checked zeros outside)
}

// sum over the 16 lanes of a DPP row (rows: lanes 0-15, 16-31, ...); every lane receives its row's total
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xf, 0xf, false));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x122, 0xf, 0xf, false));  // row_ror:2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x121, 0xf, 0xf, false));  // row_ror:1
  return v;
}

}  // namespace unet
