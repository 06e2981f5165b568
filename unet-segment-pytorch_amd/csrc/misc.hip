// misc.hip — bilinear adjoint, NCHW resize (deep-supervision heads), OutConv, layout, fill.
#include "halo_items.h"

namespace unet {

// sum over destination indices u in [0, up) whose interpolation touches source index i
// (weight (1-l) on i0, l on i1 — PyTorch's linear rule, align_corners=True)
__device__ __forceinline__ void up_range(float scale, int i, int in_size, int up, int& lo, int& hi) {
  if (scale > 0.f) {
    lo = (int)floorf((float)(i - 1) / scale) - 1;
    hi = (int)ceilf((float)(i + 1) / scale) + 1;
    lo = lo < 0 ? 0 : lo;
    hi = hi > up - 1 ? up - 1 : hi;
  } else {
    lo = 0;
    hi = up - 1;
  }
}
__device__ __forceinline__ float up_weight(float scale, int u, int in_size, int i) {
  int i0, i1;
  float l;
  lin_idx(scale, u, in_size, i0, i1, l);
  return (i0 == i ? 1.f - l : 0.f) + (i1 == i ? l : 0.f);
}

// 4-channel vectorised form (C % 4 == 0): the index/weight arithmetic is shared by 4 channels
__global__ void upsample_bwd4_kernel(long long N, int C, int Hs, int Ws, int up_h, int up_w, int pt, int pl, int Hp,
                                     int Wp, float sh, float sw, const float* dup, float* dx, int accum) {
  const int C4 = C / 4;
  const long long total = N * Hs * (long long)Ws * C4;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int c4 = e % C4;
    long long t = e / C4;
    const int j = t % Ws;
    t /= Ws;
    const int i = t % Hs;
    const long long n = t / Hs;
    int ulo, uhi, vlo, vhi;
    up_range(sh, i, Hs, up_h, ulo, uhi);
    up_range(sw, j, Ws, up_w, vlo, vhi);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int u = ulo; u <= uhi; ++u) {
      const float wy = up_weight(sh, u, Hs, i);
      const int yy = u + pt;
      if (wy == 0.f || yy < 0 || yy >= Hp) continue;
      const float4* row = reinterpret_cast<const float4*>(dup + ((n * Hp + yy) * (long long)Wp) * C) + c4;
      for (int v = vlo; v <= vhi; ++v) {
        const float wx = up_weight(sw, v, Ws, j);
        const int xx = v + pl;
        if (wx == 0.f || xx < 0 || xx >= Wp) continue;
        const float4 g = row[(long long)xx * C4];
        const float w = wy * wx;
        acc.x += w * g.x; acc.y += w * g.y; acc.z += w * g.z; acc.w += w * g.w;
      }
    }
    float4* o = reinterpret_cast<float4*>(dx) + e;
    if (accum) {
      const float4 a = *o;
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    *o = acc;
  }
}

// same adjoint with the destination windows precomputed (host-checked: each window spans <= 8 rows /
// columns, true for every x2-or-less upsample): the 8 row and 8 column weights (0 outside
// the window, the padded frame or the source support) are computed once per element instead of inside
// the 2-D loop, and only the nonzero taps issue loads
// (I: element index type, unsigned when N*Hs*Ws*C/4 < 2^31 — 32-bit divisions, as materialize_fast_kernel)
template <typename I = unsigned>
__global__ __launch_bounds__(256) void upsample_bwd4w_kernel(long long N, int C, int Hs, int Ws, int up_h, int up_w,
                                                             int pt, int pl, int Hp, int Wp, float sh, float sw,
                                                             const float* dup, float* dx, int accum) {
  const int C4 = C / 4;
  const I total = (I)(N * Hs * (long long)Ws * C4);
  for (I e = (I)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (I)gridDim.x * blockDim.x) {
    I t = e / (I)C4;
    const int c4 = (int)(e - t * (I)C4);
    I t2 = t / (I)Ws;
    const int j = (int)(t - t2 * (I)Ws);
    t = t2 / (I)Hs;
    const int i = (int)(t2 - t * (I)Hs);
    const long long n = (long long)t;
    // u contributes to row i only if floor(sh*u) in {i-1, i}: u in [(i-1)/sh, (i+1)/sh] (+-1 guard)
    const int ulo = max(0, (int)ceilf((float)(i - 1) / sh) - 1), uhi = min(up_h - 1, (int)floorf((float)(i + 1) / sh) + 1);
    const int vlo = max(0, (int)ceilf((float)(j - 1) / sw) - 1), vhi = min(up_w - 1, (int)floorf((float)(j + 1) / sw) + 1);
    float wy[8], wx[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int u = ulo + k, v = vlo + k;
      const int yy = u + pt, xx = v + pl;
      wy[k] = (u <= uhi && yy >= 0 && yy < Hp) ? up_weight(sh, u, Hs, i) : 0.f;
      wx[k] = (v <= vhi && xx >= 0 && xx < Wp) ? up_weight(sw, v, Ws, j) : 0.f;
    }
    // the 4 channels as two packed fp32 pairs (v_pk_fma_f32): the same fused multiply-add per channel
    typedef __attribute__((ext_vector_type(2))) float f2;
    f2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
#pragma unroll
    for (int ky = 0; ky < 8; ++ky) {
      if (wy[ky] == 0.f) continue;
      const float4* row = reinterpret_cast<const float4*>(dup + ((n * Hp + ulo + ky + pt) * (long long)Wp) * C) + c4;
#pragma unroll
      for (int kx = 0; kx < 8; ++kx) {
        if (wx[kx] == 0.f) continue;
        const float4 g = row[(long long)(vlo + kx + pl) * C4];
        const float w = wy[ky] * wx[kx];
#if UNET_PK_UP
        const f2 ww = {w, w};
        a01 = __builtin_elementwise_fma(ww, f2{g.x, g.y}, a01);
        a23 = __builtin_elementwise_fma(ww, f2{g.z, g.w}, a23);
#else
        a01[0] += w * g.x; a01[1] += w * g.y; a23[0] += w * g.z; a23[1] += w * g.w;
#endif
      }
    }
    float4 acc = make_float4(a01[0], a01[1], a23[0], a23[1]);
    float4* o = reinterpret_cast<float4*>(dx) + e;
    if (accum) {
      const float4 a = *o;
      acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w;
    }
    *o = acc;
  }
}

// Tiled adjoint (round 5): a block owns one source row i of image n, UJ source columns and 64 channels.
//  phase 1 (vertical): t[v][c] = sum_u wy(u, i) d_up[u + pt][v + pl][c] for the tile's destination columns v, each
//    d_up vector loaded once per block (the block-uniform row window and weights: no per-element index math, no
//    divergent branches, ~11 independent 16-byte loads in flight per thread); t lands in LDS;
//  phase 2 (horizontal): dx[i][j][c] (+)= sum_v wx(v, j) t[v][c] from LDS, the column weights from a per-block
//    table of the window columns' (i0, lambda).
//  Logical blocks run (channel tile, column tile, row, image) fastest-first and are dealt contiguously per XCD
//    (xcd_block), so the d_up rows shared by source rows i and i + 1 are fetched into one XCD's L2 once; the
//    element-per-thread gather measured 1.44x its algorithmic HBM bytes.
//  Summation order: rows first, then columns (fixed: deterministic; fp32-rounding-level different from the
//  per-element kernel's w_y * w_x products).
constexpr int UPB_J = 16, UPB_CT = 16, UPB_VMAX = 56;
__global__ __launch_bounds__(256) void upsample_bwd_tile_kernel(int N, int C, int Hs, int Ws, int up_h, int up_w, int pt,
                                                                int pl, int Hp, int Wp, float sh, float sw,
                                                                const float* __restrict__ dup, float* dx, int accum,
                                                                int ntj, int ntc) {
  __shared__ float4 t[UPB_VMAX][UPB_CT];
  __shared__ int tab_i0[UPB_VMAX], tab_i1[UPB_VMAX];
  __shared__ float tab_l[UPB_VMAX];
  const int tid = threadIdx.x;
  const unsigned lb = xcd_block(blockIdx.x, gridDim.x);
  const int ct = (int)(lb % (unsigned)ntc);
  unsigned r = lb / (unsigned)ntc;
  const int jt = (int)(r % (unsigned)ntj);
  r /= (unsigned)ntj;
  const int i = (int)(r % (unsigned)Hs);
  const int n = (int)(r / (unsigned)Hs);
  const int C4 = C >> 2, c4 = ct * UPB_CT + (tid & (UPB_CT - 1));
  const int j0 = jt * UPB_J;
  // destination rows touching source row i (same window and +-1 guard as upsample_bwd4w; host-checked <= 8)
  const int ulo = max(0, (int)ceilf((float)(i - 1) / sh) - 1), uhi = min(up_h - 1, (int)floorf((float)(i + 1) / sh) + 1);
  float wy[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int u = ulo + k, yy = u + pt;
    wy[k] = (u <= uhi && yy >= 0 && yy < Hp) ? up_weight(sh, u, Hs, i) : 0.f;
  }
  // destination columns touching source columns [j0, j0 + UPB_J) (host-checked <= UPB_VMAX)
  const int jlast = min(Ws - 1, j0 + UPB_J - 1);
  const int vlo = max(0, (int)ceilf((float)(j0 - 1) / sw) - 1), vhi = min(up_w - 1, (int)floorf((float)(jlast + 1) / sw) + 1);
  const int nv = vhi - vlo + 1;
  if (tid < nv) {
    const int v = vlo + tid, xx = v + pl;
    int a0, a1;
    float l;
    lin_idx(sw, v, Ws, a0, a1, l);
    const bool ok = xx >= 0 && xx < Wp;
    tab_i0[tid] = ok ? a0 : -1;
    tab_i1[tid] = ok ? a1 : -1;
    tab_l[tid] = l;
  }
  // phase 1: one (column, channel vector) item per thread and trip
  const bool cok = c4 < C4;
  const size_t rowpix = (size_t)Wp * C4;
  const float4* base = reinterpret_cast<const float4*>(dup) + ((size_t)n * Hp + (ulo + pt)) * rowpix + c4;
  for (int it = tid >> 4; it < nv; it += 256 / UPB_CT) {
    const int xx = vlo + it + pl;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (cok && xx >= 0 && xx < Wp) {
      const float4* p = base + (size_t)xx * C4;
      float4 g[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = wy[k] != 0.f ? p[(size_t)k * rowpix] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a.x = __builtin_fmaf(wy[k], g[k].x, a.x); a.y = __builtin_fmaf(wy[k], g[k].y, a.y);
        a.z = __builtin_fmaf(wy[k], g[k].z, a.z); a.w = __builtin_fmaf(wy[k], g[k].w, a.w);
      }
    }
    t[it][tid & (UPB_CT - 1)] = a;
  }
  __syncthreads();
  // phase 2: one (source column, channel vector) per thread
  const int j = j0 + (tid >> 4);
  if (j > jlast || !cok) return;
  const int vjlo = max(vlo, (int)ceilf((float)(j - 1) / sw) - 1), vjhi = min(vhi, (int)floorf((float)(j + 1) / sw) + 1);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int v = vjlo; v <= vjhi; ++v) {
    const int q = v - vlo;
    const float l = tab_l[q];
    const float w = (tab_i0[q] == j ? 1.f - l : 0.f) + (tab_i1[q] == j ? l : 0.f);
    const float4 g = t[q][tid & (UPB_CT - 1)];
    a.x = __builtin_fmaf(w, g.x, a.x); a.y = __builtin_fmaf(w, g.y, a.y);
    a.z = __builtin_fmaf(w, g.z, a.z); a.w = __builtin_fmaf(w, g.w, a.w);
  }
  float4* o = reinterpret_cast<float4*>(dx) + (((size_t)n * Hs + i) * Ws + j) * C4 + c4;
  if (accum) {
    const float4 b = *o;
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  *o = a;
}

// NHWC gather adjoint: dx[n,i,j,c] (+)= Σ_{u,v} wy(u,i) wx(v,j) d_up[n, u+pt, v+pl, c]
__global__ void upsample_bwd_kernel(long long N, int C, int Hs, int Ws, int up_h, int up_w, int pt, int pl, int Hp,
                                    int Wp, float sh, float sw, const float* dup, float* dx, int accum) {
  const long long total = N * Hs * (long long)Ws * C;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int c = e % C;
    long long t = e / C;
    const int j = t % Ws;
    t /= Ws;
    const int i = t % Hs;
    const long long n = t / Hs;
    int ulo, uhi, vlo, vhi;
    up_range(sh, i, Hs, up_h, ulo, uhi);
    up_range(sw, j, Ws, up_w, vlo, vhi);
    float acc = 0.f;
    for (int u = ulo; u <= uhi; ++u) {
      const float wy = up_weight(sh, u, Hs, i);
      if (wy == 0.f) continue;
      const int yy = u + pt;
      if (yy < 0 || yy >= Hp) continue;
      float racc = 0.f;
      for (int v = vlo; v <= vhi; ++v) {
        const float wx = up_weight(sw, v, Ws, j);
        if (wx == 0.f) continue;
        const int xx = v + pl;
        if (xx < 0 || xx >= Wp) continue;
        racc += wx * dup[((n * Hp + yy) * (long long)Wp + xx) * C + c];
      }
      acc += wy * racc;
    }
    dx[e] = accum ? dx[e] + acc : acc;
  }
}

// fp32 NCHW bilinear (align_corners=True) forward: y[nc, u, v]
__global__ void resize_nchw_kernel(long long NC, int Hi, int Wi, int Ho, int Wo, float sh, float sw, const float* x,
                                   float* y) {
  const long long total = NC * Ho * (long long)Wo;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int v = e % Wo;
    long long t = e / Wo;
    const int u = t % Ho;
    const long long nc = t / Ho;
    int y0, y1, x0, x1;
    float ly, lx;
    lin_idx(sh, u, Hi, y0, y1, ly);
    lin_idx(sw, v, Wi, x0, x1, lx);
    const float* p = x + nc * Hi * (long long)Wi;
    const float a = p[y0 * Wi + x0], b = p[y0 * Wi + x1], c = p[y1 * Wi + x0], d = p[y1 * Wi + x1];
    y[e] = (1.f - ly) * ((1.f - lx) * a + lx * b) + ly * ((1.f - lx) * c + lx * d);
  }
}

__global__ void resize_nchw_bwd_kernel(long long NC, int Hi, int Wi, int Ho, int Wo, float sh, float sw, const float* dy,
                                       float* dx, int accum) {
  const long long total = NC * Hi * (long long)Wi;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int j = e % Wi;
    long long t = e / Wi;
    const int i = t % Hi;
    const long long nc = t / Hi;
    int ulo, uhi, vlo, vhi;
    up_range(sh, i, Hi, Ho, ulo, uhi);
    up_range(sw, j, Wi, Wo, vlo, vhi);
    const float* p = dy + nc * Ho * (long long)Wo;
    float acc = 0.f;
    for (int u = ulo; u <= uhi; ++u) {
      const float wy = up_weight(sh, u, Hi, i);
      if (wy == 0.f) continue;
      float racc = 0.f;
      for (int v = vlo; v <= vhi; ++v) {
        const float wx = up_weight(sw, v, Wi, j);
        if (wx != 0.f) racc += wx * p[u * (long long)Wo + v];
      }
      acc += wy * racc;
    }
    dx[e] = accum ? dx[e] + acc : acc;
  }
}

// ---- OutConv: logits[n,k,h,w] = b[k] + Σ_c w[k][c] · act(y)[n,h,w,c]   (layers.py:120) ----------------
constexpr int OC_MAXK = 8;

template <typename T>
__global__ void outconv_fwd_kernel(long long P, int HW, int C, int K, const T* y, const float* sc, const float* sf,
                                   int relu, const float* w, const float* b, float* out) {
  extern __shared__ float ws[];  // [K][C] then scale/shift
  for (int i = threadIdx.x; i < K * C; i += blockDim.x) ws[i] = w[i];
  float* s_sc = ws + K * C;
  float* s_sf = s_sc + C;
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    s_sc[i] = sc ? sc[i] : 1.f;
    s_sf[i] = sf ? sf[i] : 0.f;
  }
  __syncthreads();
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < P; q += (long long)gridDim.x * blockDim.x) {
    float acc[OC_MAXK];
#pragma unroll
    for (int k = 0; k < OC_MAXK; ++k) acc[k] = (k < K) ? b[k] : 0.f;
    const T* yp = y + q * C;
    for (int c = 0; c < C; ++c) {
      float a = __builtin_fmaf(to_f(yp[c]), s_sc[c], s_sf[c]);
      if (relu) a = fmaxf(a, 0.f);
#pragma unroll
      for (int k = 0; k < OC_MAXK; ++k)
        if (k < K) acc[k] += ws[k * C + c] * a;
    }
    const long long n = q / HW, hw = q % HW;
#pragma unroll
    for (int k = 0; k < OC_MAXK; ++k)
      if (k < K) out[(n * K + k) * HW + hw] = acc[k];
  }
}

// coalesced variant: G = C/8 lanes per pixel, 8 channels per lane, class sums by xor-shuffles
template <typename T, int KT>
__global__ void outconv_fwd_vec_kernel(long long P, int HW, int C, int G, const T* y, const float* sc, const float* sf,
                                       int relu, const float* w, const float* b, float* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int sub = lane % G, ppw = 64 / G;
  const int c0 = sub * 8;
  float s[8], f[8], wk[KT][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] = sc ? sc[c0 + j] : 1.f;
    f[j] = sf ? sf[c0 + j] : 0.f;
#pragma unroll
    for (int k = 0; k < KT; ++k) wk[k][j] = w[k * C + c0 + j];
  }
  const long long stride = (long long)gridDim.x * nw * ppw;
  // OC_U pixels per trip, all their loads issued first (round 6: one memory round trip per trip instead of per
  // pixel; 2.5 TB/s before); each pixel's sum is unchanged
  constexpr int OC_U = 4;
  for (long long q = ((long long)blockIdx.x * nw + wave) * ppw + lane / G; q < P; q += OC_U * stride) {
    float a[OC_U][8];
#pragma unroll
    for (int u = 0; u < OC_U; ++u) {
      const long long qq = q + u * stride < P ? q + u * stride : q;
      if constexpr (sizeof(T) == 2) {
        load_vec<T>(y + qq * C + c0, a[u]);
      } else {
        load_vec<float>((const float*)y + qq * C + c0, a[u]);
        load_vec<float>((const float*)y + qq * C + c0 + 4, a[u] + 4);
      }
    }
#pragma unroll
    for (int u = 0; u < OC_U; ++u) {
      const long long qu = q + u * stride;
      float acc[KT];
#pragma unroll
      for (int k = 0; k < KT; ++k) acc[k] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = __builtin_fmaf(a[u][j], s[j], f[j]);
        if (relu) v = fmaxf(v, 0.f);
#pragma unroll
        for (int k = 0; k < KT; ++k) acc[k] += wk[k][j] * v;
      }
#pragma unroll
      for (int k = 0; k < KT; ++k)
        for (int o = G >> 1; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o, 64);
      if (sub == 0 && qu < P) {
        const long long n = qu / HW, hw = qu % HW;
#pragma unroll
        for (int k = 0; k < KT; ++k) out[(n * KT + k) * HW + hw] = acc[k] + b[k];
      }
    }
  }
}

// channel lanes x pixel rows: da[p][c] (+)= Σ_k w[k][c] dl[k][p]; partial dW[k][c], db[k]
template <typename T>
__global__ void outconv_bwd_kernel(long long P, int HW, int C, int CL, int K, const T* y, const float* sc,
                                   const float* sf, int relu, const float* w, const float* dl, float* da, int accum,
                                   float* part, int rows) {
  __shared__ float sh[256];
  const int tid = threadIdx.x;
  const int cx = tid % CL, py = tid / CL, R = blockDim.x / CL;
  const int c = blockIdx.x * CL + cx;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.y * per, p1 = min(P, p0 + per);
  float dw[OC_MAXK], db[OC_MAXK], wk[OC_MAXK];
#pragma unroll
  for (int k = 0; k < OC_MAXK; ++k) { dw[k] = 0.f; db[k] = 0.f; wk[k] = (k < K && c < C) ? w[k * C + c] : 0.f; }
  const float s = (c < C && sc) ? sc[c] : 1.f, f = (c < C && sf) ? sf[c] : 0.f;
  for (long long q = p0 + py; q < p1; q += R) {
    const long long n = q / HW, hw = q % HW;
    float g = 0.f;
    float dlk[OC_MAXK];
#pragma unroll
    for (int k = 0; k < OC_MAXK; ++k) {
      dlk[k] = (k < K) ? dl[(n * K + k) * HW + hw] : 0.f;
      g += wk[k] * dlk[k];
      db[k] += dlk[k];
    }
    if (c < C) {
      float a = __builtin_fmaf(to_f(y[q * C + c]), s, f);
      if (relu) a = fmaxf(a, 0.f);
#pragma unroll
      for (int k = 0; k < OC_MAXK; ++k) dw[k] += dlk[k] * a;
      float* o = da + q * C + c;
      *o = accum ? *o + g : g;
    }
  }
  // reduce over the R pixel rows sharing a channel lane
  const int F = K + 1;
  for (int k = 0; k < F; ++k) {
    float v = 0.f;
#pragma unroll
    for (int kk = 0; kk < OC_MAXK; ++kk) if (kk == k) v = dw[kk];
    if (k == K) v = 0.f;
    sh[tid] = v;
    __syncthreads();
    if (py == 0 && c < C && k < K) {
      float a = 0.f;
      for (int r = 0; r < R; ++r) a += sh[r * CL + cx];
      part[((size_t)blockIdx.y * (K + 1) + k) * C + c] = a;
    }
    __syncthreads();
  }
  // db: only channel-block 0 writes it (every lane saw all pixels of its rows)
  if (blockIdx.x == 0) {
    for (int k = 0; k < K; ++k) {
      float v = 0.f;
#pragma unroll
      for (int kk = 0; kk < OC_MAXK; ++kk) if (kk == k) v = db[kk];
      sh[tid] = (cx == 0) ? v : 0.f;
      __syncthreads();
      if (tid == 0) {
        float a = 0.f;
        for (int r = 0; r < R; ++r) a += sh[r * CL];
        part[((size_t)blockIdx.y * (K + 1) + K) * C + k] = a;  // db stored in row K, column k
      }
      __syncthreads();
    }
  }
}

// vectorised form (bf16, C % 8 == 0, G = C/8 a power of two <= 256): a thread owns 8 channels of one
// pixel per iteration — one 16-byte y load, two 16-byte da stores (or read-modify-writes); the K class
// gradients of the pixel are loaded once per thread.  Same partial-sum table as outconv_bwd_kernel:
// part[block][k][c] = Σ dl·a, part[block][K][k] = Σ dl (db).
template <typename T, int KK>
__global__ __launch_bounds__(256) void outconv_bwd_vec_kernel(long long P, int HW, int C, int G, const T* y,
                                                              const float* sc, const float* sf, int relu,
                                                              const float* w, const float* dl, float* da, int accum,
                                                              float* part) {
  constexpr int F = KK * 8 + KK;  // per-thread partials: dw[k][8], db[k]
  __shared__ float sh[256 * F];
  const int tid = threadIdx.x, v = tid % G, py = tid / G, R = 256 / G;
  const int c0 = v * 8;
  float s8[8], f8[8], wk[KK][8], dw[KK][8], db[KK];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s8[j] = sc ? sc[c0 + j] : 1.f;
    f8[j] = sf ? sf[c0 + j] : 0.f;
#pragma unroll
    for (int k = 0; k < KK; ++k) { wk[k][j] = w[k * C + c0 + j]; dw[k][j] = 0.f; }
  }
#pragma unroll
  for (int k = 0; k < KK; ++k) db[k] = 0.f;
  const float lo = relu ? 0.f : -INFINITY;
  const long long per = (P + gridDim.x - 1) / gridDim.x;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  for (long long q = p0 + py; q < p1; q += R) {
    const long long n = q / HW, hw = q % HW;
    float dlk[KK];
#pragma unroll
    for (int k = 0; k < KK; ++k) { dlk[k] = dl[(n * KK + k) * HW + hw]; db[k] += dlk[k]; }
    float a[8];
    load_vec<T>(y + q * C + c0, a);
    float g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = fmaxf(__builtin_fmaf(a[j], s8[j], f8[j]), lo);
      g[j] = 0.f;
#pragma unroll
      for (int k = 0; k < KK; ++k) { g[j] += wk[k][j] * dlk[k]; dw[k][j] += dlk[k] * a[j]; }
    }
    float4* o = reinterpret_cast<float4*>(da + q * C + c0);
    float4 g0 = make_float4(g[0], g[1], g[2], g[3]), g1 = make_float4(g[4], g[5], g[6], g[7]);
    if (accum) {
      const float4 a0 = o[0], a1 = o[1];
      g0.x += a0.x; g0.y += a0.y; g0.z += a0.z; g0.w += a0.w;
      g1.x += a1.x; g1.y += a1.y; g1.z += a1.z; g1.w += a1.w;
    }
    o[0] = g0;
    o[1] = g1;
  }
#pragma unroll
  for (int k = 0; k < KK; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[tid * F + k * 8 + j] = dw[k][j];
    sh[tid * F + KK * 8 + k] = db[k];
  }
  __syncthreads();
  // fixed-order sums over the R pixel rows: thread e < C*KK owns dw[k][c]; e < KK (extra) owns db[k]
  for (int e = tid; e < C * KK + KK; e += 256) {
    float acc = 0.f;
    if (e < C * KK) {
      const int k = e / C, c = e % C, vv = c / 8, j = c % 8;
      for (int r = 0; r < R; ++r) acc += sh[(r * G + vv) * F + k * 8 + j];
      part[((size_t)blockIdx.x * (KK + 1) + k) * C + c] = acc;
    } else {
      const int k = e - C * KK;
      for (int r = 0; r < R; ++r) acc += sh[(r * G) * F + KK * 8 + k];  // channel-vector 0 of each row
      part[((size_t)blockIdx.x * (KK + 1) + KK) * C + k] = acc;
    }
  }
}

// OutConv backward fused with the BatchNorm backward of its input activation (the last DoubleConv's output,
// whose only consumer is OutConv: unet.py:92 / :203).  The activation gradient g[px][c] = Σ_k W[k][c]·dl[k][px]
// is never stored: this pass accumulates OutConv's dW / db partials (as outconv_bwd_vec_kernel) and the
// BatchNorm-backward sums Σ g_m, Σ g_m·x̂ (g_m: g where the ReLU passed, as bn_bwd_reduce_vec_kernel) from
// one read of y and the 2-class logit gradient; bn_bwd_apply_oc_kernel recomputes g the same way.  Removes the
// fp32 [N,H,W,C] gradient write and its two reads (3 x 268 MB at 4 x 512^2 x 64).
template <typename T, int KK>
__global__ __launch_bounds__(256) void outconv_bwd_bn_kernel(long long P, int HW, int C, int G, const T* y,
                                                             const float* sc, const float* sf, int relu,
                                                             const float* w, const float* dl, const float* mean,
                                                             const float* invstd, float* part, float* bpart, int rows) {
  constexpr int F = KK * 8 + KK;  // per-thread partials: dw[k][8], db[k]
  __shared__ float sh[256 * F];
  const int tid = threadIdx.x, v = tid % G, py = tid / G, R = 256 / G;
  const int c0 = v * 8;
  float s8[8], f8[8], mu[8], is[8], wk[KK][8], dw[KK][8], db[KK], sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s8[j] = sc[c0 + j];
    f8[j] = sf[c0 + j];
    mu[j] = mean[c0 + j];
    is[j] = invstd[c0 + j];
    sg[j] = 0.f;
    sgx[j] = 0.f;
#pragma unroll
    for (int k = 0; k < KK; ++k) { wk[k][j] = w[k * C + c0 + j]; dw[k][j] = 0.f; }
  }
#pragma unroll
  for (int k = 0; k < KK; ++k) db[k] = 0.f;
  const float lo = relu ? 0.f : -INFINITY;
  const long long per = (P + gridDim.x - 1) / gridDim.x;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  // OB_U pixels per trip, loads first (round 6); the sums still run over q, q + R, ... in order (bit-identical)
  constexpr int OB_U = 4;
  for (long long q = p0 + py; q < p1; q += OB_U * R) {
    float dlu[OB_U][KK], yu[OB_U][8];
#pragma unroll
    for (int u = 0; u < OB_U; ++u) {
      const long long qq = q + u * R < p1 ? q + u * R : q;
      const long long n = qq / HW, hw = qq % HW;
#pragma unroll
      for (int k = 0; k < KK; ++k) dlu[u][k] = dl[(n * KK + k) * HW + hw];
      load_vec<T>(y + qq * C + c0, yu[u]);
      if constexpr (sizeof(T) == 4) load_vec<T>(y + qq * C + c0 + 4, yu[u] + 4);
    }
#pragma unroll
    for (int u = 0; u < OB_U; ++u) {
      if (q + u * R >= p1) break;
      const float* dlk = dlu[u];
      const float* yv = yu[u];
#pragma unroll
      for (int k = 0; k < KK; ++k) db[k] += dlk[k];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float pre = __builtin_fmaf(yv[j], s8[j], f8[j]);
        const float a = fmaxf(pre, lo);
        float g = 0.f;
#pragma unroll
        for (int k = 0; k < KK; ++k) { g += wk[k][j] * dlk[k]; dw[k][j] += dlk[k] * a; }
        const float gm = (relu && !(pre > 0.f)) ? 0.f : g;
        sg[j] += gm;
        sgx[j] += gm * (yv[j] - mu[j]) * is[j];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KK; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[tid * F + k * 8 + j] = dw[k][j];
    sh[tid * F + KK * 8 + k] = db[k];
  }
  __syncthreads();
  for (int e = tid; e < C * KK + KK; e += 256) {
    float acc = 0.f;
    if (e < C * KK) {
      const int k = e / C, c = e % C, vv = c / 8, j = c % 8;
      for (int r = 0; r < R; ++r) acc += sh[(r * G + vv) * F + k * 8 + j];
      part[((size_t)blockIdx.x * (KK + 1) + k) * C + c] = acc;
    } else {
      const int k = e - C * KK;
      for (int r = 0; r < R; ++r) acc += sh[(r * G) * F + KK * 8 + k];
      part[((size_t)blockIdx.x * (KK + 1) + KK) * C + k] = acc;
    }
  }
  __syncthreads();
  // BatchNorm-backward partial sums of the block: [2][rows][C] (unet_bn_bwd_finalize's layout)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[tid] = sg[j];
    sh[256 + tid] = sgx[j];
    __syncthreads();
    if (tid < G) {
      float a = 0.f, b = 0.f;
      for (int r = 0; r < R; ++r) { a += sh[r * G + tid]; b += sh[256 + r * G + tid]; }
      bpart[(size_t)blockIdx.x * C + tid * 8 + j] = a;
      bpart[((size_t)rows + blockIdx.x) * C + tid * 8 + j] = b;
    }
    __syncthreads();
  }
}

// dy = A·g_m + B·y + C with g recomputed from the logit gradient (bn_bwd_apply_vec_kernel's formula)
template <typename T, int KK>
__global__ __launch_bounds__(256) void bn_bwd_apply_oc_kernel(long long P, int HW, int C, const T* y, const float* scale,
                                                              const float* shift, int relu, const float* w,
                                                              const float* dl, const float* coef, T* dy) {
  const int CV = C / 8;
  const long long total = P * CV;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const int cv = (int)(e % CV);  // fixed: the stride is a multiple of CV (power of two <= 256)
  float sc[8], sf[8], A[8], B[8], Cc[8], wk[KK][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cv * 8 + j;
    sc[j] = scale[c]; sf[j] = shift[c]; A[j] = coef[c]; B[j] = coef[C + c]; Cc[j] = coef[2 * C + c];
#pragma unroll
    for (int k = 0; k < KK; ++k) wk[k][j] = w[k * C + c];
  }
  const int cvs = __builtin_ctz(CV);
  // AO_U elements per trip, every load before the stores (dy may alias the loads as far as the compiler knows,
  // which serialised one memory round trip per pixel; round 6); elementwise.  The unroll moved the compiler's
  // fma contraction of o = A g + B y + C (last bits of dy); the order is now explicit, as in bn.hip
  constexpr int AO_U = 4;
  for (; e < total; e += AO_U * stride) {
    float dlu[AO_U][KK], yu[AO_U][8];
    long long pu[AO_U];
#pragma unroll
    for (int u = 0; u < AO_U; ++u) {
      const long long p = (e + u * stride < total ? e + u * stride : e) >> cvs;
      pu[u] = p;
      const unsigned n = (unsigned)p / (unsigned)HW, hw = (unsigned)p - n * (unsigned)HW;
#pragma unroll
      for (int k = 0; k < KK; ++k) dlu[u][k] = dl[((size_t)n * KK + k) * HW + hw];
      load_vec<T>(y + p * C + cv * 8, yu[u]);
      if constexpr (sizeof(T) == 4) load_vec<T>(y + p * C + cv * 8 + 4, yu[u] + 4);
    }
#pragma unroll
    for (int u = 0; u < AO_U; ++u) {
      if (e + u * stride >= total) break;
      const long long p = pu[u];
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g = 0.f;
#pragma unroll
        for (int k = 0; k < KK; ++k) g += wk[k][j] * dlu[u][k];
        const float gj = (relu && !(__builtin_fmaf(yu[u][j], sc[j], sf[j]) > 0.f)) ? 0.f : g;
        o[j] = f32_rounded(__builtin_fmaf(A[j], gj, __builtin_fmaf(B[j], yu[u][j], Cc[j])));   // bn.hip's rounding
      }
      store_vec<T>(dy + p * C + cv * 8, o);
      if constexpr (sizeof(T) == 4) store_vec<T>(dy + p * C + cv * 8 + 4, o + 4);
    }
  }
}

// one block per output element; fixed-order fp64 block reduction over the partial rows
__global__ void outconv_bwd_finalize_kernel(const float* part, int rows, int C, int K, float* dw, float* db, int accum) {
  __shared__ double sh[4];
  const int e = blockIdx.x;
  const bool is_w = e < K * C;
  const int k = is_w ? e / C : K;
  const int c = is_w ? e % C : e - K * C;
  double s = 0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) s += part[((size_t)r * (K + 1) + k) * C + c];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (float)(sh[0] + sh[1] + sh[2] + sh[3]);
    float* o = is_w ? dw + e : db + c;
    *o = accum ? *o + v : v;
  }
}

// ---- layout ---------------------------------------------------------------------------------------
template <typename T>
__global__ void nchw_to_nhwc_kernel(long long N, int C, int H, int W, const float* x, T* y) {
  const long long total = N * C * (long long)H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int c = e % C;
    const long long p = e / C;
    const long long hw = p % ((long long)H * W), n = p / ((long long)H * W);
    y[e] = from_f<T>(x[(n * C + c) * (long long)H * W + hw]);
  }
}
// ---- materialise a virtual source (max-pool / bilinear-up + pad / BN-ReLU / gate) as a plain NHWC
// tensor.  The conv and wgrad loaders then read it as a PLAIN source: their per-element transform
// (VALU beside the MFMAs) costs more than one streaming pass over the result.
template <typename T>
__global__ void materialize_kernel(const unet_src s, long long N, int H, int W, T* out) {
  constexpr int VEC = Vec<T>::N;
  const int CV = (s.C + VEC - 1) / VEC;
  const long long total = N * H * (long long)W * CV;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int cv = (int)(e % CV);
    long long t = e / CV;
    const int x = (int)(t % W);
    t /= W;
    const int y = (int)(t % H);
    const long long n = t / H;
    float v[VEC];
    src_gather<T>(&s, 1, s.C, H, W, n, y, x, cv * VEC, v);
    T* o = out + ((n * H + y) * (long long)W + x) * s.C + cv * VEC;
    if ((s.C % VEC) == 0) {
      store_vec<T>(o, v);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (cv * VEC + j < s.C) o[j] = from_f<T>(v[j]);
    }
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(long long N, int C, int H, int W, const T* x, const float* sc, const float* sf,
                                    int relu, float* y) {
  const long long total = N * C * (long long)H * W;
  const long long HW = (long long)H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long hw = e % HW;
    const long long t = e / HW;
    const int c = t % C;
    const long long n = t / C;
    float v = to_f(x[(n * HW + hw) * C + c]);
    if (sc) v = __builtin_fmaf(v, sc[c], sf[c]);
    if (relu) v = fmaxf(v, 0.f);
    y[e] = v;
  }
}
// x * sigmoid(psi) materialised as NCHW fp32 (standalone AttentionGate output, layers.py:192)
template <typename T>
__global__ void gated_to_nchw_kernel(long long N, int C, int H, int W, const T* x, const float* sc, const float* sf,
                                     int relu, const float* p, const float* ab, float* y) {
  const long long total = N * C * (long long)H * W;
  const long long HW = (long long)H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long hw = e % HW;
    const long long t = e / HW;
    const int c = t % C;
    const long long n = t / C;
    float v = __builtin_fmaf(to_f(x[(n * HW + hw) * C + c]), sc[c], sf[c]);
    if (relu) v = fmaxf(v, 0.f);
    y[e] = v * sigmoidf_(p[n * HW + hw] * ab[0] + ab[1]);
  }
}
__global__ void fill_kernel(float* x, long long n, float v) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) x[e] = v;
}

// ConvTranspose2d(k=2, s=2) backward prep: space-to-depth of the output gradient into the gradient of
// the equivalent 1x1 conv (channel (2a+b)*Ct + c), plus per-block bias partial sums.
// Block: CLN channel lanes x PL pixel lanes; one pixel range per block (fixed order -> deterministic).
constexpr int CT_MAXCH = 4;  // channel chunks of 256 per thread (Ct <= 1024)
template <typename T>
__global__ __launch_bounds__(256) void convt_bwd_prep_kernel(long long N, int h, int w, int Ct, int Hp, int Wp, int pt,
                                                             int pl, const float* d_up, T* out, float* partial,
                                                             int rows) {
  __shared__ float red[256];
  const int tid = threadIdx.x;
  const int CLN = Ct < 256 ? Ct : 256, PL = 256 / CLN;
  const int cl = tid % CLN, pq = tid / CLN;
  const long long P = N * h * w;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float bs[CT_MAXCH];
#pragma unroll
  for (int k = 0; k < CT_MAXCH; ++k) bs[k] = 0.f;
  if (pq < PL) {
    for (long long p = p0 + pq; p < p1; p += PL) {
      const int x = p % w;
      const long long t = p / w;
      const int y = t % h;
      const long long n = t / h;
#pragma unroll
      for (int k = 0; k < CT_MAXCH; ++k) {
        const int c = cl + k * CLN;
        if (c < Ct) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const long long src = ((n * Hp + pt + 2 * y + (q >> 1)) * (long long)Wp + pl + 2 * x + (q & 1)) * Ct + c;
            const float v = d_up[src];
            out[p * 4 * Ct + q * Ct + c] = from_f<T>(v);
            bs[k] += v;
          }
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < CT_MAXCH; ++k) {
    if (k * CLN >= Ct) break;
    red[tid] = (pq < PL) ? bs[k] : 0.f;
    __syncthreads();
    if (tid < CLN && cl + k * CLN < Ct) {
      float a = 0.f;
      for (int q = 0; q < PL; ++q) a += red[q * CLN + tid];
      partial[(size_t)blockIdx.x * Ct + cl + k * CLN] = a;
    }
    __syncthreads();
  }
}

// block cap of a grid-stride launch (env override: A/B of the per-thread item count)
static inline long long block_cap(const char* env, long long dflt) {
  const char* e = getenv(env);
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? v : dflt;
}
static inline int grid_for(long long total, long long cap = 8192) {
  long long b = (total + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}
static inline int chan_lanes_m(int C) {
  int cl = 1;
  while (cl < C && cl < 64) cl <<= 1;
  return cl;
}
static inline int oc_rows(long long P) {
  long long r = (P + 1023) / 1024;
  if (r > 1024) r = 1024;
  if (r < 1) r = 1;
  return (int)r;
}

// fast form (C % VEC == 0): e = pixel * CV + cv with cv fastest, so stores are coalesced and, since
// the grid stride is a multiple of CV (a power of two <= 256 here), every thread keeps one channel
// vector: its BN scale/shift are loaded once (make_view) and each pixel is one item_issue/finish
struct MatDesc {
  int nsrc;
  unet_src src[2];
  int Cin;
};

// I: the element index type — unsigned (32-bit division: ~10 VALU instead of a ~100-instruction 64-bit
// division sequence, of which there are four per element) whenever N*H*W*CV < 2^31 (host-chosen)
template <typename T, int RAW, typename I = unsigned>
__global__ void materialize_fast_kernel(const MatDesc d, long long N, int H, int W, T* out) {
  constexpr int VEC = Vec<T>::N;
  const int C = d.src[0].C;
  const int CV = C / VEC;
  const int cvs = __builtin_ctz(CV);   // CV is a power of two (host-checked)
  const I total = (I)(N * H * (long long)W * CV);
  const I stride = (I)gridDim.x * blockDim.x;
  I e = (I)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(e & (CV - 1));
  SrcView sv;
  float sc[VEC], sf[VEC];
  make_view<T>(d, cv * VEC, sv, sc, sf);
  for (; e < total; e += stride) {
    const I px = e >> cvs;
    const I t = px / (I)W;
    const int x = (int)(px - t * (I)W);
    const I t2 = t / (I)H;
    const int y = (int)(t - t2 * (I)H);
    const int n = (int)t2;
    Item<RAW> it;
    item_issue<T, RAW>(sv, H, W, n, y, x, 1, it);
    float v[VEC];
    item_finish<T, RAW>(d, sv, sc, sf, n, y, x, cv * VEC, it, v);
    store_vec<T>(out + (size_t)px * C + cv * VEC, v);
  }
}

// The Up block's decoder input (layers.py:98-102: bilinear x2 upsample, align_corners=True, of relu(BN(x1)), then
// F.pad to x2's size) as LDS tiles (round 5).  The per-pixel form above gathers the 4 bilinear taps of every output
// vector from L2 and runs the BN affine on each (4 x the reads and the affine work of the source it needs); here a
// block owns MUP_TJ output rows x MUP_TX output columns x MUP_CT channel vectors, stages the source rows / columns
// they touch once (<= MUP_TJ/2+2 x MUP_TX/2+2 for scales <= 1/2, host-checked) as fp32 activations in LDS, and
// blends each output from there — with the same tap indices, weights and fma order as item_issue / item_finish
// (mode 4), so the map is bit-identical to the per-pixel form and to the convs' virtual UP_ACT sources.
constexpr int MUP_TJ = 8, MUP_TX = 32, MUP_SJ = MUP_TJ / 2 + 2, MUP_SX = MUP_TX / 2 + 2, MUP_CT = 8;
template <typename T>
__global__ __launch_bounds__(256) void materialize_up_tile_kernel(const unet_src s, int H, int W, T* out) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  __shared__ float4 tile[MUP_SJ * MUP_SX * MUP_CT * 2];   // 8 fp32 activations (2 float4) per source vector
  const int C = s.C, CV = C >> 3;
  const int CT = CV < MUP_CT ? CV : MUP_CT;               // a power of two: a thread keeps one channel vector
  const int tid = threadIdx.x, cv = tid & (CT - 1);
  const int tiles_h = (H + MUP_TJ - 1) / MUP_TJ;
  const int n = (int)blockIdx.y / tiles_h, oy0 = ((int)blockIdx.y - n * tiles_h) * MUP_TJ;
  const int ox0 = (int)blockIdx.x * MUP_TX;
  const int c = ((int)blockIdx.z * CT + cv) * 8;          // this thread's first channel
  // the up-region rows / columns the tile covers and the source span they read
  int ua = oy0 - s.pad_t, ub = oy0 + MUP_TJ - 1 - s.pad_t, va = ox0 - s.pad_l, vb = ox0 + MUP_TX - 1 - s.pad_l;
  ua = ua < 0 ? 0 : ua; ub = ub > s.up_h - 1 ? s.up_h - 1 : ub;
  va = va < 0 ? 0 : va; vb = vb > s.up_w - 1 ? s.up_w - 1 : vb;
  int sy0 = 0, sx0 = 0, ny = 0, nx = 0;
  if (ua <= ub && va <= vb) {
    int i0, i1;
    float l;
    lin_idx(s.sh, ua, s.H, i0, i1, l);
    sy0 = i0;
    lin_idx(s.sh, ub, s.H, i0, i1, l);
    ny = i1 - sy0 + 1;
    lin_idx(s.sw, va, s.W, i0, i1, l);
    sx0 = i0;
    lin_idx(s.sw, vb, s.W, i0, i1, l);
    nx = i1 - sx0 + 1;
    ny = ny < MUP_SJ ? ny : MUP_SJ;                        // (host-checked; a clamp keeps LDS in bounds regardless)
    nx = nx < MUP_SX ? nx : MUP_SX;
  }
  float sc[8], sf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = s.scale[c + j]; sf[j] = s.shift[c + j]; }
  // phase 1: the source span -> LDS, BN affine (+ ReLU) in fp32 as item_finish applies it per tap
  const T* src = (const T*)s.data;
  for (int i = tid; i < ny * nx * CT; i += 256) {
    const int px = i / CT, sxr = px % nx, syr = px / nx;
    const unsigned pix = ((unsigned)n * s.H + (unsigned)(sy0 + syr)) * (unsigned)s.W + (unsigned)(sx0 + sxr);
    float t[8];
    unpack16<T>(*reinterpret_cast<const uint4*>(src + (size_t)pix * C + c), t);
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      f2 r = __builtin_elementwise_fma(f2{t[j], t[j + 1]}, f2{sc[j], sc[j + 1]}, f2{sf[j], sf[j + 1]});
      if (s.relu) r = f2{fmaxf(r[0], 0.f), fmaxf(r[1], 0.f)};
      a[j] = r[0];
      a[j + 1] = r[1];
    }
    float4* d4 = tile + ((syr * MUP_SX + sxr) * MUP_CT + cv) * 2;
    d4[0] = make_float4(a[0], a[1], a[2], a[3]);
    d4[1] = make_float4(a[4], a[5], a[6], a[7]);
  }
  __syncthreads();
  // phase 2: the outputs (zero outside the up region: F.pad)
  for (int i = tid; i < MUP_TJ * MUP_TX * CT; i += 256) {
    const int px = i / CT, oxr = px % MUP_TX, oyr = px / MUP_TX;
    const int oy = oy0 + oyr, ox = ox0 + oxr;
    if (oy >= H || ox >= W) continue;
    const int uy = oy - s.pad_t, ux = ox - s.pad_l;
    float v[8];
    if (uy >= 0 && uy < s.up_h && ux >= 0 && ux < s.up_w) {
      int y0, y1, x0, x1;
      float ly, lx;
      lin_idx(s.sh, uy, s.H, y0, y1, ly);
      lin_idx(s.sw, ux, s.W, x0, x1, lx);
      const float hy0 = 1.f - ly, wx0 = 1.f - lx;
      const float w0s = hy0 * wx0, w1s = hy0 * lx, w2s = ly * wx0, w3s = ly * lx;
      const f2 w0 = {w0s, w0s}, w1 = {w1s, w1s}, w2 = {w2s, w2s}, w3 = {w3s, w3s};
      const float4* r0 = tile + (((y0 - sy0) * MUP_SX + (x0 - sx0)) * MUP_CT + cv) * 2;
      const float4* r1 = tile + (((y0 - sy0) * MUP_SX + (x1 - sx0)) * MUP_CT + cv) * 2;
      const float4* r2 = tile + (((y1 - sy0) * MUP_SX + (x0 - sx0)) * MUP_CT + cv) * 2;
      const float4* r3 = tile + (((y1 - sy0) * MUP_SX + (x1 - sx0)) * MUP_CT + cv) * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 a0 = r0[h], a1 = r1[h], a2 = r2[h], a3 = r3[h];
        const f2 p0 = __builtin_elementwise_fma(w3, f2{a3.x, a3.y}, __builtin_elementwise_fma(w2, f2{a2.x, a2.y},
                        __builtin_elementwise_fma(w1, f2{a1.x, a1.y}, w0 * f2{a0.x, a0.y})));
        const f2 p1 = __builtin_elementwise_fma(w3, f2{a3.z, a3.w}, __builtin_elementwise_fma(w2, f2{a2.z, a2.w},
                        __builtin_elementwise_fma(w1, f2{a1.z, a1.w}, w0 * f2{a0.z, a0.w})));
        v[4 * h] = p0[0]; v[4 * h + 1] = p0[1]; v[4 * h + 2] = p1[0]; v[4 * h + 3] = p1[1];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
    store_vec<T>(out + ((size_t)((unsigned)n * H + oy) * W + ox) * C + c, v);
  }
}

// MaxPool2d(2) of relu?(scale*y + shift) with argmax codes; one thread per pooled channel vector
// (I as materialize_fast_kernel)
template <typename T, typename I = unsigned>
__global__ void materialize_pool_kernel(const unet_src s, long long N, int H, int W, T* out, uint8_t* code) {
  constexpr int VEC = Vec<T>::N;
  const int C = s.C, CV = C / VEC;
  const int cvs = __builtin_ctz(CV);
  const I total = (I)(N * H * (long long)W * CV);
  const I stride = (I)gridDim.x * blockDim.x;
  I e = (I)blockIdx.x * blockDim.x + threadIdx.x;
  const int cv = (int)(e & (CV - 1));
  float sc[VEC], sf[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) { sc[j] = s.scale[cv * VEC + j]; sf[j] = s.shift[cv * VEC + j]; }
  const float lo = s.relu ? 0.f : -INFINITY;
  for (; e < total; e += stride) {
    const I px = e >> cvs;
    const I t = px / (I)W;
    const int x = (int)(px - t * (I)W);
    const I t2 = t / (I)H;
    const int y = (int)(t - t2 * (I)H);
    const long long n = (long long)t2;
    float best[VEC];
    int arg[VEC];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v[VEC];
      load_vec<T>((const T*)s.data + (((n * s.H + 2 * y + (q >> 1)) * (long long)s.W + 2 * x + (q & 1)) * C + cv * VEC), v);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float a = fmaxf(__builtin_fmaf(v[j], sc[j], sf[j]), lo);
        if (q == 0 || a > best[j] || a != a) { best[j] = a; arg[j] = q; }
      }
    }
    store_vec<T>(out + (size_t)px * C + cv * VEC, best);
    unsigned lo4 = 0, hi4 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) lo4 |= (unsigned)arg[j] << (8 * j);
    if constexpr (VEC == 8) {
#pragma unroll
      for (int j = 0; j < 4; ++j) hi4 |= (unsigned)arg[4 + j] << (8 * j);
      *reinterpret_cast<uint2*>(code + (size_t)px * C + cv * VEC) = make_uint2(lo4, hi4);
    } else {
      *reinterpret_cast<unsigned*>(code + (size_t)px * C + cv * VEC) = lo4;
    }
  }
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_upsample_bwd(long long N, int C, int Hs, int Ws, int up_h, int up_w, int pad_t, int pad_l, int Hp, int Wp,
                      float sh, float sw, const float* d_up, float* dx, int accum, void* stream) {
  const long long total = N * Hs * (long long)Ws * C;
  // widest destination window of upsample_bwd4w: floor(2/scale) + 3 taps (scale 0: the whole map)
  auto span = [](float sc, int up) { return sc > 0.f ? (int)floorf(2.f / sc) + 3 : up + 8; };
  if (C % 4 == 0 && span(sh, up_h) <= 8 && span(sw, up_w) <= 8) {
    // the tiled kernel: its destination-column window for UPB_J source columns must fit the LDS table
    const int vspan = (int)floorf((float)(UPB_J + 1) / sw) + 4;
    const char* e = getenv("UNET_UPB_TILE");
    const long long ntj = cdiv(Ws, UPB_J), ntc = cdiv(C / 4, UPB_CT), nblk = N * Hs * ntj * ntc;
    if (!(e && atoi(e) == 0) && vspan <= UPB_VMAX && nblk < (1LL << 31)) {
      hipLaunchKernelGGL(upsample_bwd_tile_kernel, dim3((unsigned)nblk), dim3(256), 0, (hipStream_t)stream, (int)N, C, Hs,
                         Ws, up_h, up_w, pad_t, pad_l, Hp, Wp, sh, sw, d_up, dx, accum, (int)ntj, (int)ntc);
      return check_launch("upsample_bwd");
    }
    if (total / 4 < (1LL << 31))
      hipLaunchKernelGGL(upsample_bwd4w_kernel<unsigned>, dim3(grid_for(total / 4, block_cap("UNET_UPB_BLOCKS", 8192))), dim3(256), 0, (hipStream_t)stream,
                         N, C, Hs, Ws, up_h, up_w, pad_t, pad_l, Hp, Wp, sh, sw, d_up, dx, accum);
    else
      hipLaunchKernelGGL(upsample_bwd4w_kernel<unsigned long long>, dim3(grid_for(total / 4, block_cap("UNET_UPB_BLOCKS", 8192))), dim3(256), 0,
                         (hipStream_t)stream, N, C, Hs, Ws, up_h, up_w, pad_t, pad_l, Hp, Wp, sh, sw, d_up, dx, accum);
    return check_launch("upsample_bwd");
  }
  if (C % 4 == 0) {
    hipLaunchKernelGGL(upsample_bwd4_kernel, dim3(grid_for(total / 4, block_cap("UNET_UPB_BLOCKS", 8192))), dim3(256), 0, (hipStream_t)stream, N, C, Hs,
                       Ws, up_h, up_w, pad_t, pad_l, Hp, Wp, sh, sw, d_up, dx, accum);
    return check_launch("upsample_bwd");
  }
  hipLaunchKernelGGL(upsample_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, Hs, Ws,
                     up_h, up_w, pad_t, pad_l, Hp, Wp, sh, sw, d_up, dx, accum);
  return check_launch("upsample_bwd");
}

int unet_resize_nchw(long long NC, int Hi, int Wi, int Ho, int Wo, float sh, float sw, const float* x, float* y,
                     void* stream) {
  hipLaunchKernelGGL(resize_nchw_kernel, dim3(grid_for(NC * Ho * (long long)Wo)), dim3(256), 0, (hipStream_t)stream,
                     NC, Hi, Wi, Ho, Wo, sh, sw, x, y);
  return check_launch("resize_nchw");
}

int unet_resize_nchw_bwd(long long NC, int Hi, int Wi, int Ho, int Wo, float sh, float sw, const float* dy, float* dx,
                         int accum, void* stream) {
  hipLaunchKernelGGL(resize_nchw_bwd_kernel, dim3(grid_for(NC * Hi * (long long)Wi)), dim3(256), 0,
                     (hipStream_t)stream, NC, Hi, Wi, Ho, Wo, sh, sw, dy, dx, accum);
  return check_launch("resize_nchw_bwd");
}

int unet_outconv_rows(long long P) { return oc_rows(P); }

int unet_outconv_fwd(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                     const float* shift, int relu, const float* w, const float* b, float* logits, void* stream) {
  if (K > OC_MAXK || K < 1) { set_error("unet_outconv_fwd: n_classes > 8 unsupported"); return UNET_ERR_UNSUPPORTED; }
  const long long P = N * H * (long long)W;
  const int G = (C % 8 == 0 && C / 8 <= 64 && ((C / 8) & (C / 8 - 1)) == 0) ? C / 8 : 0;
  if (G && K == 2) {
    long long blocks = (P * G + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (dtype == UNET_F16)
      hipLaunchKernelGGL((outconv_fwd_vec_kernel<f16, 2>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, P,
                         H * W, C, G, (const f16*)y, scale, shift, relu, w, b, logits);
    else if (dtype == UNET_BF16)
      hipLaunchKernelGGL((outconv_fwd_vec_kernel<bf16, 2>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, P,
                         H * W, C, G, (const bf16*)y, scale, shift, relu, w, b, logits);
    else
      hipLaunchKernelGGL((outconv_fwd_vec_kernel<float, 2>), dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, P,
                         H * W, C, G, (const float*)y, scale, shift, relu, w, b, logits);
    return check_launch("outconv_fwd");
  }
  const size_t shm = (size_t)(K * C + 2 * C) * sizeof(float);
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(outconv_fwd_kernel<f16>, dim3(grid_for(P)), dim3(256), shm, (hipStream_t)stream, P, H * W, C, K,
                       (const f16*)y, scale, shift, relu, w, b, logits);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(outconv_fwd_kernel<bf16>, dim3(grid_for(P)), dim3(256), shm, (hipStream_t)stream, P, H * W, C, K,
                       (const bf16*)y, scale, shift, relu, w, b, logits);
  else
    hipLaunchKernelGGL(outconv_fwd_kernel<float>, dim3(grid_for(P)), dim3(256), shm, (hipStream_t)stream, P, H * W, C,
                       K, (const float*)y, scale, shift, relu, w, b, logits);
  return check_launch("outconv_fwd");
}

int unet_outconv_bwd(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                     const float* shift, int relu, const float* w, const float* dl, float* da, int accum, float* partial,
                     void* stream) {
  if (K > OC_MAXK || K < 1 || C < K) { set_error("unet_outconv_bwd: need 1 <= n_classes <= min(8, C)"); return UNET_ERR_UNSUPPORTED; }
  const long long P = N * H * (long long)W;
  const int cl = chan_lanes_m(C), rows = oc_rows(P);
  const int G = (C % 8 == 0 && C / 8 <= 256 && ((C / 8) & (C / 8 - 1)) == 0) ? C / 8 : 0;
  if (dtype != UNET_F32 && G && K == 2) {
    if (dtype == UNET_F16)
      hipLaunchKernelGGL((outconv_bwd_vec_kernel<f16, 2>), dim3(rows), dim3(256), 0, (hipStream_t)stream, P, H * W, C, G,
                         (const f16*)y, scale, shift, relu, w, dl, da, accum, partial);
    else
      hipLaunchKernelGGL((outconv_bwd_vec_kernel<bf16, 2>), dim3(rows), dim3(256), 0, (hipStream_t)stream, P, H * W, C, G,
                         (const bf16*)y, scale, shift, relu, w, dl, da, accum, partial);
    return check_launch("outconv_bwd");
  }
  dim3 grid(cdiv(C, cl), rows);
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(outconv_bwd_kernel<f16>, grid, dim3(256), 0, (hipStream_t)stream, P, H * W, C, cl, K,
                       (const f16*)y, scale, shift, relu, w, dl, da, accum, partial, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(outconv_bwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, P, H * W, C, cl, K,
                       (const bf16*)y, scale, shift, relu, w, dl, da, accum, partial, rows);
  else
    hipLaunchKernelGGL(outconv_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, P, H * W, C, cl, K,
                       (const float*)y, scale, shift, relu, w, dl, da, accum, partial, rows);
  return check_launch("outconv_bwd");
}

int unet_outconv_bwd_bn(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                        const float* shift, int relu, const float* w, const float* dl, const float* mean,
                        const float* invstd, float* partial, float* bn_partial, void* stream) {
  const long long P = N * H * (long long)W;
  const int G = C / 8;
  if (K != 2 || C % 8 || G > 256 || (G & (G - 1)) || !scale || !shift || !mean || !invstd || P >= (1LL << 31)) {
    set_error("unet_outconv_bwd_bn: needs n_classes == 2, C % 8 == 0, C/8 a power of two <= 256, a BN activation");
    return UNET_ERR_UNSUPPORTED;
  }
  const int rows = oc_rows(P);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL((outconv_bwd_bn_kernel<f16, 2>), dim3(rows), dim3(256), 0, st, P, H * W, C, G, (const f16*)y,
                       scale, shift, relu, w, dl, mean, invstd, partial, bn_partial, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((outconv_bwd_bn_kernel<bf16, 2>), dim3(rows), dim3(256), 0, st, P, H * W, C, G, (const bf16*)y,
                       scale, shift, relu, w, dl, mean, invstd, partial, bn_partial, rows);
  else
    hipLaunchKernelGGL((outconv_bwd_bn_kernel<float, 2>), dim3(rows), dim3(256), 0, st, P, H * W, C, G,
                       (const float*)y, scale, shift, relu, w, dl, mean, invstd, partial, bn_partial, rows);
  return check_launch("outconv_bwd_bn");
}

int unet_bn_bwd_apply_oc(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                         const float* shift, int relu, const float* w, const float* dl, const float* coef, void* dy,
                         void* stream) {
  const long long P = N * H * (long long)W;
  const int CV = C / 8;
  if (K != 2 || C % 8 || CV > 256 || (CV & (CV - 1)) || P >= (1LL << 31)) {
    set_error("unet_bn_bwd_apply_oc: needs n_classes == 2, C % 8 == 0, C/8 a power of two <= 256");
    return UNET_ERR_UNSUPPORTED;
  }
  long long b = (P * CV + 255) / 256;
  if (b > 8192) b = 8192;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_apply_oc_kernel<f16, 2>), dim3((int)b), dim3(256), 0, st, P, H * W, C, (const f16*)y,
                       scale, shift, relu, w, dl, coef, (f16*)dy);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_oc_kernel<bf16, 2>), dim3((int)b), dim3(256), 0, st, P, H * W, C, (const bf16*)y,
                       scale, shift, relu, w, dl, coef, (bf16*)dy);
  else
    hipLaunchKernelGGL((bn_bwd_apply_oc_kernel<float, 2>), dim3((int)b), dim3(256), 0, st, P, H * W, C,
                       (const float*)y, scale, shift, relu, w, dl, coef, (float*)dy);
  return check_launch("bn_bwd_apply_oc");
}

int unet_outconv_bwd_finalize(const float* partial, int rows, int C, int K, float* dw, float* db, int accum,
                              void* stream) {
  const int total = K * C + K;
  hipLaunchKernelGGL(outconv_bwd_finalize_kernel, dim3(total), dim3(256), 0, (hipStream_t)stream, partial, rows, C, K,
                     dw, db, accum);
  return check_launch("outconv_bwd_finalize");
}

int unet_nchw_to_nhwc(int dtype, long long N, int C, int H, int W, const float* x, void* y, void* stream) {
  const long long total = N * C * (long long)H * W;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H, W,
                       x, (f16*)y);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H, W,
                       x, (bf16*)y);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H,
                       W, x, (float*)y);
  return check_launch("nchw_to_nhwc");
}

int unet_nhwc_to_nchw(int dtype, long long N, int C, int H, int W, const void* x, const float* scale,
                      const float* shift, int relu, float* y, void* stream) {
  const long long total = N * C * (long long)H * W;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H, W,
                       (const f16*)x, scale, shift, relu, y);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H, W,
                       (const bf16*)x, scale, shift, relu, y);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H,
                       W, (const float*)x, scale, shift, relu, y);
  return check_launch("nhwc_to_nchw");
}

int unet_gated_to_nchw(int dtype, long long N, int C, int H, int W, const void* x, const float* scale,
                       const float* shift, int relu, const float* p, const float* psi_ab, float* y, void* stream) {
  const long long total = N * C * (long long)H * W;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(gated_to_nchw_kernel<f16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H,
                       W, (const f16*)x, scale, shift, relu, p, psi_ab, y);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(gated_to_nchw_kernel<bf16>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H,
                       W, (const bf16*)x, scale, shift, relu, p, psi_ab, y);
  else
    hipLaunchKernelGGL(gated_to_nchw_kernel<float>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, C, H,
                       W, (const float*)x, scale, shift, relu, p, psi_ab, y);
  return check_launch("gated_to_nchw");
}

int unet_convt_bwd_rows(long long P) { return oc_rows(P); }

int unet_convt_bwd_prep(int dtype, long long N, int h, int w, int Ct, int Hp, int Wp, int pad_t, int pad_l,
                        const float* d_up, void* dy_s2d, float* partial, void* stream) {
  if (N <= 0 || h <= 0 || w <= 0 || Ct <= 0 || Ct > 256 * CT_MAXCH || pad_t < 0 || pad_l < 0 ||
      pad_t + 2 * h > Hp || pad_l + 2 * w > Wp) {
    set_error("unet_convt_bwd_prep: bad geometry");
    return UNET_ERR_ARG;
  }
  const int rows = oc_rows(N * h * w);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(convt_bwd_prep_kernel<f16>, dim3(rows), dim3(256), 0, st, N, h, w, Ct, Hp, Wp, pad_t, pad_l,
                       d_up, (f16*)dy_s2d, partial, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(convt_bwd_prep_kernel<bf16>, dim3(rows), dim3(256), 0, st, N, h, w, Ct, Hp, Wp, pad_t, pad_l,
                       d_up, (bf16*)dy_s2d, partial, rows);
  else
    hipLaunchKernelGGL(convt_bwd_prep_kernel<float>, dim3(rows), dim3(256), 0, st, N, h, w, Ct, Hp, Wp, pad_t, pad_l,
                       d_up, (float*)dy_s2d, partial, rows);
  return check_launch("convt_bwd_prep");
}

int unet_materialize(int dtype, const unet_src* src, long long N, int H, int W, void* out, void* stream) {
  if (!src || !out || N <= 0 || H <= 0 || W <= 0 || src->C <= 0 || !src->data || src->kind == UNET_SRC_NCHW_F32) {
    set_error("unet_materialize: bad arguments");
    return UNET_ERR_ARG;
  }
  const int vec = dtype != UNET_F32 ? 8 : 4;
  const long long total = N * H * (long long)W * ((src->C + vec - 1) / vec);
  {
    // the tiled Up-block form: 16-bit, C/8 a power of two, both scales <= 1/2 (the span bound of its LDS tile);
    // UNET_MAT_TILE=0: the per-pixel form (A/B), read per call
    const char* e = getenv("UNET_MAT_TILE");
    const int cv8 = src->C / 8;
    if ((!e || atoi(e)) && dtype != UNET_F32 && src->kind == UNET_SRC_UP_ACT && src->C % 8 == 0 && (cv8 & (cv8 - 1)) == 0 &&
        src->scale && src->shift && src->sh <= 0.5f && src->sw <= 0.5f && src->sh >= 0.f && src->sw >= 0.f &&
        N * H <= (1LL << 30) && (double)N * H * W * src->C < 4294967296.0 &&
        (double)N * src->H * src->W * src->C < 4294967296.0) {
      const int ct = cv8 < MUP_CT ? cv8 : MUP_CT;
      const dim3 grid((unsigned)cdiv(W, MUP_TX), (unsigned)(N * cdiv(H, MUP_TJ)), (unsigned)(cv8 / ct));
      hipStream_t st = (hipStream_t)stream;
      if (dtype == UNET_BF16)
        hipLaunchKernelGGL(materialize_up_tile_kernel<bf16>, grid, dim3(256), 0, st, *src, H, W, (bf16*)out);
      else
        hipLaunchKernelGGL(materialize_up_tile_kernel<f16>, grid, dim3(256), 0, st, *src, H, W, (f16*)out);
      return check_launch("materialize up tile");
    }
  }
  long long b = (total + 255) / 256;
  const long long bcap = block_cap("UNET_MAT_BLOCKS", 4096);
  if (b > bcap) b = bcap;
  const int cv = src->C / vec;
  // 32-bit gather offsets in item_issue: the source must stay below 4 GiB
  const double bytes = (double)N * src->H * src->W * src->C * (dtype != UNET_F32 ? 2 : 4);
  if (src->C % vec == 0 && cv <= 256 && (cv & (cv - 1)) == 0 && bytes < 4294967296.0) {
    MatDesc md;
    md.nsrc = 1;
    md.src[0] = *src;
    md.src[1] = *src;
    md.Cin = src->C;
    const int raw = (src->kind == UNET_SRC_POOL_ACT || src->kind == UNET_SRC_UP_ACT) ? 4 : 1;
    hipStream_t st = (hipStream_t)stream;
    const bool i32 = total < (1LL << 31);
#define UNET_MAT_LAUNCH(TT)                                                                                        \
  do {                                                                                                           \
    if (raw == 4 && i32) hipLaunchKernelGGL((materialize_fast_kernel<TT, 4, unsigned>), dim3((int)b), dim3(256), 0, st, md, N, H, W, (TT*)out); \
    else if (raw == 4) hipLaunchKernelGGL((materialize_fast_kernel<TT, 4, unsigned long long>), dim3((int)b), dim3(256), 0, st, md, N, H, W, (TT*)out); \
    else if (i32) hipLaunchKernelGGL((materialize_fast_kernel<TT, 1, unsigned>), dim3((int)b), dim3(256), 0, st, md, N, H, W, (TT*)out); \
    else hipLaunchKernelGGL((materialize_fast_kernel<TT, 1, unsigned long long>), dim3((int)b), dim3(256), 0, st, md, N, H, W, (TT*)out); \
  } while (0)
    if (dtype == UNET_BF16) UNET_MAT_LAUNCH(bf16);
    else if (dtype == UNET_F16) UNET_MAT_LAUNCH(f16);
    else UNET_MAT_LAUNCH(float);
#undef UNET_MAT_LAUNCH
    return check_launch("materialize");
  }
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(materialize_kernel<f16>, dim3((int)b), dim3(256), 0, (hipStream_t)stream, *src, N, H, W,
                       (f16*)out);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(materialize_kernel<bf16>, dim3((int)b), dim3(256), 0, (hipStream_t)stream, *src, N, H, W,
                       (bf16*)out);
  else
    hipLaunchKernelGGL(materialize_kernel<float>, dim3((int)b), dim3(256), 0, (hipStream_t)stream, *src, N, H, W,
                       (float*)out);
  return check_launch("materialize");
}

int unet_materialize_pool(int dtype, const unet_src* src, long long N, int H, int W, void* out, uint8_t* code,
                          void* stream) {
  const int vec = dtype != UNET_F32 ? 8 : 4;
  const int cv = src ? src->C / vec : 0;
  if (!src || !out || !code || src->kind != UNET_SRC_POOL_ACT || !src->scale || !src->shift || src->C % vec ||
      cv > 256 || (cv & (cv - 1)) || src->H < 2 * H || src->W < 2 * W) {
    set_error("unet_materialize_pool: needs a POOL_ACT source with C/vec a power of two <= 256");
    return UNET_ERR_ARG;
  }
  const long long total = N * H * (long long)W * cv;
  long long b = (total + 255) / 256;
  if (b > 16384) b = 16384;
  hipStream_t st = (hipStream_t)stream;
  const bool i32 = total < (1LL << 31);
  if (dtype == UNET_F16 && i32)
    hipLaunchKernelGGL((materialize_pool_kernel<f16, unsigned>), dim3((int)b), dim3(256), 0, st, *src, N, H, W, (f16*)out, code);
  else if (dtype == UNET_F16)
    hipLaunchKernelGGL((materialize_pool_kernel<f16, unsigned long long>), dim3((int)b), dim3(256), 0, st, *src, N, H, W, (f16*)out, code);
  else if (dtype == UNET_BF16 && i32)
    hipLaunchKernelGGL((materialize_pool_kernel<bf16, unsigned>), dim3((int)b), dim3(256), 0, st, *src, N, H, W, (bf16*)out, code);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((materialize_pool_kernel<bf16, unsigned long long>), dim3((int)b), dim3(256), 0, st, *src, N, H, W, (bf16*)out, code);
  else if (i32)
    hipLaunchKernelGGL((materialize_pool_kernel<float, unsigned>), dim3((int)b), dim3(256), 0, st, *src, N, H, W, (float*)out, code);
  else
    hipLaunchKernelGGL((materialize_pool_kernel<float, unsigned long long>), dim3((int)b), dim3(256), 0, st, *src, N, H, W, (float*)out, code);
  return check_launch("materialize_pool");
}

int unet_fill_f32(float* x, long long n, float v, void* stream) {
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, n, v);
  return check_launch("fill");
}

}  // extern "C"
